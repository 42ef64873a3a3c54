#!/bin/bash
# round 3: lite32 parity + A/B of the first-stage plans on the bench line (one box)
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_batches.py -m gpu -x -q -k "lite32" \
  --timeout 200 --timeout-method thread > gpurun_out/lite32_tests.log 2>&1 || { echo "lite32 tests failed"; tail -30 gpurun_out/lite32_tests.log; exit 1; }
tail -2 gpurun_out/lite32_tests.log
bash tools/ab.sh gpurun_out/ab_lite32 KETOGPU_UNITS=lite KETOGPU_UNITS=lite32 "KETOGPU_UNITS=lite KETOGPU_HOST_UNITS=4" || exit 1
