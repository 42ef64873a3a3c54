#!/bin/bash
# round 3 close-out after the uniform edge count in the lite kernels: their GPU parity tests,
# then part B (PMC profile at the final kernel sources, bench, partitioned bench)
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_host_batches.py tests/test_tier.py -m gpu -q \
  --timeout 240 --timeout-method thread > gpurun_out/final/gpu_tests_lite.log 2>&1 \
  || { echo "GPU tests failed"; tail -30 gpurun_out/final/gpu_tests_lite.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests_lite.log
bash tools/r03_final_b.sh
