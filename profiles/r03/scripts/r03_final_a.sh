#!/bin/bash
# round 3 close-out, part A: the whole GPU suite, smoke, and the undelivered-copy probes
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > gpurun_out/final/gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
for k in torch engine; do
  timeout -k 10 180 rocprofv3 --memory-copy-trace --kernel-trace -d gpurun_out/final/probe_$k -o run \
    -- python3 tools/copy_probe.py $k > gpurun_out/final/probe_$k.log 2>&1 || { echo "probe $k failed"; exit 1; }
  echo "probe $k: $(grep -c 'completion callbacks' gpurun_out/final/probe_$k.log) undelivered-callback warnings"
done
