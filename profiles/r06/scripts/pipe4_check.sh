#!/bin/bash
# round 6: pipelined calls over four streams: label/writes GPU tests, host enqueue cost, a
# kernel trace of the pipelined loop, the config #2 bench line (no CPU baseline)
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "label or writes" --timeout 120 --timeout-method thread > gpurun_out/t_pipe4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe_trace4 -o run \
  -- python3 tools/label_ab.py --heads 0,0 --steps 20 > gpurun_out/pipe_trace4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --parity sample > gpurun_out/bench_pipe4.log 2>&1 || exit 1
