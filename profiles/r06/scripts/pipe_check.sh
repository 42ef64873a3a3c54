#!/bin/bash
# round 6: pipelined calls without the drain: label GPU tests, host enqueue cost, a kernel
# trace of the pipelined loop, and the config #2 bench line (no CPU baseline)
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "label or writes" --timeout 120 --timeout-method thread > gpurun_out/t_pipe.log 2>&1 || exit 1
timeout -k 10 300 python tools/host_enqueue_probe.py > gpurun_out/host_enq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe_trace2 -o run \
  -- python3 tools/label_ab.py --heads 0,0 --steps 20 > gpurun_out/pipe_trace2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --parity sample > gpurun_out/bench_pipe2.log 2>&1 || exit 1
