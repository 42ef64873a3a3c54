#!/bin/bash
# round 6: kernel trace of config #2 label_ab (one wait per call, then pipelined over two
# streams) to see how the dense pass overlaps the next call's first stage
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe_trace -o run \
  -- python3 tools/label_ab.py --heads 0,0 --steps 20 > gpurun_out/pipe_trace.log 2>&1 || exit 1
