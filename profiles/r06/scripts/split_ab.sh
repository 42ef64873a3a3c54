#!/bin/bash
# round 6: split pipeline (first stages on one stream, dense passes on a high-priority side
# stream) against the two-stream rotation: the pipelined GPU tests, then the config #2 bench
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
mkdir -p gpurun_out/split
KETOGPU_PIPE_SPLIT=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/split/bench_split_prio.log 2>&1 || exit 1
KETOGPU_PIPE_SPLIT=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/split/bench_rotate2.log 2>&1 || exit 1
