#!/bin/bash
# round 3 close-out, part B: PMC profile of the bench (kernel trace + counter passes), the
# bench line with full parity and both CPU baselines, the partitioned line with parity
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 700 bash tools/profile.sh r03z > gpurun_out/final/profile.log 2>&1 \
  || { echo "profile failed"; tail -20 gpurun_out/final/profile.log; exit 1; }
tail -1 gpurun_out/final/profile.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/final/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log | cut -c1-300
timeout -k 10 400 python3 -u bench.py --mode partitioned > gpurun_out/final/bench_partitioned.log 2>&1 \
  || { echo "partitioned bench failed"; tail -20 gpurun_out/final/bench_partitioned.log; exit 1; }
tail -1 gpurun_out/final/bench_partitioned.log | cut -c1-300
