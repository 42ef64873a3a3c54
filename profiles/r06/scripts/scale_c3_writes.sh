#!/bin/bash
# round 6: config #3 at 5e8 rows (pipelined over two streams) with the oracle, R2 and expand
# pins; then the write path at config #2 with a background relabel crossing its threshold
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --parity sample > gpurun_out/bench_probe.log 2>&1 || exit 1
timeout -k 10 800 python -u tools/bench_scale.py --workload folders --tuples 500000000 --steps 20 \
  --oracle-sample 20000 --r2-sample 20000 > gpurun_out/scale_folders_500m_r06.log 2>&1 || exit 1
timeout -k 10 360 python -u tools/bench_writes.py --sizes 1,10,100,1000 --relabel-permille 2 \
  > gpurun_out/writes_config2_bg.log 2>&1 || exit 1
