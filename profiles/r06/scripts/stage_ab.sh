#!/bin/bash
# round 6: the dense pass's LDS stage per request (kFullStage words: 256 = 16 KB per workgroup,
# 10 workgroups per CU) against 192 and 128 (more workgroups resident at once), config #2 bench
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
mkdir -p gpurun_out/stage
for v in 256 128 192; do
  L=keto_amd/libketogpu.so; [ $v != 256 ] && L=ab_build/libketogpu_fs$v.so
  KETOGPU_LIB=$PWD/$L timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/stage/bench_$v.log 2>&1 || exit 1
done
