#!/bin/bash
# round 6: dense-pass LDS stage, part 2: config #2 bench at 96 and 64 words, then the config #3
# folder shape at 1e8 rows (64-word heads, longer lists) at 256 / 128 / 96 (tools/label_ab.py)
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
mkdir -p gpurun_out/stage
for v in 96 64; do
  KETOGPU_LIB=$PWD/ab_build/libketogpu_fs$v.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/stage/bench_$v.log 2>&1 || exit 1
done
for v in 256 128 96; do
  L=keto_amd/libketogpu.so; [ $v != 256 ] && L=ab_build/libketogpu_fs$v.so
  KETOGPU_LIB=$PWD/$L timeout -k 10 400 python -u tools/label_ab.py --workload folders --tuples 100000000 --steps 20 > gpurun_out/stage/folders_$v.log 2>&1 || exit 1
done
