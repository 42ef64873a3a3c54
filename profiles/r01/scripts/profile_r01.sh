#!/bin/bash
# Profiles bench.py on the GPU box (run through gpurun).  Kernel trace + stats first,
# then one rocprofv3 --pmc pass per counter group on the traversal kernels.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01
mkdir -p $OUT
B="bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
  tag=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C -T --output-format csv --kernel-include-regex "expand_kernel|pull_kernel|reset_kernel|gather_kernel|seed_kernel" -d $OUT/pmc_$tag -o run -- python3 $B > $OUT/pmc_$tag.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$tag.log; exit 1; }
done
echo profile done
