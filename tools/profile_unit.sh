#!/bin/bash
# rocprofv3 counters of the LDS unit kernel on config #2 (run through gpurun)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_unit
mkdir -p $OUT
B="bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $C -T --output-format csv --kernel-include-regex "unit_kernel" -d $OUT/pmc_$tag -o run -- python3 $B > $OUT/pmc_$tag.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$tag.log; exit 1; }
done
echo profile done
