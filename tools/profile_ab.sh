#!/bin/bash
# Profile plan label's kernels on any workload (run through gpurun): tools/label_ab.py under
#   1. rocprofv3 --kernel-trace --stats (per-kernel durations),
#   2. one rocprofv3 --pmc pass per counter group (each its own run, within the per-block
#      slot limits of MI355X_MICROARCH.md),
#   3. tools/pmc_traffic.py -> gpurun_out/prof_<tag>/summary/{kernel_stats.csv,traffic.json}.
# usage: tools/profile_ab.sh <tag> <label_ab.py args...>
#   e.g. tools/profile_ab.sh folders50m --workload folders --tuples 50000000 --heads 0,0 --steps 5
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
B="tools/label_ab.py $*"
KRX="label_kernel|label_host_kernel|label_full_kernel"
echo "[profile] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 $B > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  tag=$(echo "$C" | cut -d' ' -f1)
  echo "[profile] pmc $C"
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv --kernel-include-regex "$KRX" \
    -d "$OUT/pmc_$tag" -o run -- python3 $B > "$OUT/pmc_$tag.log" 2>&1 \
    || { echo "pmc $C failed"; tail -5 "$OUT/pmc_$tag.log"; exit 1; }
done
python3 tools/pmc_traffic.py "$OUT" "$OUT/summary" --workload "${WORKLOAD:-label_ab}" || exit 1
echo "[profile] done"
