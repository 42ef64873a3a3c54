#!/bin/bash
# Profile bench.py (config #2) on the GPU box (run through gpurun):
#   1. rocprofv3 --kernel-trace --stats over the bench (per-kernel durations),
#   2. one rocprofv3 --pmc pass per counter group on the traversal kernels (each pass
#      its own run, within the per-block slot limits of MI355X_MICROARCH.md),
#   3. tools/pmc_traffic.py -> profiles/<tag>/{kernel_stats.csv,traffic.json}.
# usage: tools/profile.sh <tag> [extra bench.py args]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r01}
shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
B="bench.py --no-cpu-baseline --parity sample --steps 5 --warmup 2 $*"
KRX="bidi_kernel|bidi_host_kernel|lite_kernel|lite_host_kernel|label_kernel|label_host_kernel|label_rest_kernel|label_full_kernel|unit2_kernel|expand_kernel|pull_kernel|part_|tier_"
echo "[profile] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 $B > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
python3 tools/timeline.py "$OUT/trace" --calls 2 > "$OUT/timeline.txt" 2>&1 || true
grep '^{"metric"' "$OUT/trace.log" > "$OUT/bench_line.json"
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  tag=$(echo "$C" | cut -d' ' -f1)
  echo "[profile] pmc $C"
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv --kernel-include-regex "$KRX" \
    -d "$OUT/pmc_$tag" -o run -- python3 $B > "$OUT/pmc_$tag.log" 2>&1 \
    || { echo "pmc $C failed"; tail -5 "$OUT/pmc_$tag.log"; exit 1; }
done
python3 tools/pmc_traffic.py "$OUT" "$OUT/summary" --workload "${WORKLOAD:-config2_rbac}" || exit 1
echo "[profile] done"
