#!/bin/bash
# Counter passes over tools/label_probe.py on a saved snapshot (run through gpurun):
#   1. generate + save the workload once (--save), 2. rocprofv3 --kernel-trace --stats,
#   3. one rocprofv3 --pmc pass per counter group (each its own run, within the per-block
#   slot limits of MI355X_MICROARCH.md), 4. tools/pmc_traffic.py summary.
# usage: tools/profile_probe.sh <tag> [label_probe.py args, e.g. --workload social --tuples 2e8]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-probe}
shift
OUT=gpurun_out/prof_$TAG
SNAP=/tmp/probe_snap_$TAG
mkdir -p "$OUT"
KRX="label_kernel|label_host_kernel|label_rest_kernel|label_full_kernel|lite_kernel|unit2_kernel|bidi_kernel"
echo "[probe] generate + save"
timeout -k 10 600 python3 tools/label_probe.py --save "$SNAP" "$@" > "$OUT/save.log" 2>&1 || { tail -20 "$OUT/save.log"; exit 1; }
echo "[probe] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 tools/label_probe.py --load "$SNAP" --host > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
python3 tools/timeline.py "$OUT/trace" --calls 2 > "$OUT/timeline.txt" 2>&1 || true
python3 tools/timeline.py "$OUT/trace" --calls 2 --match "label_kernel<" > "$OUT/timeline_resident.txt" 2>&1 || true
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  tag=$(echo "$C" | cut -d' ' -f1)
  echo "[probe] pmc $C"
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv --kernel-include-regex "$KRX" \
    -d "$OUT/pmc_$tag" -o run -- python3 tools/label_probe.py --load "$SNAP" --host > "$OUT/pmc_$tag.log" 2>&1 \
    || { echo "pmc $C failed"; tail -5 "$OUT/pmc_$tag.log"; exit 1; }
done
python3 tools/pmc_traffic.py "$OUT" "$OUT/summary" --workload "${WORKLOAD:-config2_rbac}" || exit 1
echo "[probe] done"
