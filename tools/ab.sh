#!/bin/bash
# A/B of library builds or settings on the bench line (run through gpurun):
#   tools/ab.sh OUTDIR VARIANT...
# each variant is "base" (keto_amd/libketogpu.so), a name under keto_amd/variants/, or an
# environment setting VAR=VALUE for the base library (e.g. KETOGPU_PIPE_DMA=1).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=$1
shift
mkdir -p "$OUT"
for round in 1 2; do
  for v in "$@"; do
    lib=""
    envset=()
    case "$v" in
      base) ;;
      *=*) read -r -a envset <<< "$v" ;;
      *) lib="$PWD/keto_amd/variants/libketogpu_$v.so" ;;
    esac
    # AB_ARGS: extra bench.py arguments (e.g. "--mode partitioned --scale 0.01")
    env "${envset[@]}" KETOGPU_LIB="$lib" timeout -k 10 240 python3 bench.py --no-cpu-baseline --parity sample \
      --steps 10 --warmup 3 $AB_ARGS > "$OUT/${v}_$round.json" 2> "$OUT/${v}_$round.err" \
      || { echo "$v failed"; tail -5 "$OUT/${v}_$round.err"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$OUT/${v}_$round.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', $round, d['value'], d.get('hbm_resident_checks_per_s'), r['ms_per_launch'], r['frac'], d.get('parity',{}).get('mismatches'))"
  done
done
