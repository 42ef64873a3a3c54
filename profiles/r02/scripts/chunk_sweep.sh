#!/bin/bash
# host-to-host chunk size sweep of bench.py (run through gpurun): tools/chunk_sweep.sh OUTDIR SIZE...
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=$1
shift
mkdir -p "$OUT"
for c in "$@"; do
  KETOGPU_PIPE_CHUNK=$c timeout -k 10 240 python3 bench.py --no-cpu-baseline --parity sample --steps 10 --warmup 3 \
    > "$OUT/chunk_$c.json" 2> "$OUT/chunk_$c.err" || { echo "$c failed"; tail -5 "$OUT/chunk_$c.err"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/chunk_$c.json').read().strip().splitlines()[-1])
print('chunk $c', d['value'], d.get('median_call_checks_per_s'), d['ms_per_step'])"
done
