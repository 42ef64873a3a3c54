#!/bin/bash
# A/B of library variants (keto_amd/variants/libketogpu_<v>.so, or "base") on the config #4
# shape in one box:  tools/u2_variant_ab.sh TUPLES VARIANT...
export TMPDIR=/tmp
T=$1; shift
for round in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != base ] && lib="$PWD/keto_amd/variants/libketogpu_$v.so"
    KETOGPU_LIB="$lib" timeout -k 10 280 python3 -u tools/bench_scale.py --workload social --tuples $T --r2-sample 0 \
      --sample 2000 > gpurun_out/u2v_${v}_$round.log 2>&1 || { echo "$v failed"; exit 1; }
    echo "$v $round $(grep 'timed:' gpurun_out/u2v_${v}_$round.log)"
  done
done
