#!/bin/bash
# A/B of the unit2 cascade (persistent stages vs host-synchronized launches) on the config #4
# shape, in one box:  tools/u2_cascade_ab.sh [tuples]
export TMPDIR=/tmp
T=${1:-200000000}
for round in 1 2; do
  for v in device sync; do
    envset=""; [ "$v" = sync ] && envset="KETOGPU_U2_SYNC=1"
    env $envset timeout -k 10 280 python3 -u tools/bench_scale.py --workload social --tuples $T --r2-sample 0 \
      --sample 2000 > gpurun_out/u2cas_${v}_$round.log 2>&1 || { echo "$v failed"; exit 1; }
    echo "$v $round $(grep 'timed:' gpurun_out/u2cas_${v}_$round.log)"
  done
done
