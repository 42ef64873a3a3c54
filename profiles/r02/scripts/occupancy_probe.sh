#!/bin/bash
# unit2_kernel time vs workgroups per CU (extra dynamic LDS shrinks residency)
cd "$(dirname "$0")/.." || exit 1
for pad in 0 2000 12000 25000 50000; do
  echo "pad $pad"
  KETOGPU_LDS_PAD=$pad timeout -k 10 200 python -u tools/tune_units.py v2 2>&1 | grep median || exit 1
done
