#!/bin/bash
# unit2 table / frontier sizes on the config #3 and #4 shapes (5M tuples), one process per library
cd "$(dirname "$0")/.." 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/u2ab
for wl in folders social; do
  for v in ${U2V:-base u2f256 u2h10 u2h10f256}; do
    lib=""; [ "$v" != base ] && lib="$PWD/keto_amd/variants/libketogpu_$v.so"
    echo "== $wl $v"
    KETOGPU_LIB="$lib" timeout -k 10 150 python3 tools/tune_units.py v2 --workload=$wl 2>&1 | grep -E "median|Error|error" || exit 1
  done
done
