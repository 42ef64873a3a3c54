export TMPDIR=/tmp
for v in base u2a u2b u2c; do
  lib=""; [ "$v" != base ] && lib="$PWD/keto_amd/variants/libketogpu_$v.so"
  KETOGPU_LIB="$lib" timeout -k 10 280 python3 -u tools/bench_scale.py --workload social --tuples 200000000 --r2-sample 0 --sample 2000 > gpurun_out/u2ab_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  grep "timed:" gpurun_out/u2ab_$v.log
done
