#!/bin/bash
# lazy spill cascade: GPU parity tests (incl. the lazy second pass), then the bench with the
# cascade launched up front (KETOGPU_CASCADE_EAGER=1) and lazily, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out/lazy
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_batches.py -m gpu -q \
  --timeout 240 --timeout-method thread > gpurun_out/lazy/gpu_tests.log 2>&1 \
  || { echo "GPU tests failed"; tail -30 gpurun_out/lazy/gpu_tests.log; exit 1; }
tail -1 gpurun_out/lazy/gpu_tests.log
for k in 1 2; do
  for mode in eager lazy; do
    if [ $mode = eager ]; then export KETOGPU_CASCADE_EAGER=1; else unset KETOGPU_CASCADE_EAGER; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --parity sample --steps 20 --warmup 3 \
      > gpurun_out/lazy/bench_${mode}_$k.log 2>&1 || { echo "bench $mode failed"; tail -20 gpurun_out/lazy/bench_${mode}_$k.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/lazy/bench_${mode}_$k.log') if l.startswith('{\"metric\"')][-1])
print('$mode', $k, d['value'], d['ms_per_step'], d['hbm_resident_checks_per_s'], d['roofline']['ms_per_launch'])"
  done
done
