#!/bin/bash
# Two-tier exchange path with 8-byte replies and HBM-staged requests: GPU tier tests, the
# world-1 RCCL exchange bench (config #5 x0.01) and a kernel trace of the same command.
export TMPDIR=/tmp
mkdir -p gpurun_out/x8
timeout -k 10 400 python -u -m pytest tests/test_tier.py tests/test_partition.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/x8/gpu_tests_tier.log 2>&1 || { echo "tier tests failed"; tail -30 gpurun_out/x8/gpu_tests_tier.log; exit 1; }
tail -1 gpurun_out/x8/gpu_tests_tier.log
timeout -k 10 400 python3 -u bench.py --mode partitioned --scale 0.01 --tier-exchange --no-cpu-baseline --steps 10 \
    --warmup 3 > gpurun_out/x8/bench_tier_exchange.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/x8/bench_tier_exchange.log; exit 1; }
tail -1 gpurun_out/x8/bench_tier_exchange.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x8/prof -o run -- python3 -u bench.py \
    --mode partitioned --scale 0.01 --tier-exchange --no-cpu-baseline --steps 4 --warmup 2 > gpurun_out/x8/bench_t.log 2>&1 \
    || { echo "profile failed"; tail -30 gpurun_out/x8/bench_t.log; exit 1; }
echo done
