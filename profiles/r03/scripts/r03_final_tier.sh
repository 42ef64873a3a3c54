export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -m pytest tests/test_tier.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final/gpu_tests_tier.log 2>&1 || { echo "tier tests failed"; tail -30 gpurun_out/final/gpu_tests_tier.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests_tier.log
