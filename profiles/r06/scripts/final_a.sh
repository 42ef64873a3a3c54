#!/bin/bash
# round 6 final (A): the whole GPU suite, smoke, the config #2 bench line, and the 64-word
# head A/B (by lines vs whole) on the config #3 shape
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
V=$PWD/keto_amd/variants/libketogpu_whole.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_lines2.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_whole2.log 2>&1 || exit 1
