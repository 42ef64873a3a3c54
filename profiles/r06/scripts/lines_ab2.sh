#!/bin/bash
# round 6: label GPU tests, then 64-word heads by lines (both heads' first lines together,
# then the second lines the lists need) against whole heads, config #3 and #2 shapes
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
V=$PWD/keto_amd/variants/libketogpu_whole.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "label" --timeout 120 --timeout-method thread > gpurun_out/t_label8.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_lines2.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_whole2.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --heads 0,0 32,64 > gpurun_out/ab_r_lines2.log 2>&1 || exit 1
