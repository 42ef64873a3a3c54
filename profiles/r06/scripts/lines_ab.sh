#!/bin/bash
# round 6: label/pipelined GPU tests, then A/B of 64-word heads read by lines (the second
# line only when the list needs it) against whole heads, on the config #3 shape; the
# config #2 bench line
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
V=$PWD/keto_amd/variants/libketogpu_whole.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "label" --timeout 120 --timeout-method thread > gpurun_out/t_label6.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_lines.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_whole.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench3.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --heads 0,0 32,64 > gpurun_out/ab_r_lines.log 2>&1 || exit 1
