#!/bin/bash
# round 6: label GPU tests, then A/B of label_block8 without per-entry bounds predicates
# (padded rows) against the previous build, on the config #3 and #2 shapes
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
V=$PWD/keto_amd/variants/libketogpu_prev.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "label" --timeout 120 --timeout-method thread > gpurun_out/t_label7.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_pad.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_prev.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --heads 0,0 > gpurun_out/ab_r_pad.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --heads 0,0 > gpurun_out/ab_r_prev.log 2>&1 || exit 1
