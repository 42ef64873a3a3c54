#!/bin/bash
# round 6: GPU label tests, then A/B of the LDS lookups (block8 vs splitter rows) on the
# config #3 and config #2 shapes
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
V=$PWD/keto_amd/variants/libketogpu_split.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "label or writes" --timeout 120 --timeout-method thread > gpurun_out/t_label5.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_def.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --workload folders --tuples 50000000 --heads 0,0 > gpurun_out/ab_f_split.log 2>&1 || exit 1
timeout -k 10 300 python tools/label_ab.py --heads 0,0 > gpurun_out/ab_r_def.log 2>&1 || exit 1
KETOGPU_LIB=$V timeout -k 10 300 python tools/label_ab.py --heads 0,0 > gpurun_out/ab_r_split.log 2>&1 || exit 1
