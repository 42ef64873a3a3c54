#!/bin/bash
# round 6: label/pipelined GPU tests, the config #2 bench line, then a kernel-trace + PMC
# profile of plan label on the config #3 shape at 5e7 rows
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "label" --timeout 120 --timeout-method thread > gpurun_out/t_label6.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench3.log 2>&1 || exit 1
WORKLOAD=config3_folders_5e7 tools/profile_ab.sh folders50m --workload folders --tuples 50000000 --heads 0,0 --steps 5 || exit 1
