#!/bin/bash
# round 6 final (D), at the final sources: the whole GPU suite and smoke, kernel trace + PMC
# passes of the config #2 bench (tools/profile.sh) as profiles/r06/traffic.json, then the
# bench line reading it
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_final_d.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final_d.log 2>&1 || exit 1
tools/profile.sh r06d || exit 1
cp gpurun_out/prof_r06d/summary/traffic.json profiles/r06/traffic.json || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_final_d.log 2>&1 || exit 1
