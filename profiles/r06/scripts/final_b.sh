#!/bin/bash
# round 6 final (B): kernel trace + PMC passes of the config #2 bench (tools/profile.sh),
# its summary as profiles/r06/traffic.json, then the bench line reading it (same sources)
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
tools/profile.sh r06 || exit 1
cp gpurun_out/prof_r06/summary/traffic.json profiles/r06/traffic.json || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_r06.log 2>&1 || exit 1
