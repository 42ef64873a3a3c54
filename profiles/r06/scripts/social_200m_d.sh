#!/bin/bash
# round 6 (after the dense-pass stage change): config #4 shape at 2e8 rows, 50 steps, the
# pipelined rate over more calls than the 1e9-row run's 10
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 700 python -u tools/bench_scale.py --workload social --tuples 200000000 --steps 50 \
  --r2-sample 0 --sample 20000 > gpurun_out/scale_social_200m_d.log 2>&1 || exit 1
