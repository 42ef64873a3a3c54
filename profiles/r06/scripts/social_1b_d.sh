#!/bin/bash
# round 6 (after the dense-pass stage change): config #4 (power-law, 1.0e9 rows, 125M users, 10M groups) on plan label, one wait
# per call and pipelined, with the R2 checker and a cross-plan sample
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 1150 python -u tools/bench_scale.py --workload social --tuples 1000000000 --users 125000000 \
  --groups 10000000 --steps 10 --r2-sample 20000 > gpurun_out/scale_social_1b_r06d.log 2>&1 || exit 1
