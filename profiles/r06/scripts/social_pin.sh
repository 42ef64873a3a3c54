#!/bin/bash
# round 6: plan label on the config #4 shape at 2e8 rows against the
# reference DFS (oracle/keto_oracle.c, per-request budget) and the R2 checker
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 1150 python -u tools/bench_scale.py --workload social --tuples 200000000 --steps 10 \
  --oracle-sample 400 --oracle-seconds 420 --oracle-request-seconds 20 --r2-sample 20000 \
  > gpurun_out/scale_social_200m.log 2>&1 || exit 1
