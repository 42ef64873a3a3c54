#!/bin/bash
# round 6: the 64 negatives with the largest root closures of the
# config #4 shape at 2e8 rows, answered by plan label and by the R2 checker, then by the
# reference DFS under a per-request budget
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
timeout -k 10 560 python -u tools/hard_negatives.py pick gpurun_out/hard_200m.json --tuples 2e8 --users 20000000 \
  --groups 2000000 --candidates 20000 --keep 64 > gpurun_out/hard_200m_pick.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/hard_negatives.py oracle gpurun_out/hard_200m.json gpurun_out/hard_200m_oracle.json \
  --tuples 2e8 --users 20000000 --groups 2000000 --budget 60 --seconds 420 > gpurun_out/hard_200m_oracle.log 2>&1 || exit 1
