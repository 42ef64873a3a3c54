#!/bin/bash
# round 6: kernel trace + PMC passes of plan label on the config #3 shape at 5e7 rows
set -o pipefail
cd "$(dirname "$0")/../../.." || exit 1
WORKLOAD=config3_folders_5e7 tools/profile_ab.sh folders50m --workload folders --tuples 50000000 --heads 0,0 --steps 5 || exit 1
