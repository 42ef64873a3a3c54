#!/bin/bash
# traces of host-to-host calls under several host-batch settings (plan label)
set -o pipefail
cd /root/repo || exit 1
export TMPDIR=/tmp
for v in "direct" "dma KETOGPU_PIPE_DMA=1" "dma128k KETOGPU_PIPE_DMA=1 KETOGPU_PIPE_CHUNK=131072"; do
  name=${v%% *}; envs=${v#* }; [ "$name" = "$v" ] && envs=""
  env KETOGPU_UNITS=label $envs timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/tr_$name -o run -- python3 bench.py --no-cpu-baseline --parity sample --steps 5 --warmup 2 \
    > gpurun_out/tr_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/tr_$name.log; exit 1; }
  python3 tools/timeline.py gpurun_out/tr_$name --calls 2 > gpurun_out/tl_$name.txt 2>&1 || true
done
