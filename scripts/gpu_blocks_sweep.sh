#!/bin/bash
# Persistent-grid cap sweep (KATIB_HIP_MAX_BLOCKS) for the B5 and default DARTS benches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/blocks_sweep.jsonl
for cfg in b5 default; do
  for mb in 512 1024 2048 4096; do
    KATIB_HIP_MAX_BLOCKS=$mb timeout -k 10 240 python bench.py --config $cfg --steps 30 --warmup 5 > gpurun_out/bs.log 2>&1 || exit $?
    grep '^{' gpurun_out/bs.log | sed "s/^{/{\"max_blocks\": $mb, /" >> gpurun_out/blocks_sweep.jsonl
  done
done
