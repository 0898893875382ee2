#!/bin/bash
# DARTS B5 step time vs the per-launch workgroup cap (KATIB_HIP_MAX_BLOCKS)
set -o pipefail
mkdir -p gpurun_out
for mb in 1024 2048 4096 8192 16384; do
  KATIB_HIP_MAX_BLOCKS=$mb timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/mb_$mb.json 2> gpurun_out/mb_$mb.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/mb_$mb.json').read().strip().splitlines()[-1]); print($mb, d['ms_per_step'])"
done
