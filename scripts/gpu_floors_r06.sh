#!/bin/bash
# Per-rank step floors (dp1 at global batch 128 / 64 / 32 / 16) for the DP projection, B5 and darts-gpu.yaml default.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=gpurun_out/floors_r06.log
: > $L
for cfg in b5 default; do
  for b in 128 64 32 16; do
    S="--steps 20 --warmup 5"; [ $cfg = default ] && S="--steps 8 --warmup 3"
    timeout -k 10 300 python bench.py --config $cfg --batch $b $S --trials 0 --b1 0 --experiment 0 --comparator-steps 0 \
      --full-search 0 --floor 0 --valid-batches 1 > gpurun_out/fl.json 2>/dev/null || exit 1
    echo "$cfg $b $(python -c "import json; print(json.loads(open('gpurun_out/fl.json').read().strip().splitlines()[-1])['ms_per_step'])")" >> $L
  done
done
