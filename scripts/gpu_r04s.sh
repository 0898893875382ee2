#!/bin/bash
# A/B: depthwise-backward channel groups of 4 (KATIB_HIP_DWB_GROUP=4) vs 8, B5 and darts-gpu.yaml, 3 rounds.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04s.log
: > $L
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
for r in 1 2 3; do
  for e in KATIB_AB_NONE=1 KATIB_HIP_DWB_GROUP=4; do
    echo "=== b5 $e $(date +%T)" >> $L
    timeout -k 10 300 env $e python bench.py --steps 40 --warmup 5 $Q >> $L 2>&1 || exit 1
  done
done
for r in 1 2; do
  for e in KATIB_AB_NONE=1 KATIB_HIP_DWB_GROUP=4; do
    echo "=== default $e $(date +%T)" >> $L
    timeout -k 10 300 env $e python bench.py --config default --steps 10 --warmup 3 $Q >> $L 2>&1 || exit 1
  done
done
echo done >> $L
