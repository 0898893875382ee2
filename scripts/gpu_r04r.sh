#!/bin/bash
# B5 step: launch-heuristic sweep through env knobs (no rebuild).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04r.log
: > $L
Q="--steps 40 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0"
for e in KATIB_AB_NONE=1 KATIB_HIP_MAX_BLOCKS=1024 KATIB_HIP_MAX_BLOCKS=4096 KATIB_HIP_DWB_GROUP=4 KATIB_HIP_DWB_MIN_WG=512 \
         KATIB_HIP_DWB_MIN_WG=2048 KATIB_HIP_PW_PX_V4=1 KATIB_HIP_VEC_MASK=1 KATIB_HIP_VEC_MASK=4 KATIB_AB_NONE=1; do
  echo "=== $e $(date +%T)" >> $L
  timeout -k 10 300 env $e python bench.py $Q >> $L 2>&1 || exit 1
done
echo done >> $L
