#!/bin/bash
# Self-fold + fused edge backward: DARTS numerics tests, then B5 / default bench over the
# (KATIB_HIP_SELFFOLD, KATIB_HIP_EDGE_BWD) grid, then the B5 kernel timeline with both on.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03b.log
: > $L
echo "=== tests" >> $L
timeout -k 10 900 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for cfg in "1 1" "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  echo "=== SELFFOLD=$1 EDGE=$2 b5" >> $L
  KATIB_HIP_SELFFOLD=$1 KATIB_HIP_EDGE_BWD=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
for cfg in "1 1" "0 0"; do
  set -- $cfg
  echo "=== SELFFOLD=$1 EDGE=$2 default" >> $L
  KATIB_HIP_SELFFOLD=$1 KATIB_HIP_EDGE_BWD=$2 timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
bash scripts/gpu_prof_timeline.sh b5 || exit 1
echo done >> $L
