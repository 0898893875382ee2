#!/bin/bash
# DARTS mixed-variant launches: numerics tests, then B5 / default bench with KATIB_HIP_MULTI=1 vs 0,
# then the B5 kernel timeline with the multi launches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/multi_ab.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for m in 1 0 1 0; do
  echo "=== MULTI=$m b5" >> $L
  KATIB_HIP_MULTI=$m timeout -k 10 300 python bench.py --steps 30 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
for m in 1 0; do
  echo "=== MULTI=$m default" >> $L
  KATIB_HIP_MULTI=$m timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
done
bash scripts/gpu_prof_timeline.sh b5 || exit 1
echo done >> $L
