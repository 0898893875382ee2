#!/bin/bash
# Round 5: LDS quad reads in the 4-pixel plane paths. DARTS GPU tests, then A/B of the vector
# mask (5: C=4 only, the old default; 15: C=4 and C=8) on B5 and darts-gpu.yaml.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r05b.log
: > $L
echo "=== pytest $(date +%T)" >> $L
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_darts.py >> $L 2>&1 || exit 1
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
for r in 1 2; do
  for m in 5 15 31; do
    echo "=== b5 mask=$m $(date +%T)" >> $L
    timeout -k 10 300 env KATIB_HIP_VEC_MASK=$m python bench.py --steps 40 --warmup 5 $Q >> $L 2>&1 || exit 1
  done
done
for m in 5 15; do
  echo "=== default mask=$m $(date +%T)" >> $L
  timeout -k 10 300 env KATIB_HIP_VEC_MASK=$m python bench.py --config default --steps 10 --warmup 3 $Q >> $L 2>&1 || exit 1
done
echo done >> $L
