#!/bin/bash
# Round 5: bf16-intermediates DARTS A/B on darts-gpu.yaml, its trajectory test,
# and the HyperBand + median-stop ResNet-18 experiment re-run on the fused ResNet step.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05q.log
: > $L
B="--config default --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for rep in 1 2; do
  echo "=== fp32 rep $rep $(date +%T)" >> $L
  timeout -k 10 300 python bench.py $B >> $L 2>&1 || exit 1
  echo "=== bf16 rep $rep $(date +%T)" >> $L
  timeout -k 10 300 python bench.py $B --dtype bf16 >> $L 2>&1 || exit 1
done
echo "=== bf16 trajectory test $(date +%T)" >> $L
timeout -k 10 320 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_darts_bf16.py >> $L 2>&1 || exit 1
echo "=== hyperband resnet18 $(date +%T)" >> $L
timeout -k 10 400 python scripts/experiments_r05.py --only hyperband-resnet18 >> $L 2>&1 || exit 1
echo done >> $L
echo "=== hessian stacking bound (B5) $(date +%T)" >> $L
B5="--steps 40 --warmup 5 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for rep in 1 2; do
  echo "--- default rep $rep" >> $L
  timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
  echo "--- sequential hessian passes rep $rep" >> $L
  KATIB_DARTS_HESS_CONCURRENT=0 timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
  echo "--- hessian passes skipped (bound) rep $rep" >> $L
  KATIB_DARTS_DEBUG_SKIP_HESSIAN_PASSES=1 timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
done
echo "=== grid barrier probe (flat vs hierarchical per-XCD) $(date +%T)" >> $L
timeout -k 10 120 scripts/grid_barrier_probe 200 >> $L 2>&1 || exit 1
timeout -k 10 120 scripts/grid_barrier_probe 50 >> $L 2>&1 || exit 1
echo done2 >> $L
