#!/bin/bash
# Round 5: combine_fwd running-stat updates spread over the grid: DARTS numerics + B5 / default timing.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05z.log
: > $L
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_darts.py tests/test_darts_parity.py >> $L 2>&1 || exit 1
B5="--steps 40 --warmup 5 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
echo done >> $L
