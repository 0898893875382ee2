#!/bin/bash
# Round 5: B1 module-path trial step with zero_grad(set_to_none=True) vs the fill + accumulate form
# (KATIB_MLP_SET_TO_NONE=0): MLP GPU tests, then train_seconds of B1-shaped trials (3 layers, bf16, batch 64,
# 3 epochs) per optimizer, interleaved, then the B1 experiment (12 cold trials, parallel 3) both ways.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05hh.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "mlp or mnist" >> $L 2>&1 || exit 1
for rep in 1 2; do
  for opt in sgd adam ftrl; do
    echo "--- set_to_none $opt rep $rep" >> $L
    timeout -k 10 120 python -m katib_amd.workloads.mnist_mlp --batch-size=64 --lr=0.05 --num-layers=3 --optimizer=$opt --epochs=3 2>&1 | grep -E "train_seconds|Validation" >> $L || exit 1
    echo "--- fill+add $opt rep $rep" >> $L
    KATIB_MLP_SET_TO_NONE=0 timeout -k 10 120 python -m katib_amd.workloads.mnist_mlp --batch-size=64 --lr=0.05 --num-layers=3 --optimizer=$opt --epochs=3 2>&1 | grep -E "train_seconds|Validation" >> $L || exit 1
  done
done
echo done >> $L
