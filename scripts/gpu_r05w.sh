#!/bin/bash
# Round 5: synthetic datasets drawn on the device (ResNet / MLP trial start-up), workload tests,
# B1 trials/hour and the HyperBand ResNet-18 experiment.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05w.log
: > $L
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_workloads.py \
  tests/test_gpu_mlp.py tests/test_gpu_mlp_unroll.py tests/test_gpu_resnet_step.py >> $L 2>&1 || exit 1
echo "=== resnet run $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.resnet_cifar --epochs 2 >> $L 2>&1 || exit 1
for rep in 1 2; do
  echo "=== b1 rep $rep $(date +%T)" >> $L
  timeout -k 10 300 python bench_trials.py --experiment examples/hp-tuning/b1-random-mnist-mlp.yaml >> $L 2>&1 || exit 1
done
echo "=== hyperband resnet18 $(date +%T)" >> $L
timeout -k 10 400 python scripts/experiments_r05.py --only hyperband-resnet18 >> $L 2>&1 || exit 1
echo done >> $L
