#!/bin/bash
# Round check on one MI355X: GPU tests, graft smoke, workloads, trials/hour bench, DARTS bench.
# Each GPU step has its own time limit; the script stops at the first crash/timeout (exit > 1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/round.log
: > $L
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name" >> $L
  return $rc
}
step pytest-gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?; [ $rc -gt 1 ] && exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step mnist-mlp 300 python -m katib_amd.workloads.mnist_mlp --epochs 3 || exit 1
step resnet18 600 python -m katib_amd.workloads.resnet_cifar --epochs 1 --max-steps 60 || exit 1
step gpt2-small 600 python -m katib_amd.workloads.gpt2_pbt --steps 30 --batch-size 16 || exit 1
step bench-trials 900 python bench_trials.py --trials 24 --parallel 8 --epochs 3 || exit 1
step bench-darts 600 python bench.py || exit 1
echo done >> $L
