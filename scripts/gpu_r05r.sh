#!/bin/bash
# Round 5: unrolled MLP replays (U steps per graph) + warm-daemon B1 trials/hour.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05r.log
: > $L
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_mlp_unroll.py tests/test_gpu_workloads.py -k "unroll or mlp or mnist" >> $L 2>&1 || exit 1
for rep in 1 2; do
  echo "=== b1 warm daemon rep $rep $(date +%T)" >> $L
  timeout -k 10 300 python bench_trials.py --experiment examples/hp-tuning/b1-random-mnist-mlp.yaml >> $L 2>&1 || exit 1
done
echo "=== b1 unroll 1 (old) $(date +%T)" >> $L
KATIB_MLP_UNROLL=1 timeout -k 10 300 python bench_trials.py --experiment examples/hp-tuning/b1-random-mnist-mlp.yaml >> $L 2>&1 || exit 1
echo "=== tpe warm workers $(date +%T)" >> $L
timeout -k 10 300 python bench_trials.py --trials 12 --parallel 1 >> $L 2>&1 || exit 1
echo done >> $L
