#!/bin/bash
# Round 5: cold-trial phase breakdown and trials/hour - the B1-shaped experiment (12 cold batch/v1 Job
# trials, parallel 3) with the fork server (default) and with fork + exec (KATIB_AMD_ZYGOTE=0), and the
# warm-worker TPE experiment at 12 trials.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r05g.log
: > $L
for r in 1 2 3; do
  echo "=== b1 zygote $(date +%T)" >> $L
  timeout -k 10 300 python bench_trials.py --experiment examples/hp-tuning/b1-random-mnist-mlp.yaml >> $L 2>&1 || exit 1
done
echo "=== tpe warm 12 $(date +%T)" >> $L
timeout -k 10 300 python bench_trials.py --trials 12 --parallel 1 --epochs 3 >> $L 2>&1 || exit 1
echo done >> $L
