#!/bin/bash
# Round 5: DARTS validation grouping A/B (KATIB_DARTS_EVAL_GROUP) and the PBT GPT-2 / DARTS B5 experiments
# re-run on the final kernels.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05aa.log
: > $L
B5="--steps 40 --warmup 5 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for g in 8 16 32; do
  echo "--- eval group $g" >> $L
  KATIB_DARTS_EVAL_GROUP=$g timeout -k 10 300 python bench.py $B5 >> $L 2>&1 || exit 1
done
echo "=== experiments $(date +%T)" >> $L
timeout -k 10 500 python scripts/experiments_r05.py --only pbt-gpt2 --pbt-trials 32 >> $L 2>&1 || exit 1
timeout -k 10 300 python scripts/experiments_r05.py --only darts-b5 --slots 1 >> $L 2>&1 || exit 1
echo done >> $L
