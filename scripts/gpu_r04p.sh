#!/bin/bash
# Grouped validation forward: GPU DARTS tests, B5 bench with the default group (4) vs 1, full search.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04p.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
Q="--trials 0 --b1 0 --comparator-steps 0"
step darts-tests 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for r in 1 2; do
  step "b5 group4" 300 python bench.py --steps 40 --warmup 5 $Q --full-search 0 || exit 1
  step "b5 group1" 300 env KATIB_DARTS_EVAL_GROUP=1 python bench.py --steps 40 --warmup 5 $Q --full-search 0 || exit 1
  step "b5 group8" 300 env KATIB_DARTS_EVAL_GROUP=8 python bench.py --steps 40 --warmup 5 $Q --full-search 0 || exit 1
done
step "b5 full-search" 300 python bench.py --steps 40 --warmup 5 $Q --full-search 1 || exit 1
echo done >> $L
