#!/bin/bash
# Quick kernel iteration: GPU DARTS tests, B5 bench x2, B5 timeline.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04n.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
step darts-tests 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step b5 300 python bench.py --steps 40 --warmup 5 $Q || exit 1
step b5 300 python bench.py --steps 40 --warmup 5 $Q || exit 1
step default 300 python bench.py --config default --steps 10 --warmup 3 $Q || exit 1
bash scripts/gpu_r04.sh tl >> $L 2>&1 || exit 1
echo done >> $L
