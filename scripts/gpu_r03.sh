#!/bin/bash
# Round-3 check on one MI355X: GPU tests, smoke, bench (with trials/h + torch comparator),
# a rocprofv3 kernel profile of the bench. Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03.log
: > $L
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
SEL=${1:-all}
if [ "$SEL" = all ] || [ "$SEL" = tests ]; then
  step pytest-gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ "$SEL" = all ] || [ "$SEL" = bench ]; then
  step bench 600 python bench.py || exit 1
  step bench-default 600 python bench.py --config default --steps 10 --warmup 3 --trials 0 --comparator-steps 3 --full-search 0 || exit 1
fi
echo done >> $L
