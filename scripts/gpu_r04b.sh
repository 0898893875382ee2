#!/bin/bash
# Round 4: launch-cost probe, SyncBN / xGMI GPU tests, self-launched 2-rank bench on one GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04b.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}
step probe 240 python scripts/launch_cost_probe.py || exit 1
step syncbn-tests 600 python -u -m pytest tests/test_gpu_syncbn.py tests/test_gpu_xgmi.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider || exit 1
step bench-dp2 400 python bench.py --gpus 2 --steps 20 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 || exit 1
echo done >> $L
