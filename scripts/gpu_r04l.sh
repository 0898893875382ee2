#!/bin/bash
# Confirmation after removing pw_fwd_px: DARTS GPU tests, B5 bench, and the 2-rank self-launched bench
# (both ranks on the box's one GPU: SyncBN + one-shot IPC all-reduce) that the multi-GPU driver run uses.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04l.log
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
step darts-tests 600 python -u -m pytest tests/test_gpu_darts.py tests/test_gpu_syncbn.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider || exit 1
step b5 300 python bench.py --steps 40 --warmup 5 $Q || exit 1
step b5-gpus2-shared 400 python bench.py --gpus 2 --steps 10 --warmup 3 $Q || exit 1
step b5 300 python bench.py --steps 40 --warmup 5 $Q || exit 1
echo done >> $L
