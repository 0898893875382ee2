#!/bin/bash
# SyncBN with concurrent Hessian branches on per-branch workspaces: streamed 2-rank worker runs, the
# SyncBN GPU test, and the self-launched 2-rank bench (A/B KATIB_DARTS_HESS_CONCURRENT=0).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04m.log
: > $L
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "[rc=$rc] $name $(date +%T)" >> $L
  return $rc
}

step syncbn-diag 200 env CASES="1 1" bash scripts/gpu_syncbn_diag.sh || exit 1
grep -q "SYNCBN_RESULT" gpurun_out/syncbn_diag.log || { echo "diag: no result" >> $L; exit 1; }
step syncbn-test 450 python -u -m pytest tests/test_gpu_syncbn.py -v --timeout 420 --timeout-method thread -p no:cacheprovider || exit 1
Q="--trials 0 --b1 0 --comparator-steps 0 --full-search 0"
step gpus2 400 python bench.py --gpus 2 --steps 10 --warmup 3 $Q || exit 1
step gpus2-seq-hessian 400 env KATIB_DARTS_HESS_CONCURRENT=0 python bench.py --gpus 2 --steps 10 --warmup 3 $Q || exit 1
echo done >> $L
