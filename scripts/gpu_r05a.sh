#!/bin/bash
# Round 5, first GPU call: RCCL-in-graph capture test, the distributed GPU tests (SyncBN, xGMI),
# and a quick B5 bench on this box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r05a.log
: > $L
echo "=== pytest $(date +%T)" >> $L
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_rccl_capture.py tests/test_gpu_syncbn.py tests/test_gpu_xgmi.py >> $L 2>&1 || exit 1
echo "=== bench b5 $(date +%T)" >> $L
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --trials 0 --b1 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
echo done >> $L
