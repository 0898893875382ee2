#!/bin/bash
# DARTS numerics tests + B5 and default-config benches on one MI355X.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/darts_bench.log
: > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 300 python bench.py >> $L 2>&1 || exit $?
timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 >> $L 2>&1 || exit $?
echo done >> $L
