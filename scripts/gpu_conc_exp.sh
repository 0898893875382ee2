#!/bin/bash
# DARTS: numerics with concurrent launch groups, then B5 bench with / without them.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/conc_exp.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for c in 1 0 1 0; do KATIB_HIP_CONCURRENT=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 | sed "s/^/CONC=$c /" >> $L 2>&1 || exit $?; done
KATIB_HIP_CONCURRENT=1 timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 | sed "s/^/DEFAULT CONC=1 /" >> $L 2>&1 || exit $?
echo done >> $L
