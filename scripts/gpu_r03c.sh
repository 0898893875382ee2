#!/bin/bash
# Sharded self-fold counters + edge_bwd band sweep: DARTS numerics with both paths forced on, then
# B5 bench variants.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03c.log
: > $L
echo "=== tests SELFFOLD=1 EDGE=1" >> $L
KATIB_HIP_SELFFOLD=1 KATIB_HIP_EDGE_BWD=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
b5() { echo "=== $*" >> $L; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1; }
b5 KATIB_HIP_SELFFOLD=0 KATIB_HIP_EDGE_BWD=0 || exit 1
b5 KATIB_HIP_SELFFOLD=1 KATIB_HIP_EDGE_BWD=0 || exit 1
b5 KATIB_HIP_SELFFOLD=0 KATIB_HIP_EDGE_BWD=1 || exit 1
b5 KATIB_HIP_SELFFOLD=0 KATIB_HIP_EDGE_BWD=1 KATIB_HIP_EDGE_LDS_KB=24 KATIB_HIP_EDGE_WG=2048 || exit 1
b5 KATIB_HIP_SELFFOLD=0 KATIB_HIP_EDGE_BWD=1 KATIB_HIP_EDGE_LDS_KB=32 KATIB_HIP_EDGE_WG=4096 || exit 1
b5 KATIB_HIP_SELFFOLD=0 KATIB_HIP_EDGE_BWD=1 KATIB_HIP_EDGE_LDS_KB=64 KATIB_HIP_EDGE_WG=512 || exit 1
b5 KATIB_HIP_SELFFOLD=0 KATIB_HIP_EDGE_BWD=0 || exit 1
b5 KATIB_HIP_SELFFOLD=1 KATIB_HIP_EDGE_BWD=0 || exit 1
echo done >> $L
