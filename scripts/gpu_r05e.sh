#!/bin/bash
# Round 5: layout-native GEMM (gemm_lt: NN dgrad / TN wgrad via ds_read_b64_tr_b16, split-K):
# numerics tests, then the forward + backward GEMM table against hipBLASLt at 8192 and 16384 tokens.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r05e.log
: > $L
echo "=== pytest $(date +%T)" >> $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py >> $L 2>&1 || exit 1
echo "=== tile128 16384 $(date +%T)" >> $L
timeout -k 10 400 env KATIB_HIP_GEMM_TILE=128 python benchmarks/bench_gemm.py --backward-only --tokens 16384 >> $L 2>&1 || exit 1
echo "=== tile256 16384 $(date +%T)" >> $L
timeout -k 10 400 env KATIB_HIP_GEMM_TILE=256 python benchmarks/bench_gemm.py --backward-only --tokens 16384 >> $L 2>&1 || exit 1
echo done >> $L
