#!/bin/bash
# gemm256 (256x256-tile 8-wave ping-pong GEMM): numerics vs fp32, then the GPT-2 GEMM table vs hipBLASLt.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06b.log
: > $L
echo "=== gemm256 tests $(date +%T)" >> $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -v --timeout 120 --timeout-method thread -m gpu -k "gemm256" >> $L 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread -m gpu -k "cross_entropy" >> $L 2>&1 || exit 1
echo "=== bench_gemm256 $(date +%T)" >> $L
timeout -k 10 400 python benchmarks/bench_gemm256.py --square >> $L 2>&1 || exit 1
echo done >> $L
