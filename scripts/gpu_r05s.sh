#!/bin/bash
# Round 5 mid-point: the whole GPU suite, smoke(), and the default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05s.log
: > $L
echo "=== attention bench $(date +%T)" >> $L
timeout -k 10 120 python benchmarks/bench_attn.py >> $L 2>&1 || exit 1
echo "=== pytest -m gpu $(date +%T)" >> $L
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
echo "=== smoke $(date +%T)" >> $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || exit 1
echo "=== bench $(date +%T)" >> $L
timeout -k 10 600 python bench.py >> $L 2>&1 || exit 1
echo done >> $L
