#!/bin/bash
# Round 6 first GPU call: the whole GPU suite on the round-start code + ADVICE fixes, smoke(), the
# default bench line (N=1) and a 2-rank shared-GPU rehearsal carrying the new per-rank-BN /
# distinct_devices keys.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r06a.log
: > $L
echo "=== pytest -m gpu $(date +%T)" >> $L
timeout -k 10 1000 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
echo "=== smoke $(date +%T)" >> $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || exit 1
echo "=== bench N=1 $(date +%T)" >> $L
timeout -k 10 600 python bench.py >> $L 2>&1 || exit 1
echo "=== bench N=2 (shared GPU) $(date +%T)" >> $L
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 \
  --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
echo done >> $L
