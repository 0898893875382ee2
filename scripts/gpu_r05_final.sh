#!/bin/bash
# Round 5 final GPU round on the final code: the whole GPU suite, smoke(), the default bench line (N=1),
# and 2- / 4-rank rehearsals of bench.py --gpus N (all ranks sharing the one GPU through IPC).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05_final.log
: > $L
echo "=== pytest -m gpu $(date +%T)" >> $L
timeout -k 10 1000 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
echo "=== smoke $(date +%T)" >> $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || exit 1
echo "=== bench N=1 $(date +%T)" >> $L
timeout -k 10 600 python bench.py >> $L 2>&1 || exit 1
echo "=== bench N=2 (shared GPU) $(date +%T)" >> $L
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 \
  --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
echo "=== bench N=4 (shared GPU) $(date +%T)" >> $L
timeout -k 10 400 python bench.py --gpus 4 --steps 5 --warmup 2 --trials 0 --b1 0 --experiment 0 \
  --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
echo done >> $L
