#!/bin/bash
# Rendezvous counts of the darts-gpu.yaml default config (2 ranks sharing the GPU), concurrent vs stacked
# Hessian passes, for the DP projection.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06g.log
: > $L
B="--config default --steps 4 --warmup 2 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 --per-rank-bn 0 --valid-batches 1"
for h in concurrent stacked; do
  echo "--- default config, 2 ranks, SyncBN, hessian $h" >> $L
  timeout -k 10 500 python bench.py --gpus 2 $B --hessian $h > gpurun_out/bd.json 2>>$L || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/bd.json').read().strip().splitlines()[-1]); print(json.dumps({k: r[k] for k in ('ms_per_step','rendezvous_per_step','rendezvous_in_graph','syncbn_path','hessian_stack')}))" >> $L || exit 1
done
echo done >> $L
