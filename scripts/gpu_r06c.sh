#!/bin/bash
# Stacked finite-difference Hessian passes: numerics (stacked vs concurrent vs sequential, vs the torch
# oracle, SyncBN 2-rank, graph hygiene), then an interleaved B5 A/B of --hessian stacked / concurrent,
# then the gemm256 ablations.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06c.log
: > $L
echo "=== darts tests $(date +%T)" >> $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_darts.py -k "stacked or trajectory" -x -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
B5="--steps 40 --warmup 5 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0"
for rep in 1 2; do
  for h in stacked concurrent; do
    echo "--- hessian $h rep $rep" >> $L
    timeout -k 10 300 python bench.py $B5 --hessian $h > gpurun_out/b.json 2>>$L || exit 1
    python -c "import json; r=json.load(open('gpurun_out/b.json')); print(json.dumps({k: r[k] for k in ('ms_per_step','value','hessian_stack')}))" >> $L || exit 1
  done
done


echo done >> $L
