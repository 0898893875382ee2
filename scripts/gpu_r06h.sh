#!/bin/bash
# Hoisted first-element loads in combine_fwd / combine_bwd_reduce / pool_bwd: DARTS GPU tests, then the
# B5 bench (N=1) for the step time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$(pwd)
L=gpurun_out/r06h.log
: > $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_darts.py tests/test_gpu_darts_bf16.py >> $L 2>&1 || exit 1
B="--steps 20 --warmup 10 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 --floor 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/bh.json 2>>$L || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/bh.json').read().strip().splitlines()[-1]); print(json.dumps({k: r.get(k) for k in ('value','ms_per_step')}))" >> $L || exit 1
done
echo done >> $L
