#!/bin/bash
# Round-6 final check on the final code: the whole GPU suite, smoke, the B5 bench line (N=1), a 2-rank
# shared-GPU rehearsal of the N>1 path, and the B5 kernel timeline (rocprofv3 kernel trace).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r06_final.log
: > $L
echo "=== pytest -m gpu $(date +%T)" >> $L
timeout -k 10 1000 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
echo "=== smoke $(date +%T)" >> $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || exit 1
echo "=== bench N=1 $(date +%T)" >> $L
timeout -k 10 600 python bench.py >> $L 2>&1 || exit 1
echo "=== bench --gpus 2 (both ranks on this one GPU: a rehearsal of the N>1 path, not a scaling number) $(date +%T)" >> $L
timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 \
  --full-search 0 --floor 0 >> $L 2>&1 || exit 1
echo "=== B5 timeline $(date +%T)" >> $L
timeout -k 10 400 bash scripts/gpu_prof_timeline.sh b5 >> $L 2>&1 || exit 1
cat gpurun_out/darts_b5_timeline.txt >> $L
echo done >> $L
