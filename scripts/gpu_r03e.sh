#!/bin/bash
# Round check after the deferred-fold commits: GPU tests, graft smoke, the driver's default bench
# line, then a kernel-trace profile of the B5 step (per-kernel stats + launch count).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03e.log
: > $L
echo "=== pytest-gpu" >> $L
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
echo "=== smoke" >> $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || exit 1
echo "=== bench" >> $L
timeout -k 10 600 python bench.py >> $L 2>&1 || exit 1
echo "=== prof" >> $L
rm -rf gpurun_out/prof_e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o b5 -- python3 bench.py --steps 20 --warmup 5 --trials 0 --comparator-steps 0 --full-search 0 >> $L 2>&1 || exit 1
echo done >> $L
