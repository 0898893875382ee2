#!/bin/bash
# Stem-conv kernels: DARTS GPU tests, both DARTS bench configs, steady-state kernel profiles.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/stem.log
: > $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_darts.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread >> $L 2>&1 || exit $?
for cfg in b5 default; do
  timeout -k 10 300 python bench.py --config $cfg >> $L 2>&1 || exit $?
done
for cfg in b5 default; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_stem_$cfg -o run -- \
    python3 bench.py --config $cfg --steps 10 --warmup 3 --capture 0 > gpurun_out/prof_stem_$cfg.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_stem_$cfg -name '*kernel_trace.csv' | head -n 1)
  python3 scripts/prof_steady.py "$f" 30 > gpurun_out/darts_${cfg}_steady_stem.txt || exit 1
done
echo done >> $L
