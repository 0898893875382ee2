#!/bin/bash
# DARTS kernel iteration on one MI355X: numerics tests, B5 + default benches, default-config kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/darts_iter.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_darts.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $L 2>&1 || exit $?
timeout -k 10 300 python bench.py --config default --steps 10 --warmup 3 >> $L 2>&1 || exit $?
# A/B: the default config under experiment switches, ';'-separated (e.g. "KATIB_HIP_DWB_GROUP=8;KATIB_HIP_DW_GROUP=8")
IFS=';' read -ra EXPS <<< "${DARTS_EXP_ENV:-}"
for e in "${EXPS[@]}"; do
  echo "exp: $e" >> $L
  timeout -k 10 300 env $e python bench.py --config default --steps 10 --warmup 3 >> $L 2>&1 || exit $?
done
rm -rf gpurun_out/prof_darts_default
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_darts_default -o run -- \
  python3 bench.py --config default --steps 5 --warmup 2 >> $L 2>&1 || exit 1
f=$(find gpurun_out/prof_darts_default -name '*kernel_stats.csv' | head -n 1)
python3 scripts/prof_summary.py "$f" 45 > gpurun_out/darts_default_kernel_stats.txt || exit 1
echo done >> $L
