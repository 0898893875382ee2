#!/bin/bash
# NHWC depthwise conv kernels: numerics tests, ENAS child trial run, kernel profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/dwconv.log
: > $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_dwconv.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider >> $L 2>&1 || exit $?
ARCH="[[0], [1, 0], [2, 0, 1], [3, 0, 0, 1], [4, 0, 1, 0, 0], [5, 0, 0, 0, 0, 1]]"
timeout -k 10 300 python -m katib_amd.workloads.enas_child --num_epochs 1 --num-train 12800 --num-valid 2000 \
  --architecture "$ARCH" --nn_config "$(python scripts/enas_nn_config.py)" >> $L 2>&1 || exit $?
rm -rf gpurun_out/prof_enas_child
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enas_child -o run -- \
  python3 -m katib_amd.workloads.enas_child --num_epochs 1 --num-train 12800 --num-valid 2000 \
  --architecture "$ARCH" --nn_config "$(python scripts/enas_nn_config.py)" >> $L 2>&1 || exit $?
f=$(find gpurun_out/prof_enas_child -name '*kernel_stats.csv' | head -n 1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/enas_child_kernel_stats.txt || exit 1
echo done >> $L
