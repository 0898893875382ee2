#!/bin/bash
# numerics tests, then per-config bench sweep over the persistent-grid block cap
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/sweep.log
: > $L
timeout -k 10 600 python -m pytest tests/test_gpu_darts.py -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "[pytest rc=$rc]" >> $L
[ $rc -gt 1 ] && exit $rc
for cfg in b5 default; do
  for mb in ${SWEEP:-256 512 1024 2048}; do
    echo "cfg=$cfg maxblocks=$mb" >> $L
    KATIB_HIP_MAX_BLOCKS=$mb timeout -k 10 300 python bench.py --ops hip --capture 1 --steps 20 --warmup 3 --config $cfg >> $L 2>&1 || exit 1
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_hip_def -o run -- python3 $R/bench.py --ops hip --capture 0 --steps 2 --warmup 1 --config default >> $R/$L 2>&1
mkdir -p $R/gpurun_out/prof_hip_def && find /tmp/prof_hip_def -name "*stats*" -exec cp {} $R/gpurun_out/prof_hip_def/ \;
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_hip -o run -- python3 $R/bench.py --ops hip --capture 0 --steps 3 --warmup 1 >> $R/$L 2>&1
mkdir -p $R/gpurun_out/prof_hip && find /tmp/prof_hip -name "*stats*" -exec cp {} $R/gpurun_out/prof_hip/ \;
echo done >> $R/$L
