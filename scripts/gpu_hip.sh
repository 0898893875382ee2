#!/bin/bash
# GPU check of the HIP DARTS path: numerics tests, bench (eager + graph), kernel profile.
# Stops at the first step that crashes/aborts/times out (exit > 1).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/hip.log
run() { "$@"; rc=$?; echo "[rc=$rc] $*" >> $R/$L; return $rc; }
timeout -k 10 600 python -m pytest tests/test_gpu_darts.py -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "[pytest rc=$rc]" >> $L
[ $rc -gt 1 ] && exit $rc
run timeout -k 10 300 python bench.py --ops hip --capture 0 --steps 10 --warmup 3 >> $L 2>&1 || exit 1
run timeout -k 10 300 python bench.py --ops hip --capture 1 --steps 30 --warmup 3 >> $L 2>&1 || exit 1
run timeout -k 10 300 python bench.py --ops hip --capture 1 --steps 20 --warmup 3 --config default >> $L 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_hip -o run -- python3 $R/bench.py --ops hip --capture 0 --steps 3 --warmup 1 >> $R/$L 2>&1
mkdir -p $R/gpurun_out/prof_hip && find /tmp/prof_hip -name "*stats*" -exec cp {} $R/gpurun_out/prof_hip/ \;
echo done >> $R/$L
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_hip_def -o run -- python3 $R/bench.py --ops hip --capture 0 --steps 2 --warmup 1 --config default >> $R/$L 2>&1
mkdir -p $R/gpurun_out/prof_hip_def && find /tmp/prof_hip_def -name "*stats*" -exec cp {} $R/gpurun_out/prof_hip_def/ \;
echo done2 >> $R/$L
