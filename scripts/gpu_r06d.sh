#!/bin/bash
# Round 6 check after the knob pruning and the restored gemm256 schedule: the whole GPU suite, smoke, the
# B5 bench line, the GPT-2 member (fused eval cross-entropy + argmax) with its kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r06d.log
: > $L
echo "=== pytest -m gpu $(date +%T)" >> $L
timeout -k 10 1000 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu >> $L 2>&1 || exit 1
echo "=== smoke $(date +%T)" >> $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || exit 1
echo "=== bench N=1 $(date +%T)" >> $L
timeout -k 10 600 python bench.py >> $L 2>&1 || exit 1
echo "=== gpt2 member $(date +%T)" >> $L
timeout -k 10 300 python -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 40 --checkpoint-dir /tmp/g2 --save-files 0 >> $L 2>&1 || exit 1
echo "=== gpt2 prof $(date +%T)" >> $L
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gpt2 -o run -- \
  python3 -m katib_amd.workloads.gpt2_pbt --batch-size 16 --steps 12 --checkpoint-dir /tmp/g3 --save-files 0) >> $L 2>&1 || exit 1
mkdir -p $R/gpurun_out/prof_gpt2_r06 && find /tmp/prof_gpt2 -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_gpt2_r06/ \;
echo done >> $L
