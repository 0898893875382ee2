#!/bin/bash
# GPU probe: eager vs graph-captured DARTS step on torch ops + kernel profile summary
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/probe.log
python -c "import torch;print(torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))" > $L 2>&1 || exit 1
timeout -k 10 300 python bench.py --ops torch --capture 0 --steps 10 --warmup 3 >> $L 2>&1 || exit 1
timeout -k 10 300 python bench.py --ops torch --capture 1 --steps 30 --warmup 3 >> $L 2>&1 || exit 1
timeout -k 10 300 python bench.py --ops torch --capture 1 --steps 20 --warmup 3 --config default >> $L 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_eager -o run -- python3 $R/bench.py --ops torch --capture 0 --steps 3 --warmup 1 >> $R/$L 2>&1
find /tmp/prof_eager -name "*stats*" -exec cp {} $R/gpurun_out/ \; ; ls -la /tmp/prof_eager >> $R/$L 2>&1
echo done >> $R/$L
