#!/bin/bash
# Round 5: B1 trial step composition (module path: --num-layers / --optimizer given) - train_seconds and kernels per
# step for bf16 autocast vs fp32, sgd vs adam, one trial alone on the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
L=gpurun_out/r05gg.log
: > $L
for dt in bf16 fp32; do
  for opt in sgd adam; do
    echo "--- $dt $opt" >> $L
    timeout -k 10 120 python -m katib_amd.workloads.mnist_mlp --batch-size=64 --lr=0.05 --num-layers=3 --optimizer=$opt --epochs=2 --dtype $dt >> $L 2>&1 || exit 1
  done
done
cd /tmp
for dt in bf16 fp32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_mlp_$dt -o run -- python3 -m katib_amd.workloads.mnist_mlp --batch-size=64 --lr=0.05 --num-layers=3 --optimizer=sgd --epochs=1 --num-train 6400 --dtype $dt >> $R/$L 2>&1 || exit 1
  python3 - "$dt" >> $R/$L 2>&1 <<'PY' || exit 1
import sqlite3, sys
dt = sys.argv[1]
c = sqlite3.connect(f"/tmp/prof_mlp_{dt}/run_results.db")
rows = list(c.execute("select name,total_calls,total_duration,average from top_kernels"))
print(dt, "kernels", sum(r[1] for r in rows), "total_us", round(sum(r[2] for r in rows)))
for n, k, t, a in rows[:24]:
    print(f"  {n[:90]:90s} {k:6d} {a:7.2f}")
PY
done
echo done >> $R/$L
