#!/bin/bash
# Replica-count x fold-strategy sweep of the DARTS cross-workgroup reductions on one MI355X:
# in-tree build (REP=32) and variants built with _build.build_hip(defines=["KATIB_HIP_REP=R"],
# out=variants/repR/_hipkern.so), each with fold launches (KATIB_HIP_FOLD=1) and with
# consumer-side replica sums (KATIB_HIP_FOLD=0).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/rep_sweep.log
: > $L
for v in "" variants/rep16/_hipkern.so variants/rep8/_hipkern.so; do
  for fold in 1 0; do
    echo "=== so=${v:-in-tree} fold=$fold" >> $L
    KATIB_AMD_HIPKERN=$v KATIB_HIP_FOLD=$fold timeout -k 10 240 python bench.py --steps 40 --warmup 5 \
      --full-search 0 >> $L 2>&1 || exit $?
  done
done
KATIB_AMD_HIPKERN=variants/rep8/_hipkern.so KATIB_HIP_FOLD=0 timeout -k 10 300 python -m pytest -q -x \
  tests/test_gpu_darts.py -k "search_step or evaluate" -p no:cacheprovider >> $L 2>&1 || exit $?
echo done >> $L
