#!/bin/bash
# A/B of the hoisted first-element loads (combine_fwd / combine_bwd_reduce / pool_bwd): B5 kernel timeline with
# the HEAD library (_hipkern_base.so) and the working tree's, alternated twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06i.log
: > $L
for rep in 1 2; do
for lib in base new; do
  if [ $lib = base ]; then export KATIB_AMD_HIPKERN=$(pwd)/katib_amd/_hipkern_base.so; else unset KATIB_AMD_HIPKERN; fi
  rm -rf gpurun_out/prof_ab
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ab -o run -- \
    python3 bench.py --steps 10 --warmup 3 --trials 0 --b1 0 --experiment 0 --comparator-steps 0 --full-search 0 --floor 0 \
    > gpurun_out/prof_ab.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_ab -name '*kernel_trace.csv' | head -n 1)
  echo "=== $lib (rep $rep)" >> $L
  python3 scripts/prof_timeline.py "$f" virtual_step_kernel 5 >> $L || exit 1
done
done
rm -rf gpurun_out/prof_ab
echo done >> $L
