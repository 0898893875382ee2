#!/bin/bash
# Round 5: experiment-level numbers (scripts/experiments_r05.py) - DARTS B5 create -> Succeeded,
# HyperBand + median stop on ResNet-18 to maxTrialCount, PBT on GPT-2 with the exploit hand-offs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r05i.log
: > $L
for x in darts-b5 hyperband-resnet18 pbt-gpt2; do
  echo "=== $x $(date +%T)" >> $L
  timeout -k 10 900 python scripts/experiments_r05.py --only $x >> $L 2>&1 &
  pid=$!
  while kill -0 $pid 2> /dev/null; do sleep 20; echo "[hb] $x $(date +%T)" >> $L; done
  wait $pid || exit 1
done
echo done >> $L
