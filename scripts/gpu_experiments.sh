#!/bin/bash
# The BASELINE experiment configs end to end through the scheduler on one MI355X (all trial
# slots on GPU 0): DARTS B5 search, TPE on the MNIST MLP, HyperBand + median stop on
# ResNet-18, ENAS and PBT on GPT-2 small (ENAS / PBT budgets reduced to 16 trials).
# ONLY=1 runs just ENAS and PBT; SKIP_PBT=1 drops PBT.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out /tmp/katib_exp
export TMPDIR=/tmp
L=gpurun_out/experiments.log
: > $L
run() {  # run <name> <timeout> <yaml>
  echo "=== $1" >> $L
  local t0=$(date +%s.%N)
  timeout -k 10 $2 python -m katib_amd run "$3" --slots-per-gpu 8 --state-dir /tmp/katib_exp/$1 >> $L 2>&1 &
  local pid=$!
  while kill -0 $pid 2> /dev/null; do  # heartbeat: the CLI prints only at the end
    sleep 20
    echo "[hb] $1 t=$(python3 -c "import time; print(round(time.time() - $t0))")s state=$(du -sk /tmp/katib_exp/$1 2> /dev/null | cut -f1)KB" >> $L
  done
  wait $pid
  local rc=$?
  echo "[rc=$rc] $1 wall_s=$(python3 -c "import time; print(round(time.time() - $t0, 2))")" >> $L
  return $rc
}
sed 's/maxTrialCount: 64/maxTrialCount: 16/' examples/nas/enas-cifar10.yaml > /tmp/katib_exp/enas16.yaml
sed 's/maxTrialCount: 64/maxTrialCount: 16/' examples/pbt/pbt-gpt2-small.yaml > /tmp/katib_exp/pbt16.yaml
[ -n "$ONLY" ] || { run darts-b5 300 examples/nas/darts-cifar10.yaml || exit $?; }
[ -n "$ONLY" ] || { run tpe-mnist-mlp 300 examples/hp-tuning/tpe-mnist-mlp.yaml || exit $?; }
[ -n "$ONLY" ] || { run hyperband-resnet18 600 examples/early-stopping/hyperband-medianstop-resnet18.yaml || exit $?; }
run enas 600 /tmp/katib_exp/enas16.yaml || exit $?
[ -n "$SKIP_PBT" ] || { run pbt-gpt2 600 /tmp/katib_exp/pbt16.yaml || exit $?; }
echo done >> $L
