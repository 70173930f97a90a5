#!/bin/bash
# Training-quality runs, the seeds side by side on the one GPU (each run is
# launch-bound at 128 envs, so they share the card well):
#   CONFIG=<yaml> SEEDS="0 1 2" TAG=<name> bash tools/train_quality.sh
# One train_rl.py run per seed (fp16 + GradScaler, fused path), each under its own time limit;
# metrics, quick evals and the summary come back under gpurun_out/train_<TAG>_s<seed>/.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-configs/training/16x16x40_medium.yaml}
TAG=${TAG:-default}
LIMIT=${LIMIT:-1100}
pids=()
for S in ${SEEDS:-0}; do
  D=gpurun_out/train_${TAG}_s$S
  mkdir -p $D
  timeout -k 10 $LIMIT python3 -u train_rl.py --config $CONFIG --seed $S --out /tmp/run_${TAG}_s$S \
    --quick_eval_interval 100 > $D/train.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
for S in ${SEEDS:-0}; do
  D=gpurun_out/train_${TAG}_s$S
  cp /tmp/run_${TAG}_s$S/train_metrics.csv /tmp/run_${TAG}_s$S/summary.json $D/ 2>/dev/null
  grep -h "quick eval\|final eval\|Early" $D/train.log > $D/quick_evals.log
  echo "seed $S:"; tail -2 $D/quick_evals.log
done
exit $rc
