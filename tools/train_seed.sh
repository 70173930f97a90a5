#!/bin/bash
# Training-quality run of the shipped config (fp16 + GradScaler, fused path) for one seed:
# SEED=1 bash tools/train_seed.sh. Checkpoints stay on the box; metrics come back.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
S=${SEED:-1}
mkdir -p gpurun_out/train_s$S
timeout -k 10 1080 python3 -u train_rl.py --config configs/training/16x16x40_medium.yaml --seed $S \
  --out /tmp/run_s$S --quick_eval_interval 100 > gpurun_out/train_s$S/train.log 2>&1
rc=$?
cp /tmp/run_s$S/train_metrics.csv /tmp/run_s$S/summary.json gpurun_out/train_s$S/ 2>/dev/null
grep -h "quick eval\|final eval\|Early" gpurun_out/train_s$S/train.log > gpurun_out/train_s$S/quick_evals.log
tail -3 gpurun_out/train_s$S/quick_evals.log
exit $rc
