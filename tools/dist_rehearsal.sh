#!/bin/bash
# The driver's N>1 bench path (torchrun, one process per rank, barriers, max-over-ranks
# timing, the Trainer's flat-gradient all-reduce) rehearsed on a one-GPU box: 2 ranks share
# cuda:0 over gloo (MS_BENCH_BACKEND=gloo), small step counts.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MS_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 50 --warmup 5 \
  --extras 16x16x40:8192 --ppo-updates 1 --ppo-steps-per-env 16 > gpurun_out/dist_rehearsal.log 2>&1
rc=$?; tail -3 gpurun_out/dist_rehearsal.log | cut -c1-600; exit $rc
