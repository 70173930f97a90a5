#!/bin/bash
# Late-start cost (shared vs keyed generator), then one full-length (4000-update, no early stop)
# training run of the shipped config, seed 0.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/late_bench.py --envs 4096 --steps 100 > gpurun_out/late_bench.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/late_bench.txt; [ $rc -ne 0 ] && exit $rc
CONFIG=configs/training/16x16x40_medium_noearlystop.yaml SEEDS="0" TAG=full4000 LIMIT=1060 bash tools/train_quality.sh
