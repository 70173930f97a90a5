#!/bin/bash
# Trunk-kernel change check: forward phase attribution, then the fused parity tests (all sizes).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/fwd_diag.py --n 32768 2>&1 | grep -v amdgpu
timeout -k 10 120 python3 tools/fused_micro.py --n 32768 --bwd --no-torch --iters 10 2>&1 | grep -v amdgpu
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_gpu.py \
  tests/test_fused_model_gpu.py tests/test_parity_gpu.py > gpurun_out/trunk_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/trunk_tests.txt; exit $rc
