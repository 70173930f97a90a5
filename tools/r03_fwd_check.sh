#!/bin/bash
# The weight-resident forward: same-process A/B against the per-sample kernel (tools/fwd_ab.py),
# then the fused parity tests (both kernels) and the model-level fused tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/fwd_ab.py --n 32768 --iters 10 > gpurun_out/fwd_ab.txt 2>&1
rc=$?; cat gpurun_out/fwd_ab.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=15 \
  tests/test_fused_gpu.py tests/test_fused_model_gpu.py tests/test_trainer_prod_gpu.py > gpurun_out/fwd_tests.txt 2>&1
rc=$?; tail -22 gpurun_out/fwd_tests.txt; exit $rc
