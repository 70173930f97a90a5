#!/bin/bash
# Same-box A/B of the trunk kernels: tools/fused_micro.py (one 96->96 layer at N=32768)
# alternating tools/bin/ab/libmsenv_base.so (A) and tools/bin/ab/libmsenv_b.so (B); the
# fused-kernel parity tests run against B first.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=$PWD/tools/bin/ab/libmsenv_base.so; B=$PWD/tools/bin/ab/libmsenv_b.so
MSENV_LIB=$B timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abf_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/abf_tests.txt; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MSENV_LIB=$lib timeout -k 10 120 python3 tools/fused_micro.py --no-torch --iters 20 ${ABF_ARGS:-} > gpurun_out/abf_$v.log 2>&1 || { tail -5 gpurun_out/abf_$v.log; exit 1; }
    echo "$v $(grep -h "ms" gpurun_out/abf_$v.log | tr '\n' ' ')"
  done
done
