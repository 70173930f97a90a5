#!/bin/bash
# Same-box A/B/... of trunk-kernel candidates: the fused parity tests run against the LAST
# library first, then tools/fused_micro.py alternates every library (tools/bin/ab/libmsenv_<v>.so
# for v in $AB_LIBS, default "base b") three times. ABF_ARGS is passed to fused_micro.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${AB_LIBS:-"base b"}
last=${LIBS##* }
MSENV_LIB=$PWD/tools/bin/ab/libmsenv_$last.so timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abm_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/abm_tests.txt; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in $LIBS; do
    MSENV_LIB=$PWD/tools/bin/ab/libmsenv_$v.so timeout -k 10 120 python3 tools/fused_micro.py --no-torch --iters 20 ${ABF_ARGS:-} > gpurun_out/abm_$v.log 2>&1 || { tail -5 gpurun_out/abm_$v.log; exit 1; }
    echo "$v $(grep -h "ms" gpurun_out/abm_$v.log | tr '\n' ' ')"
  done
done
