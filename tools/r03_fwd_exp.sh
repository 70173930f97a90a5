#!/bin/bash
# Forward-kernel timing experiments: the product library, then tools/bin/exp1 (memory wave without
# the epilogue arithmetic) and tools/bin/exp2 (compute waves without the convolution).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in prod exp1 exp2; do
  lib=""; [ $v != prod ] && lib=$PWD/tools/bin/$v/libmsenv.so
  MSENV_LIB=$lib timeout -k 10 200 python3 -u tools/fwd_ab.py --n 32768 --iters 10 --reps 2 --dtypes fp16 > gpurun_out/fwd_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -v amdgpu.ids gpurun_out/fwd_$v.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
