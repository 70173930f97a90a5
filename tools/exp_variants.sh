#!/bin/bash
# Timing attribution for the fused layer kernels: build libmsenv variants with parts of
# the forward kernel compiled out (MC_EXP_* hooks in csrc/mscnn.hip; results are WRONG
# by design) and time each with tools/fused_micro.py. Run on the GPU box:
#   bash tools/exp_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PKG=minesweeper-ppo_amd
SRCS="$PKG/csrc/msenv.hip $PKG/csrc/mscnn.hip $PKG/csrc/mscnn_bwd.hip $PKG/csrc/msheads.hip"
for v in ${VARIANTS:-base NO_EPI NO_WLOAD NO_STATS NO_IN NO_MFMA}; do
  so=/tmp/libmsenv_exp_$v.so
  D=""; [ $v != base ] && D="-DMC_EXP_$v"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $D -shared -o $so $SRCS || exit 1
  echo "== $v" >> gpurun_out/exp.log
  MSENV_LIB=$so timeout -k 10 120 python tools/fused_micro.py --no-torch ${EXP_ARGS:-} >> gpurun_out/exp.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/exp.log
