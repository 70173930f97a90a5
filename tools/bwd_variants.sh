#!/bin/bash
# Timing attribution for k_bwd_data: libmsenv variants with parts compiled out (MC_EXP_B_*
# hooks in csrc/mscnn_bwd.hip; results are WRONG by design), each timed by rocprofv3's
# kernel trace over tools/fused_micro.py --bwd. Run on the GPU box: bash tools/bwd_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PKG=minesweeper-ppo_amd
SRCS="$PKG/csrc/msenv.hip $PKG/csrc/mscnn.hip $PKG/csrc/mscnn_bwd.hip $PKG/csrc/msheads.hip"
: > gpurun_out/bwd_variants.log
for v in ${VARIANTS:-base NO_DGRAD NO_EPI NO_P1LOAD NO_DYSTORE}; do
  so=tools/bin/libmsenv_exp_$v.so  # prebuilt on the CPU container (BUILD=1 builds here)
  [ $v = base ] && so=$PKG/libmsenv.so
  if [ "${BUILD:-0}" = "1" ] && [ $v != base ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DMC_EXP_B_$v -shared -o $so $SRCS || exit 1
  fi
  rm -rf /tmp/bv_$v
  MSENV_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/bv_$v -o t --output-format csv -- \
    python3 tools/fused_micro.py --no-torch --bwd ${EXP_ARGS:-} > /tmp/bv_$v.log 2>&1 || exit $?
  f=$(find /tmp/bv_$v -name "*kernel_stats.csv")
  echo "== $v" >> gpurun_out/bwd_variants.log
  python3 -c "
import csv, sys
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('k_bwd_data', 'k_wgrad', 'k_conv_gn_fwd')):
        print(f\"{r['Name'][:70]} avg_us={float(r['AverageNs']) / 1e3:.1f} calls={r['Calls']}\")
" >> gpurun_out/bwd_variants.log
done
cat gpurun_out/bwd_variants.log
