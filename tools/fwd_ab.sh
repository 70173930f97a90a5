#!/bin/bash
# A/B of the forward layer kernels: parity tests of the fused path, then per-kernel
# durations (rocprofv3 --stats) of tools/fused_micro.py with MC_FWD_RW=0 / 1.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fused_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/fused_tests.txt; [ $rc -ne 0 ] && exit $rc
for rw in ${RWS:-0 1}; do
  d=/tmp/ab_$rw
  MC_FWD_RW=$rw timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o s --output-format csv -- \
    python3 tools/fused_micro.py --no-torch --bwd --iters 5 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep -v amdgpu.ids $d.log
  python3 - "$(find $d -name '*kernel_stats.csv')" $rw <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["Percentage"]) > 1.0:
        print(f"  rw={sys.argv[2]} {r['Name'][:70]:70s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']}")
PY
done
