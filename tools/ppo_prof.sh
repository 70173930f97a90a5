#!/bin/bash
# Fused-path parity tests, then a kernel trace of PPO minibatch updates (tools/ppo_micro.py).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fused_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/fused_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppo -o p --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 > gpurun_out/ppo_micro.log 2>&1 || { tail -5 gpurun_out/ppo_micro.log; exit 1; }
grep -v "amdgpu.ids\|^W2026\|^E2026" gpurun_out/ppo_micro.log | tail -5
cp $(find /tmp/ppo -name "*kernel_stats.csv") gpurun_out/ppo_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/ppo_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:72]:72s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4s} {float(r['Percentage']):5.1f}%")
PY
