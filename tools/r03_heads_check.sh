#!/bin/bash
# k_heads_bwd (64-row tiles, two workgroups per CU): heads / fused-model / parity GPU tests,
# then the PPO minibatch under a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_model_gpu.py tests/test_parity_gpu.py tests/test_trainer_prod_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/heads_tests.log 2>&1
rc=$?; tail -3 gpurun_out/heads_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/hprof -o h --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 > gpurun_out/heads_prof.log 2>&1 || exit $?
grep "ms/iter" gpurun_out/heads_prof.log
cp $(find /tmp/hprof -name "*kernel_stats.csv") gpurun_out/heads_kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/heads_kernel_stats.csv")):
    if "heads" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
