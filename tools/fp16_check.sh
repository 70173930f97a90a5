set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_model_gpu.py tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread -k "fused or heads or conv_gn" > gpurun_out/fp16_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/fp16_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/ppo_micro.py --mb 32768 --iters 5 --amp bf16 2>&1 | grep mb= &&
timeout -k 10 200 python3 tools/ppo_micro.py --mb 32768 --iters 5 --amp fp16 2>&1 | grep mb= &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppo16 -o p --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 --amp fp16 > gpurun_out/ppo_micro16.log 2>&1 &&
cp $(find /tmp/ppo16 -name "*kernel_stats.csv") gpurun_out/ppo16_kernel_stats.csv && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/ppo16_kernel_stats.csv")))
for r in rows[:10]:
    print(f"{r['Name'][:80]:80s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4s} {float(r['Percentage']):5.1f}%")
PY
