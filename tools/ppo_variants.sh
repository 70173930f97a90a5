cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for a in "" "--benchmark" "--channels-last" "--channels-last --benchmark" "--fwd-only --benchmark" "--fwd-only --channels-last --benchmark" "--mb 8192 --benchmark" "--amp fp16 --benchmark"; do
  timeout -k 10 300 python tools/ppo_micro.py --mb 32768 $a 2>&1 | grep -v amdgpu.ids | tail -1 || { echo "FAIL $a"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pprof -o ppo --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --benchmark --iters 3 > /dev/null 2>&1
