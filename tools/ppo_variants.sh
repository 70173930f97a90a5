cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for a in "--pure-bf16" "--pure-bf16 --channels-last" "--pure-bf16 --fwd-only" "--pure-bf16 --channels-last --fwd-only"; do
  echo "variant: $a"
  timeout -k 10 240 python -u tools/ppo_micro.py --mb 32768 $a 2>&1 | grep -v amdgpu.ids
done
echo "rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pprof2 -o ppo --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 --pure-bf16 --channels-last
echo done
