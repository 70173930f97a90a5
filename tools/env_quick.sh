#!/bin/bash
# Env-path check after a board-step / tape change: the env + RL GPU tests, the k_tape / k_step
# timeline of the headline bench under a kernel trace (tools/step_gaps.py), then an untraced
# env-only bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_rl_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tape_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/tape_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sg -o s --output-format csv -- python3 bench.py --no-cpu-baseline --ppo-updates 0 --extras= --steps 200 --warmup 10 > gpurun_out/sg.log 2>&1 || exit $?
python3 tools/step_gaps.py --trace /tmp/sg || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --ppo-updates 0 --steps 200 --warmup 10 > gpurun_out/b_env.log 2>&1 || exit $?
grep "^{" gpurun_out/b_env.log | tail -1 | python3 -c '
import json, sys
l = json.loads(sys.stdin.read())
print("headline", l["value"], "ms/step", l["ms_per_step"], "frac", l["roofline"]["frac"])
for p in l.get("north_star_points", []):
    print(p["board"], p["envs_per_gpu"], p["value"], p["roofline"]["frac"])'
