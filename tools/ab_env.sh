#!/bin/bash
# Same-box A/B of the env path: bench.py env lines (no PPO, no CPU baseline) alternating
# between tools/bin/ab/libmsenv_base.so (A, a baseline build) and tools/bin/ab/libmsenv_b.so
# (B, the candidate) when it exists, else the product libmsenv.so. AB_TESTS=1 first runs the
# env GPU tests against B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BLIB=$PWD/tools/bin/ab/libmsenv_b.so
[ -f "$BLIB" ] || BLIB=$PWD/minesweeper-ppo_amd/libmsenv.so
if [ "${AB_TESTS:-0}" = 1 ]; then
  MSENV_LIB=$BLIB timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_rl_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.txt 2>&1
  rc=$?; tail -2 gpurun_out/ab_tests.txt; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export MSENV_LIB=$PWD/tools/bin/ab/libmsenv_base.so; else export MSENV_LIB=$BLIB; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --ppo-updates 0 --steps 300 --warmup 20 ${AB_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    grep "^{" gpurun_out/ab_$v.log | tail -1 | python3 -c '
import json, sys
l = json.loads(sys.stdin.read())
f = lambda p: "%s@%d %.0fM/s k %.3f ms %.3f" % (p.get("board", p.get("config", {}).get("board")), p.get("envs_per_gpu", p.get("config", {}).get("envs_per_gpu", 0)), p["value"] / 1e6, p["roofline"]["frac"], p.get("multistep", {}).get("roofline", {}).get("frac", 0))
print("'$v'", " | ".join([f(l)] + [f(p) for p in l.get("north_star_points", [])]))'
  done
done
