#!/bin/bash
# Produce the rocprofv3 evidence for one round under gpurun_out/prof_<tag>/:
#  1. kernel trace + stats of the default bench command (env step, graph mode)
#  2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE (separate passes: gfx950 TCC slots)
# Every GPU step has its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="--no-cpu-baseline --ppo-updates 0 --steps 200 --warmup 20"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py $B > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o bench --output-format csv -- python3 bench.py $B --graph 0 > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o bench --output-format csv -- python3 bench.py $B --graph 0 > $OUT/pmc_write.log 2>&1 || exit $?
if [ "${PPO:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/ppo -o ppo --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 > $OUT/ppo.log 2>&1 || exit $?
fi
echo profile done
