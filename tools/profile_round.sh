#!/bin/bash
# rocprofv3 evidence for one round -> gpurun_out/prof_<tag>/ (raw traces stay in /tmp):
#  1. kernel trace + stats of the default env-step bench (graph mode; per-step line + multistep line)
#  2./3. PMC passes FETCH_SIZE and WRITE_SIZE (separate passes) -> pmc json for k_step and k_run
#  4. kernel trace + stats of PPO minibatch updates (tools/ppo_micro.py)
# Every GPU step has its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
RAW=/tmp/prof_$TAG
mkdir -p $OUT $RAW
B="--no-cpu-baseline --ppo-updates 0 --steps 200 --warmup 25"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $RAW/trace -o bench --output-format csv -- python3 bench.py $B > $OUT/bench_trace.log 2>&1 || exit $?
cp $(find $RAW/trace -name "*kernel_stats.csv") $OUT/bench_env_step_kernel_stats.csv
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $RAW/pmc_fetch -o bench --output-format csv -- python3 bench.py $B --graph 0 > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $RAW/pmc_write -o bench --output-format csv -- python3 bench.py $B --graph 0 > $OUT/pmc_write.log 2>&1 || exit $?
CMD="rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} (separate passes) -- python3 bench.py $B --graph 0"
python3 tools/pmc_summary.py --fetch $RAW/pmc_fetch --write $RAW/pmc_write --kernel k_step \
  --out $OUT/pmc_k_step_16x16x40_4096.json --command "$CMD" || exit $?
python3 tools/pmc_summary.py --fetch $RAW/pmc_fetch --write $RAW/pmc_write --kernel k_run \
  --out $OUT/pmc_k_run_16x16x40_4096.json --command "$CMD" --steps-per-launch 25 \
  --algo-bytes $((10729 * 4096 * 25)) --config "16x16x40, 4096 envs, tape 0, 25 steps per launch" || exit $?
if [ "${PPO:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $RAW/ppo -o ppo --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 > $OUT/ppo.log 2>&1 || exit $?
  cp $(find $RAW/ppo -name "*kernel_stats.csv") $OUT/ppo_minibatch_fused_kernel_stats.csv
fi
echo profile done
