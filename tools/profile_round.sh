#!/bin/bash
# rocprofv3 evidence for one round -> gpurun_out/prof_<tag>/ (raw traces stay in /tmp):
#  1. the default bench.py run under --kernel-trace --stats: its JSON line and kernel stats come
#     from the SAME process, so every roofline fraction recomputes from the committed trace
#  2. per benchmark config (headline + north-star points): FETCH_SIZE and WRITE_SIZE passes
#     (separate runs) -> pmc_k_step_<board>_<n>.json / pmc_k_run_<board>_<n>.json
#  3. PPO minibatch (tools/ppo_micro.py): kernel trace, FETCH/WRITE and MFMA-busy passes
# Every GPU step has its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/prof_$TAG
RAW=/tmp/prof_$TAG
mkdir -p $OUT $RAW
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $RAW/trace -o bench --output-format csv -- python3 bench.py > $OUT/bench_trace.log 2>&1 || exit $?
  grep '^{' $OUT/bench_trace.log | tail -1 > $OUT/bench_line_n1.json
  cp $(find $RAW/trace -name "*kernel_stats.csv") $OUT/bench_kernel_stats.csv
  python3 tools/trace_check.py --trace $RAW/trace --line $OUT/bench_line_n1.json --out $OUT/trace_check.json || exit $?
fi
if [ "${PMC:-1}" = "1" ]; then
  for cfg in 16x16x40:4096 16x16x40:32768 9x9x10:8192 30x16x99:8192; do
    b=${cfg%%:*}; n=${cfg##*:}
    B="--no-cpu-baseline --ppo-updates 0 --extras= --steps 100 --warmup 10 --graph 0 --board $b --envs $n"
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $RAW/f_${b}_${n} -o p --output-format csv -- python3 bench.py $B > $OUT/pmc_fetch_${b}_$n.log 2>&1 || exit $?
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $RAW/w_${b}_${n} -o p --output-format csv -- python3 bench.py $B > $OUT/pmc_write_${b}_$n.log 2>&1 || exit $?
    H=${b%%x*}; r=${b#*x}; W=${r%%x*}; A=$((H * W))
    BPE=$((40 * A + A + 8 + 4 + 1 + 12 + 2 * (2 * ((A + 7) / 8) + 32) + 16))
    CMD="rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} (separate passes) -- python3 bench.py $B"
    python3 tools/pmc_summary.py --fetch $RAW/f_${b}_${n} --write $RAW/w_${b}_${n} --kernel k_step \
      --out $OUT/pmc_k_step_${b}_$n.json --command "$CMD" --algo-bytes $((BPE * n)) \
      --config "$b, $n envs, tape 0" || exit $?
    python3 tools/pmc_summary.py --fetch $RAW/f_${b}_${n} --write $RAW/w_${b}_${n} --kernel k_run \
      --out $OUT/pmc_k_run_${b}_$n.json --command "$CMD" --algo-bytes $((BPE * n)) \
      --bench-log $OUT/pmc_write_${b}_$n.log --config "$b, $n envs, tape 0" || exit $?
  done
fi
if [ "${PPO:-1}" = "1" ]; then
  P="python3 tools/ppo_micro.py --mb 32768 --iters 3"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $RAW/ppo -o ppo --output-format csv -- $P > $OUT/ppo.log 2>&1 || exit $?
  cp $(find $RAW/ppo -name "*kernel_stats.csv") $OUT/ppo_minibatch_fused_kernel_stats.csv
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $RAW/ppo_f -o p --output-format csv -- $P > $OUT/ppo_pmc_f.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $RAW/ppo_w -o p --output-format csv -- $P > $OUT/ppo_pmc_w.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $RAW/ppo_m -o p --output-format csv -- $P > $OUT/ppo_pmc_m.log 2>&1 || exit $?
  python3 tools/ppo_pmc_summary.py --fetch $RAW/ppo_f --write $RAW/ppo_w --mfma $RAW/ppo_m --trace $RAW/ppo \
    --samples 32768 --out $OUT/pmc_ppo_minibatch_32768.json || exit $?
fi
echo profile done
