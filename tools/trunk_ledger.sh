#!/bin/bash
# Byte ledger of the trunk kernels: tools/ppo_micro.py (one 32,768-sample
# PPO minibatch, fp16) under rocprofv3 -- kernel trace, FETCH_SIZE, WRITE_SIZE and MFMA-busy /
# GRBM_GUI_ACTIVE passes, each in its own run -- for the library named by LIBS (label=path,
# space-separated; default: the in-tree libmsenv.so) -> gpurun_out/ledger_<label>.json
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-"tree=$PWD/minesweeper-ppo_amd/libmsenv.so"}
P="python3 tools/ppo_micro.py --mb 32768 --iters 3"
for ent in $LIBS; do
  lab=${ent%%=*}; lib=${ent#*=}; RAW=/tmp/ledger_$lab
  rm -rf $RAW; mkdir -p $RAW
  export MSENV_LIB=$lib
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $RAW/t -o t --output-format csv -- $P > gpurun_out/ledger_${lab}_t.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $RAW/f -o p --output-format csv -- $P > gpurun_out/ledger_${lab}_f.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $RAW/w -o p --output-format csv -- $P > gpurun_out/ledger_${lab}_w.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $RAW/m -o p --output-format csv -- $P > gpurun_out/ledger_${lab}_m.log 2>&1 || exit $?
  python3 tools/ppo_pmc_summary.py --fetch $RAW/f --write $RAW/w --mfma $RAW/m --trace $RAW/t \
    --samples 32768 --out gpurun_out/ledger_$lab.json > gpurun_out/ledger_$lab.txt || exit $?
  echo "== $lab"; head -8 gpurun_out/ledger_$lab.txt
done
