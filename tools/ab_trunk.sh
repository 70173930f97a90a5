#!/bin/bash
# Same-box A/B of the one-launch trunk: tools/trunk_pp_check.py --skip-check (training forward,
# backward and no-grad forward of every forward variant at one 32,768-sample minibatch),
# alternating tools/bin/ab/libmsenv_base.so (A, built from the previous commit) and the
# in-tree libmsenv.so (B), each in its own process.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
A=$PWD/tools/bin/ab/libmsenv_base.so; B=$PWD/minesweeper-ppo_amd/libmsenv.so
for rep in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MSENV_LIB=$lib timeout -k 10 200 python3 -u tools/trunk_pp_check.py --skip-check ${ABT_ARGS:-} > gpurun_out/abt_$v.log 2>&1 || { tail -5 gpurun_out/abt_$v.log; exit 1; }
    grep "round 0" gpurun_out/abt_$v.log | sed "s/^/$v rep $rep: /"
  done
done
