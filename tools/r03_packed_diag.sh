#!/bin/bash
# Phase stamps of k_step_packed vs k_step (MS_DBG_ONE_BOARD_PER_WAVE) at 9x9x10 @ 8192.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for fl in ${FLAGS:-0 8}; do
  timeout -k 10 120 python3 -u tools/diag_step.py --board 9x9x10 --envs 8192 --steps 20 --debug-flags $fl \
    > gpurun_out/pdiag_$fl.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/pdiag_$fl.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
