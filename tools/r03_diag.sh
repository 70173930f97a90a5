#!/bin/bash
# Phase stamps of k_step (libmsenv_diag.so) at the headline and the 9x9 point, with the
# placement sub-phases (tools/diag_step.py).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 16x16x40:4096 9x9x10:8192 30x16x99:8192; do
  timeout -k 10 120 python3 -u tools/diag_step.py --board ${b%%:*} --envs ${b##*:} --steps 20 > gpurun_out/diag_${b%%:*}.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/diag_${b%%:*}.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
