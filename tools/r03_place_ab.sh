#!/bin/bash
# Placement A/B (closed-form Floyd collisions in place_fixpoint) + 16x16 phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
AB_TESTS=1 bash tools/ab_env.sh || exit $?
timeout -k 10 120 python3 -u tools/diag_step.py --board 16x16x40 --envs 4096 --steps 20 > gpurun_out/diag_16.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/diag_16.txt; exit $rc
