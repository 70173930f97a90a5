#!/bin/bash
# One rocprofv3 --pmc pass (wave states + MFMA busy) over the trunk kernel variants at N = 32,768:
# the per-sample kernels (variant 1), the pixel-split wave-specialised forward / backward
# (variant 3) and the channel-split forward (variants 4, 5) -> gpurun_out/ws_sq/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/ws_sq
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d /tmp/ws_sq -o p --output-format csv -- python3 tools/fused_micro.py --no-torch --iters 3 --mask --bwd --variants 1,3,4,5 \
  > $OUT/pass.log 2>&1 || { tail -5 $OUT/pass.log; exit 1; }
python3 tools/ws_sq_summary.py --pmc /tmp/ws_sq --out $OUT/sq_wait_states_ws.csv
