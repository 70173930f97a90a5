#!/bin/bash
# Stagger sweep for the persistent layer kernels: per-kernel average durations
# (rocprofv3 --kernel-trace --stats) of one fused layer fwd + bwd at the PPO
# minibatch size, for start delays MC_{FWD,BWD,WG}_STAGGER (10-ns ticks).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/stagger.txt
: > $OUT
for v in ${VARIANTS:-"0 0 0" "1800 2250 400" "-1800 -2250 -400" "900 1100 200" "3000 3500 800"}; do
  set -- $v
  d=/tmp/stg_$1_$2_$3
  MC_FWD_STAGGER=$1 MC_BWD_STAGGER=$2 MC_WG_STAGGER=$3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o s \
    --output-format csv -- python3 tools/fused_micro.py --no-torch --bwd --iters 5 > $d.log 2>&1 || { echo "fail $v"; tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv")
  python3 - "$f" "$v" >> $OUT <<'PY'
import csv, sys
rows = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(sys.argv[1]))}
pick = lambda key: next((v for k, v in rows.items() if key in k), float("nan"))
print(f"stagger {sys.argv[2]:>18}: fwd {pick('k_conv_gn_fwd<96')/1e3:8.1f} us  bwd_data {pick('k_bwd_data<2, true')/1e3:8.1f} us  wgrad {pick('k_wgrad<96')/1e3:8.1f} us")
PY
done
cat $OUT
