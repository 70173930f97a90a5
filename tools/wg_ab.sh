#!/bin/bash
# Same-box A/B of one trunk-kernel toggle: kernel trace of tools/ppo_micro.py with VAR=0 and VAR=1.
# usage: VAR=MC_WG_PF bash tools/wg_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0 1; do
  rm -rf /tmp/ab
  env $VAR=$v true
  export $VAR=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ab -o p --output-format csv -- python3 tools/ppo_micro.py --mb 32768 --iters 3 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "== $VAR=$v: $(grep 'ms/iter' gpurun_out/ab_$v.log)"
  python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("/tmp/ab/**/*kernel_stats.csv", recursive=True)[0])))
for r in rows[:6]:
    print(f"   {r['Name'][:64]:64s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4s}")
PY
done
