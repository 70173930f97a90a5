#!/bin/bash
# Kernel trace of bench.py's combined PPO update loop (rollout + GAE + 3x8 minibatches,
# N=4096, T=64): where a whole update's GPU time goes, next to its wall time.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pu -o p --output-format csv -- python3 bench.py --no-cpu-baseline --extras= --no-multistep --steps 20 --warmup 5 --ppo-updates 2 > gpurun_out/ppo_update_prof.log 2>&1 || { tail -5 gpurun_out/ppo_update_prof.log; exit 1; }
grep "^{" gpurun_out/ppo_update_prof.log | tail -1 > gpurun_out/ppo_update_prof.json
cp $(find /tmp/pu -name "*kernel_stats.csv") gpurun_out/ppo_update_kernel_stats.csv
python3 - <<'PY'
import csv, json
l = json.load(open("gpurun_out/ppo_update_prof.json"))["ppo"]
print("s/update", l["s_per_update"], "rollout", l["rollout_s"], "ppo", l["ppo_s"])
rows = list(csv.DictReader(open("gpurun_out/ppo_update_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel total s", tot / 1e9)
for r in rows[:25]:
    print(f"{r['Name'][:80]:80s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5s} {float(r['Percentage']):5.1f}%")
PY
