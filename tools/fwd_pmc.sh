#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the layer kernels at the
# PPO minibatch size, per forward variant (MC_FWD_RW=0/1).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rw in ${RWS:-0 1}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MC_FWD_RW=$rw timeout -s KILL 90 rocprofv3 --pmc $c -d /tmp/pmc_${rw}_$c -o p --output-format csv -- \
      python3 tools/fused_micro.py --no-torch --bwd --iters 2 > /tmp/pmc_${rw}_$c.log 2>&1 || { tail -3 /tmp/pmc_${rw}_$c.log; exit 1; }
  done
  python3 - $rw <<'PY'
import csv, glob, sys
from collections import defaultdict
rw = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = defaultdict(list)
    for f in glob.glob(f"/tmp/pmc_{rw}_{c}/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == c:
                acc[(r["Kernel_Name"], r.get("Dispatch_Id"))] += float(r["Counter_Value"])
        for (k, d), v in acc.items():
            per[k].append(v)
    for k, v in sorted(per.items()):
        if any(s in k for s in ("k_conv", "k_bwd_data", "k_wgrad", "k_reduce")):
            print(f"rw={rw} {c:10s} {k[:60]:60s} {sum(v)/len(v)/1024/1024:9.3f} GB/launch")
PY
done
