#!/bin/bash
# C3 (9x9x10, 8,192 envs, one GPU) env-step A/B over the boards-per-wave layouts: MS_DBG flags
# 0 (k_step_packed, 4 boards a wave), 8 (2 boards a wave), 4 (k_step, one board a wave)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2; do
  for f in 0 8 4; do
    timeout -k 10 200 python3 -u bench.py --board 9x9x10 --envs 8192 --extras= --ppo-updates 0 --no-cpu-baseline \
      --no-multistep --env-debug-flags $f > gpurun_out/c3_$f.log 2>&1 || { tail -5 gpurun_out/c3_$f.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/c3_$f.log') if l.startswith('{')][-1])
r=d.get('roofline',{})
print('flags $f rep $rep: %.4g %s, ms/step %.5f, kernel frac %.3f (%s)'%(d['value'],d['unit'],d['ms_per_step'],r.get('frac',0),r.get('kernel','')))
"
  done
done
