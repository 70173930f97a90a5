#!/bin/bash
# k_step A/B: the product library vs tools/bin/noplace (a fixed mine pattern instead of the
# placement; timing only) at the headline and the 9x9 point, alternated twice. The noplace build
# hook was removed after the measurement; this script stays as the record of how
# profiles/r03/k_step_noplacement_ab.txt was made.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in prod noplace; do
    lib=""; [ $v != prod ] && lib=$PWD/tools/bin/$v/libmsenv.so
    MSENV_LIB=$lib timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-multistep \
      --ppo-updates 0 --extras 9x9x10:8192 > gpurun_out/stepab_$v.log 2>&1 || { tail -5 gpurun_out/stepab_$v.log; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/stepab_{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
p = d["north_star_points"][0]
print(sys.argv[1], "16x16@4096 k_step", round(d["roofline"]["kernel_ms"] * 1e3, 2), "us frac", round(d["roofline"]["frac"], 3),
      "| 9x9@8192 k_step", round(p["roofline"]["kernel_ms"] * 1e3, 2), "us frac", round(p["roofline"]["frac"], 3))
PY
  done
done
