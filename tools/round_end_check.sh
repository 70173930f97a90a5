#!/bin/bash
# What the driver runs at round end, in the same order: the GPU test suite, smoke(), and the
# default bench.py line (each under its own time limit; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -5 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
grep "^{" gpurun_out/bench_default.log | tail -1 > gpurun_out/bench_default.json
python3 - <<'PY'
import json
l = json.load(open("gpurun_out/bench_default.json"))
print("value", l["value"], l["unit"], "frac", round(l["roofline"]["frac"], 3), "cpu", l["cpu_baseline"]["value"],
      "gpu/cpu", round(l.get("gpu_over_cpu", 0), 1))
ppo = l.get("ppo") or {}
print("ppo", ppo.get("updates_per_s"), ppo.get("amp"), "multistep", (l.get("multistep") or {}).get("value"))
PY
