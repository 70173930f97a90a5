#!/bin/bash
# Round 3 check: the tests this round added first (production-size fused kernels, the Trainer's
# fp16 update at 4096 envs, keyed dropout, the data-parallel fp16 / overflow cases), then the
# rest of the GPU suite, then the bench line as the driver runs it (--steps 20 --warmup 5) and
# with its defaults. Each step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_trainer_prod_gpu.py tests/test_dist_trainer_gpu.py tests/test_fused_gpu.py \
  > gpurun_out/r03_new_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r03_new_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 $T -q -m gpu tests --deselect tests/test_fused_gpu.py --ignore tests/test_trainer_prod_gpu.py \
  --ignore tests/test_dist_trainer_gpu.py > gpurun_out/r03_rest_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r03_rest_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -5 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_s20.log 2>&1 || { tail -5 gpurun_out/bench_s20.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
for f in bench_s20 bench_default; do grep "^{" gpurun_out/$f.log | tail -1 > gpurun_out/$f.json; done
python3 - <<'PY'
import json
for f in ("bench_s20", "bench_default"):
    l = json.load(open(f"gpurun_out/{f}.json"))
    print(f, "value", round(l["value"] / 1e6, 1), "M frac", round(l["roofline"]["frac"], 3), "cpu",
          round(l["cpu_baseline"]["value"] / 1e6, 2), "M gpu/cpu", round(l.get("gpu_over_cpu", 0), 1),
          "ppo", round((l.get("ppo") or {}).get("updates_per_s", 0), 3))
    for p in l.get("north_star_points", []):
        print("  ", p["board"], p["envs_per_gpu"], round(p["value"] / 1e6, 1), "M frac", round(p["roofline"]["frac"], 3),
              "gpu/cpu", round(p.get("gpu_over_cpu", 0), 1))
PY
