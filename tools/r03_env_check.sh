#!/bin/bash
# Env-kernel change check: the env / RL GPU parity tests, then k_step timing (bench headline +
# 9x9 point) and the placement phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_env_gpu.py tests/test_rl_gpu.py \
  tests/test_eval.py > gpurun_out/env_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/env_tests.txt; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-multistep --ppo-updates 0 \
    --extras 9x9x10:8192,30x16x99:8192 > gpurun_out/envchk.log 2>&1 || { tail -5 gpurun_out/envchk.log; exit 1; }
  python3 - <<'PY'
import json
d = json.loads([x for x in open("gpurun_out/envchk.log") if x.startswith("{")][-1])
print("16x16@4096 k_step", round(d["roofline"]["kernel_ms"] * 1e3, 2), "us frac", round(d["roofline"]["frac"], 3),
      "value", round(d["value"] / 1e6, 1), "M", *[f"| {p['board']}@{p['envs_per_gpu']} k_step {p['roofline']['kernel_ms']*1e3:.2f} us frac {p['roofline']['frac']:.3f} value {p['value']/1e6:.1f} M" for p in d["north_star_points"]])
PY
done
timeout -k 10 120 python3 -u tools/diag_step.py --board 9x9x10 --envs 8192 --steps 20 2>&1 | grep -v amdgpu | head -16
