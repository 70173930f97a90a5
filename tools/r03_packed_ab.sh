#!/bin/bash
# k_step_packed (four small boards per wave) vs k_step (MS_DBG_ONE_BOARD_PER_WAVE) on the same
# box: the env parity tests first, then the 9x9x10 @ 8192 and 8x8x10 points, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/packed_tests.log 2>&1 || { tail -30 gpurun_out/packed_tests.log; exit 1; }
tail -2 gpurun_out/packed_tests.log
for rep in 1 2; do
  for fl in 0 4 8; do
    timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --ppo-updates 0 \
      --board 9x9x10 --envs 8192 --extras 8x8x10:8192,9x9x10:32768 --env-debug-flags $fl \
      > gpurun_out/packed_ab_$fl.log 2>&1 || { tail -5 gpurun_out/packed_ab_$fl.log; exit 1; }
    python3 - "$fl" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/packed_ab_{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
name = {"0": "packed4", "4": "one-per-wave", "8": "packed2"}[sys.argv[1]]
pts = [d] + d["north_star_points"]
print(name, " | ".join(f'{p.get("board", d["config"].get("board"))}@{p.get("envs_per_gpu", d["config"].get("envs_per_gpu"))} '
                       f'{p["roofline"]["kernel_ms"]*1e3:.2f} us frac {p["roofline"]["frac"]:.3f} value {p["value"]/1e6:.0f}M'
                       for p in pts))
PY
  done
done
