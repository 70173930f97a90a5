"""Where a rollout's time goes (bench configuration: 16x16x40 medium, 4096 envs x 64 steps, fp16,
u8-code buffer): wall time of collect_rollout against the host-side enqueue time it reports.
Run under rocprofv3 --kernel-trace --stats to get the kernels' total. python tools/rollout_prof.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402
from ms_amd.rollout import collect_rollout  # noqa: E402
from ms_amd.train import Trainer, load_config  # noqa: E402

dev = torch.device("cuda:0")
cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
cfg.num_envs, cfg.steps_per_env = 4096, 64
tr = Trainer(cfg, env_d, model_d, extras, seed=0, amp="fp16", device=dev)
tr.model.train()
buf = None
for it in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    buf, aux = collect_rollout(tr.vec, tr.model, 64, dev, 0.05, 0.0, amp_dtype=torch.float16, buffer=buf,
                               sample_seed=1, sample_counter=it << 20, obs_codes=True)
    enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"rollout {it}: wall {wall * 1e3:.1f} ms, host enqueue {enq * 1e3:.1f} ms", flush=True)
