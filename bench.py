"""Benchmark: env steps/sec of the HIP board step on BASELINE.json's config
(16x16x40, N=4096 envs per GPU; weak scaling over ranks), with the dominant
kernel's HBM roofline fraction and the CPU restatement timed on this host.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

A step = one synthetic-policy action pass (ms_tape_actions) + one board step
(ms_step, all outputs: obs, mask, reward, done, aux) over every env of the
rank. Inputs are resident in HBM; the timed region is bracketed by a barrier
and torch.cuda.synchronize() on both sides; the MAX over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec


def algo_bytes_per_env_step(H: int, W: int) -> int:
    """obs 40HW + mask HW + action 8 + reward 4 + done 1 + aux 12
    + packed board state read+write 2*(2*ceil(HW/8) + 32) + PCG inc read 16."""
    A = H * W
    return 40 * A + A + 8 + 4 + 1 + 12 + 2 * (2 * ((A + 7) // 8) + 32) + 16


def pmc_traffic(H, W, K, n, kernel="k_step"):
    """HBM bytes per env step of all n envs (k_step: one launch; k_run: a launch / its
    steps) from the committed rocprofv3 PMC passes (FETCH_SIZE + WRITE_SIZE, separate
    passes; tools/profile_round.sh) of the latest round under profiles/, for this exact
    board and env count."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{kernel}_{H}x{W}x{K}_{n}.json")))
    if not cands:
        return None, None
    with open(cands[-1]) as f:
        d = json.load(f)
    per_step = d.get("traffic_bytes_per_step", d["traffic_bytes_per_launch"])
    return per_step, os.path.relpath(cands[-1], ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--board", default="16x16x40")
    ap.add_argument("--tape", type=int, default=0, help="0 uniform-valid, 1 safe-biased")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline sample budget of the headline point (each extra point: half)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-multistep", action="store_true", help="skip the one-launch ms_run_tape line")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the CPUs this process may use: min(affinity mask, cgroup quota)")
    ap.add_argument("--extras", default="16x16x40:32768,9x9x10:8192@total,30x16x99:8192@total",
                    help="north-star points measured after the headline: board:envs per GPU, or board:envs@total "
                         "for a GLOBAL env count split over the ranks (C3 / C5 are 8192 envs in all); '' disables")
    ap.add_argument("--min-timed-steps", type=int, default=1000,
                    help="the captured K-step graph is replayed until at least this many steps are timed "
                         "(SURVEY.md §8d: >= 1,000 timed steps)")
    ap.add_argument("--diag-no-obs", action="store_true", help="diagnostic: skip obs/mask outputs")
    ap.add_argument("--env-debug-flags", type=int, default=0,
                    help="diagnostic A/B only: msenv_debug.h MS_DBG_* flags of the env handles (4: no lane packing)")
    ap.add_argument("--graph", type=int, default=1, help="capture the timed steps in a HIP graph")
    ap.add_argument("--ppo-updates", type=int, default=6,
                    help="timed combined rollout+GAE+PPO updates (0 disables; +1 untimed warm-up)")
    ap.add_argument("--ppo-steps-per-env", type=int, default=64)
    ap.add_argument("--amp", default="fp16", choices=["bf16", "fp16", "fp32"],
                    help="PPO autocast type (fp16 + GradScaler = the reference's training precision)")
    return ap.parse_args()


def _cgroup_cpu_quota():
    """CPUs granted by the cgroup (cpu.max quota / period), or None when unlimited/unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def effective_cpus():
    """CPUs this process can actually use: min(affinity mask, cgroup CPU quota)."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpu_quota()
    return max(1, min(aff, int(-(-quota // 1)))) if quota else aff


# The reference's own env step (env.py VecMinesweeper.step, pure-Python BFS: numba is not in the
# image), 1 core, measured in the survey container (BASELINE.md:27-32). It cannot
# run on the GPU box (the reference does not travel), so the ratio uses these figures.
REF_PY_1CORE = {"16x16x40": (6980.0, "16x16x40 N=4096"), "9x9x10": (8338.0, "9x9x10 N=8192"),
                "16x30x99": (8423.0, "16x30x99 N=1024"),
                "30x16x99": (8423.0, "16x30x99 N=1024 (the same Expert board, transposed)")}


def ref_python_ratio(board, value):
    ref = REF_PY_1CORE.get(board)
    if ref is None:
        return None
    return {"value": value / ref[0], "ref_env_steps_per_s": ref[0], "ref_config": ref[1],
            "source": "BASELINE.md:27-32 (reference env.py step, 1 core, Python BFS, survey container)"}


def cpu_baseline(H, W, K, n_envs, seed, tape, budget_s, threads):
    """Oracle (CPU restatement of env.py / env_numba, C + pthreads) timed on this host over a
    bounded sample: each thread owns a block of envs and runs tape action + board step for
    all of them, step after step, without synchronising (one env per task). ``threads`` =
    the CPUs the process may use (effective_cpus), so ``cores`` is what the sample ran on."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    v = O.OracleVec(H, W, K, n_envs, seed=seed)
    v.reset()
    A = H * W
    bufs = (np.zeros((n_envs, 10, H, W), np.float32), np.zeros((n_envs, A), np.uint8),
            np.zeros(n_envs, np.float32), np.zeros(n_envs, np.uint8), np.zeros(n_envs, np.int32),
            np.zeros(n_envs, np.int32), np.zeros(n_envs, np.float64), np.zeros(n_envs, np.int8))
    v.run_baseline(0, 5, tape, threads, bufs)  # warm-up: page in, first clicks
    t0 = time.perf_counter()
    v.run_baseline(5, 5, tape, threads, bufs)  # calibrate
    per_step = (time.perf_counter() - t0) / 5
    steps = int(max(3, min(200000, budget_s / max(per_step, 1e-9))))
    t0 = time.perf_counter()
    v.run_baseline(10, steps, tape, threads, bufs)
    el = time.perf_counter() - t0
    quota = _cgroup_cpu_quota()
    return dict(value=n_envs * steps / el, unit="env_steps/s", cores=threads, kind="port",
                nproc=os.cpu_count(), affinity_cpus=len(os.sched_getaffinity(0)), cgroup_cpu_quota=quota,
                sample=f"{steps} steps x {n_envs} envs {H}x{W}x{K} (tape {tape}) in {el:.1f}s, "
                       f"oracle/ms_oracle.c mso_run_baseline on {threads} threads = min(affinity mask "
                       f"{len(os.sched_getaffinity(0))}, cgroup quota "
                       f"{'none' if quota is None else f'{quota:g} CPUs'}); nproc {os.cpu_count()}")


class DispatchTimer:
    """Pairs of HIP events stamped by the kernel dispatch itself (ms_set_timing_events ->
    hipExtLaunchKernel): elapsed = the kernel's execution time as rocprofv3 traces it."""

    def __init__(self, lib, L, h, n):
        import ctypes
        self.lib, self.L, self.h = lib, L, h
        self.ev = []
        for _ in range(n):
            pair = []
            for _ in range(2):
                e = ctypes.c_void_p()
                L.check(lib.ms_event_create(ctypes.byref(e)))
                pair.append(e.value)
            self.ev.append(pair)

    def arm(self, i):
        self.L.check(self.lib.ms_set_timing_events(self.h, self.ev[i][0], self.ev[i][1]))

    def disarm(self):
        self.L.check(self.lib.ms_set_timing_events(self.h, None, None))

    def elapsed_ms(self, i):
        import ctypes
        ms = ctypes.c_float()
        self.L.check(self.lib.ms_event_elapsed_ms(self.ev[i][0], self.ev[i][1], ctypes.byref(ms)))
        return ms.value

    def close(self):
        self.disarm()
        for pair in self.ev:
            for e in pair:
                self.lib.ms_event_destroy(e)


def multistep_bench(args, world, lib, h, L, n_local, n_total, H, W, bpe, dev):
    """ms_run_tape: the same synthetic tape + board step, S steps per launch (boards held
    in registers between steps), every step's outputs in their own slot as in a rollout
    buffer. Launch durations summed / K is its per-step kernel time."""
    A = H * W
    # every step writes its own slot (slots=1) of an S-step region holding > 1 GiB, so the
    # stores stream to HBM rather than into the 256 MiB Infinity Cache; K steps = ceil(K/S)
    # launches of S steps (the last one shorter)
    total = max(args.steps, args.min_timed_steps)
    S = max(1, min(total, -(-(1 << 30) // (n_local * 41 * A))))
    bufs = [torch.empty((S, n_local, 10, H, W), dtype=torch.float32, device=dev),
            torch.empty((S, n_local, A), dtype=torch.bool, device=dev),
            torch.empty((S, n_local), dtype=torch.float32, device=dev),
            torch.empty((S, n_local), dtype=torch.bool, device=dev),
            torch.empty((S, n_local), dtype=torch.int32, device=dev),
            torch.empty((S, n_local), dtype=torch.int32, device=dev),
            torch.empty((S, n_local), dtype=torch.float64, device=dev),
            torch.empty((S, n_local), dtype=torch.int8, device=dev)]
    ptrs = [L.ptr(b) for b in bufs]
    sp = torch.cuda.current_stream(dev).cuda_stream
    t_base = 1 << 24  # tape indices past those of the per-step measurement
    # warm-up: one full S-step launch (so every profiled k_run dispatch but the last is S steps)
    L.check(lib.ms_run_tape(h, t_base, S, args.tape, 1, None, *ptrs, sp))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    n_launch = -(-total // S)
    timer = DispatchTimer(lib, L, h, n_launch)
    t0 = time.perf_counter()
    done_steps = 0
    i = 0
    while done_steps < total:
        T = min(S, total - done_steps)
        timer.arm(i)
        L.check(lib.ms_run_tape(h, t_base + S + done_steps, T, args.tape, 1, None, *ptrs, sp))
        done_steps += T
        i += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = sum(timer.elapsed_ms(j) for j in range(n_launch)) / total
    timer.close()
    if world > 1:
        t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms = float(t[0]), float(t[1])
    achieved = bpe * n_local / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(H, W, args.board_k, n_local, "k_run")
    return {"metric": "env steps/sec, S synthetic-policy steps per launch (ms_run_tape)",
            "value": n_total * total / el, "unit": "env_steps/s", "ms_per_step": el / total * 1e3,
            "timed_steps": total,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes per step",
                         "traffic_source": traffic_src, "kernel": "k_run",
                         "kernel_ms_per_step": kern_ms, "steps_per_launch": S,
                         "kernel_ms_method": "dispatch-stamped HIP events (hipExtLaunchKernel) of each "
                                             "S-step launch, summed / K"}}


# fwd / fwd+bwd GFLOP per 16x16 sample of the shipped model (torch flop counter)
GFLOP_FWD_16, GFLOP_FWDBWD_16 = 0.4388, 1.3073
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 / fp16


def ppo_kernel_profile():
    """The PPO minibatch's trunk kernels at N = 32,768 from the committed rocprofv3 passes
    (tools/profile_round.sh step 3 -> profiles/r*/pmc_ppo_minibatch_32768.json): mean
    launch time, HBM bytes per launch (FETCH_SIZE doubled for 16-B/lane streams + WRITE_SIZE),
    MFMA-busy fraction and TFLOP/s on the 2*N*P*96*96*9 algorithmic flops of a 96->96 layer."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_ppo_minibatch_32768.json")))
    if not cands:
        return None
    d = json.load(open(cands[-1]))
    out = {"source": os.path.relpath(cands[-1], ROOT)}
    for name, k in d["kernels"].items():
        short = name.split("(anonymous namespace)::", 1)[-1].split("((anonymous")[0]
        if short in out or "achieved_TFLOPs" not in k:
            continue
        out[short] = {"mean_us": k["mean_us"], "traffic_bytes_per_launch": k["traffic_bytes"],
                      "hbm_frac": k["traffic_bytes"] / (k["mean_us"] * 1e-6) / (HBM_PEAK_GBS * 1e9),
                      "mfma_busy": k.get("mfma_busy_frac"), "achieved_TFLOPs": k["achieved_TFLOPs"],
                      "mfma_frac": k["mfma_frac_of_2500"]}
    return out


def ppo_bench(args, world, rank, local_rank, dev):
    """Combined rollout + GAE + PPO-update loop (BASELINE metric, 2nd half):
    configs/16x16x40_medium.yaml with num_envs = envs_per_gpu * world (global),
    T = 64, 3 epochs x 8 minibatches, flat-gradient RCCL all-reduce per minibatch."""
    from ms_amd.dist import DistInfo
    from ms_amd.train import Trainer, load_config
    cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
    cfg.num_envs = args.envs * world
    cfg.steps_per_env = args.ppo_steps_per_env
    cfg.total_updates = 4000
    info = DistInfo(rank=rank, world=world, local_rank=local_rank,
                    group=dist.group.WORLD if world > 1 else None)
    tr = Trainer(cfg, env_d, model_d, extras, seed=args.seed, info=info, amp=args.amp, device=dev)
    tr.update(0)  # warm-up: MIOpen kernel selection, allocator
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    prof, per_update = [], []
    for u in range(args.ppo_updates):
        tu = time.perf_counter()
        prof.append(tr.update(1 + u, profile=True))
        torch.cuda.synchronize()  # per-update wall time (the update ends in host reads anyway)
        per_update.append(time.perf_counter() - tu)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el] + per_update, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, per_update = float(t[0]), [float(v) for v in t[1:]]
    spu = el / args.ppo_updates
    med = float(np.median(per_update))
    n_mb = cfg.ppo_epochs * cfg.mini_batches
    comm = {"allreduce": None, "note": "world 1: no collective"}
    if world > 1:
        # the per-minibatch RCCL all-reduce of the flat fp32 gradient bucket (FlatGrads), timed
        # alone: barrier, 5 warm-up calls, then 20 calls between two synchronisations; max over ranks
        flat = tr.flat
        for _ in range(5):
            flat.all_reduce_mean(info.group)
        torch.cuda.synchronize()
        dist.barrier()
        ta = time.perf_counter()
        for _ in range(20):
            flat.all_reduce_mean(info.group)
        torch.cuda.synchronize()
        ar_s = (time.perf_counter() - ta) / 20
        t = torch.tensor([ar_s], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ar_s = float(t[0])
        comm = {"allreduce_ms_per_minibatch": ar_s * 1e3, "bytes": flat.flat.numel() * 4,
                "allreduces_per_update": n_mb, "bus_GBps": 2 * (world - 1) / world * flat.flat.numel() * 4 / ar_s / 1e9,
                "share_of_update": n_mb * ar_s / spu, "backend": dist.get_backend()}
    n_loc, T = args.envs, cfg.steps_per_env
    gflop = (T * n_loc * GFLOP_FWD_16 + n_loc * GFLOP_FWD_16 + cfg.ppo_epochs * T * n_loc * GFLOP_FWDBWD_16)
    mean = lambda k: float(np.mean([p[k] for p in prof]))  # noqa: E731
    kprof = ppo_kernel_profile()
    dom = max((k for k in (kprof or {}) if k != "source"), key=lambda k: kprof[k]["mean_us"], default=None)
    return {"metric": "PPO updates/sec (combined rollout + GAE + 3x8 minibatch update)",
            "updates_per_s": 1.0 / spu, "s_per_update": spu,
            # the spread over the timed updates (each timed alone, max over ranks), so that a change of
            # a few per cent can be told from box-to-box noise
            "updates": args.ppo_updates, "s_per_update_median": med,
            "s_per_update_spread": (max(per_update) - min(per_update)) / med,
            "s_per_update_each": [round(v, 4) for v in per_update],
            "samples_per_s": n_loc * world * T / spu, "envs_total": n_loc * world, "steps_per_env": T,
            "rollout_s": mean("rollout_s"), "gae_s": mean("gae_s"), "ppo_s": mean("ppo_s"),
            # the reference's rollout timing buckets (train_rl.py:278-288), GPU time per update
            "rollout_buckets_s": {k[len("rollout_"):]: mean(k) for k in sorted(prof[-1]) if k.startswith("rollout_")
                                  and k.endswith("_total_s")},
            "amp": args.amp, "rollout_buffer_obs": "u8 cell codes" if tr.obs_codes else "f32 one-hot",
            "model": "cnn_residual 96ch x 5 blocks (950,947 params)",
            "roofline": {"bound": "mfma", "achieved": gflop / spu / 1e3, "peak": BF16_DENSE_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": gflop / spu / 1e3 / BF16_DENSE_PEAK_TFLOPS,
                         "traffic": kprof[dom]["traffic_bytes_per_launch"] if dom else None,
                         "traffic_kernel": dom, "traffic_unit": "HBM bytes per launch at N=32768",
                         "algo_gflop_per_update_per_gpu": gflop, "trunk_kernels": kprof},
            "comm": comm, "loss": prof[-1].get("loss"), "entropy": prof[-1].get("entropy")}


def env_bench(args, world, rank, dev, H, W, K, n_local, multistep=True):
    """Env-step measurement of one board / env count: K graph-replayed (tape + step) steps, the
    k_step roofline, and (optionally) the multistep ms_run_tape line."""
    from ms_amd import EnvConfig, VecMinesweeper
    from ms_amd import _lib as L

    n_total = n_local * world
    vec = VecMinesweeper(n_total, EnvConfig(H=H, W=W, mine_count=K), seed=args.seed, device=dev,
                         shard=(rank, world))
    assert vec.num_envs == n_local
    if args.env_debug_flags:
        vec.set_debug_flags(args.env_debug_flags)
    A = H * W
    # obs/mask go to a ring of R slots holding > 512 MiB (2x the 256 MiB Infinity Cache), as a
    # rollout buffer would: a single re-written 44 MB buffer stays cache-resident and its
    # stores never reach HBM, which would flatter the HBM roofline
    R = max(1, -(-(512 << 20) // (n_local * 41 * A)))
    obs_ring = torch.empty((R, n_local, 10, H, W), dtype=torch.float32, device=dev)
    mask_ring = torch.empty((R, n_local, A), dtype=torch.bool, device=dev)
    obs, mask = obs_ring[0], mask_ring[0]
    rew = torch.empty(n_local, dtype=torch.float32, device=dev)
    done = torch.empty(n_local, dtype=torch.bool, device=dev)
    step_i = torch.empty(n_local, dtype=torch.int32, device=dev)
    lnew = torch.empty(n_local, dtype=torch.int32, device=dev)
    frac = torch.empty(n_local, dtype=torch.float64, device=dev)
    outc = torch.empty(n_local, dtype=torch.int8, device=dev)
    act = torch.empty(n_local, dtype=torch.int64, device=dev)
    lib, h = vec._lib, vec._h
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    ptrs = [L.ptr(x) for x in (act, obs, mask, rew, done, step_i, lnew, frac, outc)]
    if args.diag_no_obs:
        ptrs[1] = ptrs[2] = None

    def one_step(t, sp, ev=None):
        L.check(lib.ms_tape_actions(h, t, args.tape, ptrs[0], sp))
        if ev is not None:
            ev[0].record()
        pt = list(ptrs)
        if not args.diag_no_obs:
            pt[1], pt[2] = L.ptr(obs_ring[t % R]), L.ptr(mask_ring[t % R])
        L.check(lib.ms_step(h, *pt, sp))
        if ev is not None:
            ev[1].record()

    vec.reset(out={"obs": obs, "action_mask": mask})
    for t in range(args.warmup):
        one_step(t, stream.cuda_stream)
    torch.cuda.synchronize()

    # Timed region: the K steps (2K kernel launches) are captured once into a
    # HIP graph and replayed, so host launch cost is off the critical path.
    def capture(tape_only: bool):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cs = torch.cuda.current_stream().cuda_stream
            for k in range(args.steps):
                if tape_only:
                    L.check(lib.ms_tape_actions(h, args.warmup + k, args.tape, ptrs[0], cs))
                else:
                    one_step(args.warmup + k, cs)
        torch.cuda.synchronize()
        return g  # capture does not execute: the board state is still at step `warmup`

    graph = capture(False) if args.graph else None
    # the K-step graph is replayed back to back until >= min_timed_steps steps are timed, so a
    # short --steps does not leave the one host-side graph launch as a visible share of the span
    reps = max(1, -(-args.min_timed_steps // args.steps))
    timed = args.steps * reps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(reps):
            graph.replay()
    else:
        for k in range(timed):
            one_step(args.warmup + k % args.steps, sp)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # Dominant-kernel duration (kernel_ms): the span of a replay of the K-step graph minus
    # the span of a graph holding only its K tape launches, / K = what one ms_step adds to a
    # step, launch boundary included. Cross-check (kernel_ms_isolated): Km eager ms_step
    # launches, each run alone (the host waits for its tape launch first: stamped back to
    # back, the start stamp would be taken while k_tape still runs) with dispatch-stamped
    # events (ms_set_timing_events -> hipExtLaunchKernel). Untraced, the isolated figure reads
    # 1-15 % above the span (each isolated launch starts on an idle GPU); under rocprofv3 both absorb the profiler's per-dispatch overhead on these
    # ~10-us launches, so tools/trace_check.py's trace fraction is the one to quote there.
    Km = min(timed, 200)
    timer = DispatchTimer(lib, L, h, Km)
    t_iso = args.warmup + 2 * args.steps
    for k in range(Km):
        t = t_iso + k
        L.check(lib.ms_tape_actions(h, t, args.tape, ptrs[0], sp))
        torch.cuda.synchronize()
        pt = list(ptrs)
        if not args.diag_no_obs:
            pt[1], pt[2] = L.ptr(obs_ring[t % R]), L.ptr(mask_ring[t % R])
        timer.arm(k)
        L.check(lib.ms_step(h, *pt, sp))
    timer.disarm()
    torch.cuda.synchronize()
    iso_ms = float(np.mean([timer.elapsed_ms(k) for k in range(Km)]))
    timer.close()
    if graph is not None:
        gt = capture(True)
        ev_full = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev_tape = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        # the step graph is replayed once more for the span: the boards move on, the work per
        # step is statistically the same
        ev_full[0].record()
        for _ in range(reps):
            graph.replay()
        ev_full[1].record()
        ev_tape[0].record()
        for _ in range(reps):
            gt.replay()
        ev_tape[1].record()
        torch.cuda.synchronize()
        kern_ms = (ev_full[0].elapsed_time(ev_full[1]) - ev_tape[0].elapsed_time(ev_tape[1])) / timed
        kern_method = "graph span difference (tape+step vs tape only, each K-step graph replayed R times) / (K*R)"
        del gt
    else:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        for k in range(args.steps):
            one_step(args.warmup + args.steps + k, sp, evs[k])
        torch.cuda.synchronize()
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        kern_method = "events around each ms_step (eager)"
    del graph
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, iso_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, iso_ms = float(t[0]), float(t[1]), float(t[2])
    iso_method = (f"dispatch-stamped HIP events (hipExtLaunchKernel) of {Km} eager ms_step launches, "
                  "each started after its tape launch completed; mean")

    traffic, traffic_src = pmc_traffic(H, W, K, n_local)
    bpe = algo_bytes_per_env_step(H, W)
    achieved = bpe * n_local / (kern_ms * 1e-3) / 1e9
    res = {"board": f"{H}x{W}x{K}", "envs_per_gpu": n_local, "envs_total": n_total,
           "value": n_total * timed / elapsed, "unit": "env_steps/s",
           "ms_per_step": elapsed / timed * 1e3, "timed_steps": timed, "graph_replays": reps,
           "obs_ring_slots": R,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "kernel": "k_step", "kernel_ms": kern_ms, "kernel_ms_method": kern_method,
                        "kernel_ms_isolated": iso_ms, "isolated_method": iso_method,
                        "algo_bytes_per_env_step": bpe,
                        "algo_bytes_per_launch": bpe * n_local, "traffic_source": traffic_src}}
    if multistep and not args.diag_no_obs:
        args.board_k = K
        res["multistep"] = multistep_bench(args, world, lib, h, L, n_local, n_total, H, W, bpe, dev)
    del vec, obs_ring, mask_ring
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    H, W, K = (int(x) for x in args.board.lower().split("x"))
    args.board_k = K
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MS_BENCH_BACKEND=gloo with ranks sharing the visible GPUs rehearses the N>1 path
    # (barriers, max-over-ranks timing, the Trainer's flat-gradient all-reduce) on a
    # one-GPU box; the driver's multi-GPU runs use the default, RCCL with one GPU per rank.
    backend = os.environ.get("MS_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    n_local = args.envs
    head = env_bench(args, world, rank, dev, H, W, K, n_local, multistep=not args.no_multistep)
    cpu_on = rank == 0 and world == 1 and not args.no_cpu_baseline
    threads = args.cpu_threads or effective_cpus()

    def add_cpu(point, h_, w_, k_, n_, budget):
        """cpu_baseline + ratios of one measured point (rank 0, N=1 only)."""
        if not cpu_on:
            return
        cb = cpu_baseline(h_, w_, k_, n_, args.seed, args.tape, budget, threads)
        point["cpu_baseline"] = cb
        point["gpu_over_cpu"] = point["value"] / cb["value"]
        point["gpu_over_ref_python_1core"] = ref_python_ratio(f"{h_}x{w_}x{k_}", point["value"])
    out = {
        "metric": "env steps/sec (16x16x40, N envs) + PPO updates/sec at 1/2/4/8 MI355X",
        "value": head["value"],
        "unit": "env_steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "timed_steps": head["timed_steps"],
        "graph_replays": head["graph_replays"],
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64 board bits -> f32 obs",
        "data": "synthetic: numpy-seeded boards, splitmix64 action tape (SURVEY.md §8d)",
        "config": {"workload": f"board step {H}x{W}x{K}, {n_local} envs per GPU (BASELINE configs[1]"
                               f"{', configs[3] at 8 GPUs' if world == 8 else ''})",
                   "board": f"{H}x{W}x{K}", "envs_per_gpu": n_local, "envs_total": n_local * world,
                   "tape": args.tape, "parallelism": f"env-shard x{world}, no collective",
                   "obs_ring_slots": head["obs_ring_slots"]},
        "roofline": head["roofline"],
    }
    if "multistep" in head:
        out["multistep"] = head["multistep"]
    pts = []
    if args.extras and not args.diag_no_obs:
        for item in args.extras.split(","):
            b, n = item.split(":")
            h_, w_, k_ = (int(x) for x in b.lower().split("x"))
            if n.endswith("@total"):  # a GLOBAL env count, split over the ranks
                n_tot = int(n[:-len("@total")])
                if n_tot % world:
                    raise SystemExit(f"--extras {item}: {n_tot} envs do not split over {world} ranks")
                n_pg = n_tot // world
            else:
                n_pg = int(n)
            r = env_bench(args, world, rank, dev, h_, w_, k_, n_pg, multistep=not args.no_multistep)
            pts.append((r, h_, w_, k_, n_pg))
        out["north_star_points"] = [r for r, *_ in pts]
    if args.ppo_updates > 0:
        out["ppo"] = ppo_bench(args, world, rank, local_rank, dev)
    # CPU baselines last, after every GPU measurement: rank 0 at N=1, a bounded sample per point
    add_cpu(out, H, W, K, n_local, args.cpu_seconds)
    if cpu_on:
        out["gpu_over_cpu_target"] = 50.0
    for r, h_, w_, k_, n_pg in pts:
        add_cpu(r, h_, w_, k_, n_pg, args.cpu_seconds / 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
