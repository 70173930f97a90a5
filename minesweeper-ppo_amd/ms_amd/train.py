"""Training driver — the MI355X counterpart of train_rl.py (reference
train_rl.py:82-787), same YAML schema and CLI flags, one process per GPU.

    python -m ms_amd.train --config configs/training/16x16x40_medium.yaml --updates 100
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m ms_amd.train --config ...

Per update (train_rl.py:514-576): entropy / aux-weight schedules ->
collect_rollout (on device) -> GAE (ms_gae) -> ppo_epochs x mini_batches
ppo_update (bf16 autocast; RCCL flat-gradient all-reduce when world > 1) ->
CosineAnnealingLR.step(). Checkpoints keep the reference payload
{"model", "cfg", "model_meta"[, "metric"]} (train_rl.py:623-630, 715-721).
``num_envs`` is GLOBAL: each rank steps num_envs / world envs of the global
seed list, so the trajectories do not depend on the world size.
"""
from __future__ import annotations

import argparse
import math
import csv
import json
import logging
import os
import time
from dataclasses import asdict, dataclass
from typing import Dict

import numpy as np
import torch
import yaml
from torch.optim import AdamW
from torch.optim.lr_scheduler import CosineAnnealingLR

from .buffers import RolloutBuffer
from .dist import DistInfo, broadcast_module, init_from_env
from .dropout import MINIBATCH, keyed_dropout, mix_seed
from .env import EnvConfig, VecMinesweeper
from .models import build_model, strip_compile_prefix
from .ppo import FlatGrads, PPOConfig, ppo_update
from .profiling import prange
from .rollout import collect_rollout


@dataclass
class PPOTrainConfig:  # train_rl.py:82-107
    H: int = 8
    W: int = 8
    mine_count: int = 10
    guarantee_safe_neighborhood: bool = True
    num_envs: int = 256
    steps_per_env: int = 128
    mini_batches: int = 8
    ppo_epochs: int = 3
    gamma: float = 0.995
    gae_lambda: float = 0.95
    clip_eps: float = 0.2
    clip_eps_v: float = 0.2
    vf_coef: float = 0.5
    ent_coef: float = 0.003
    ent_coef_min: float = 0.003
    ent_decay_updates: int = 0
    lr: float = 3e-4
    max_grad_norm: float = 0.5
    aux_mine_weight: float = 0.0
    aux_mine_calib_weight: float = 0.0
    total_updates: int = 1000


def load_config(path: str | None):
    """train_rl.py:110-143: (PPOTrainConfig, env dict, model dict, extras)."""
    if path is None:
        return PPOTrainConfig(), {}, {}, {}
    with open(path) as f:
        data = yaml.safe_load(f) or {}
    env_d = data.get("env", {}) or {}
    ppo_d = data.get("ppo", {}) or {}
    model_d = data.get("model", {}) or {}
    base = PPOTrainConfig()
    kw = {}
    for k in ("H", "W", "mine_count", "guarantee_safe_neighborhood"):
        kw[k] = env_d.get(k, getattr(base, k))
    for k in PPOTrainConfig.__dataclass_fields__:
        if k not in kw:
            kw[k] = ppo_d.get(k, getattr(base, k))
    extras = {k: v for k, v in data.items() if k not in ("env", "ppo", "model")}
    return PPOTrainConfig(**kw), env_d, model_d, extras


def ent_coef_at(cfg: PPOTrainConfig, update: int) -> float:  # train_rl.py:515-523
    if cfg.ent_decay_updates > 0:
        frac = min(1.0, update / max(1, int(cfg.ent_decay_updates)))
        return float(cfg.ent_coef + (cfg.ent_coef_min - cfg.ent_coef) * frac)
    return float(cfg.ent_coef)


def aux_weight_at(update: int, total: int, base: float, warm_w: float, final_w: float, warm_u: int,
                  power: float) -> float:  # train_rl.py:526-541
    if not (base > 0 or warm_w > 0 or final_w > 0):
        return 0.0
    if warm_u > 0 and (update + 1) <= warm_u:
        w = warm_w
    else:
        frac = (update + 1 - warm_u) / max(1, total - warm_u) if total > warm_u else 1.0
        frac = min(1.0, max(0.0, frac))
        if power != 1.0:
            frac = frac ** power
        w = warm_w + (final_w - warm_w) * frac
    return float(max(0.0, w))


def _opt(training: Dict, key: str, conv, default, post=lambda v: v):
    """One optional ``training:`` value, converted; a bad value keeps the default
    (the try/except blocks of train_rl.py:456-504)."""
    v = training.get(key)
    if v is None:
        return default
    try:
        return post(conv(v))
    except Exception:
        return default


def aux_schedule_params(cfg: PPOTrainConfig, training: Dict):
    """(base, warmup weight, final weight, warmup updates, decay power) as train_rl.py:456-504
    reads them from the YAML ``training:`` section."""
    training = training if isinstance(training, dict) else {}
    base = float(getattr(cfg, "aux_mine_weight", 0.0))
    warm_w = _opt(training, "aux_mine_warmup_weight", float, base)
    final_w = _opt(training, "aux_mine_final_weight", float, base)
    warm_u = _opt(training, "aux_mine_warmup_updates", int, 0, lambda v: max(0, v))
    power = _opt(training, "aux_mine_decay_power", float, 1.0, lambda v: max(1e-6, v))
    return base, warm_w, final_w, warm_u, power


def early_stop_patience(training: Dict):
    """train_rl.py:462-470: enabled only for an integer patience > 0."""
    training = training if isinstance(training, dict) else {}
    p = _opt(training, "early_stop_patience", int, None)
    return p if p is not None and p > 0 else None


class Trainer:
    """Holds env shard, model, optimizer and buffers; `update()` runs one PPO
    update. Used by main() and by bench.py's combined-loop measurement."""

    def __init__(self, cfg: PPOTrainConfig, env_d: Dict, model_d: Dict, extras: Dict, *, seed: int = 0,
                 model_name: str | None = None, info: DistInfo | None = None, amp: str = "fp16",
                 device: torch.device | None = None, obs_codes: bool = True):
        """``obs_codes``: the rollout buffer holds u8 cell codes instead of the f32 one-hot obs
        (RolloutBuffer; exact, 40x fewer bytes held and gathered per minibatch)."""
        self.cfg = cfg
        self.obs_codes = obs_codes
        self.info = info or DistInfo()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        training = extras.get("training", {}) if isinstance(extras, dict) else {}
        training = training if isinstance(training, dict) else {}
        rollout = training.get("rollout", {}) or {}
        if "num_envs" in rollout:
            cfg.num_envs = int(rollout["num_envs"])
        if "steps_per_env" in rollout:
            cfg.steps_per_env = int(rollout["steps_per_env"])
        if cfg.num_envs % self.info.world:
            # equal shards are what make every rank run the same number of minibatches (each
            # one ends in collectives) and the mean of the rank means the global mean
            raise ValueError(f"num_envs={cfg.num_envs} must be a multiple of the world size {self.info.world}")
        env_kwargs = {"H": cfg.H, "W": cfg.W, "mine_count": cfg.mine_count,
                      "guarantee_safe_neighborhood": cfg.guarantee_safe_neighborhood}
        env_kwargs.update(env_d)
        env_kwargs.pop("include_frontier_channel", None)
        self.env_cfg = EnvConfig(**env_kwargs)
        late = training.get("late_start") if isinstance(training.get("late_start"), dict) else None
        self.vec = VecMinesweeper(cfg.num_envs, self.env_cfg, seed=seed, late_start_cfg=late,
                                  late_start_seed=seed + 1, device=self.device,
                                  shard=(self.info.rank, self.info.world))
        mcfg = dict(model_d)
        self.model_name = model_name or mcfg.pop("name", "cnn")
        mcfg.pop("name", None)
        self.model_meta = {"name": self.model_name, "config": dict(mcfg)}
        torch.manual_seed(seed)
        self.model = build_model(self.model_name, obs_shape=(10, self.env_cfg.H, self.env_cfg.W),
                                 model_cfg=mcfg).to(self.device)
        broadcast_module(self.model, self.info)
        # the reference's AdamW (train_rl.py:415, default weight decay) as ONE fused kernel on the GPU:
        # the same update per element; under GradScaler the found-inf skip stays on the device (the
        # foreach path's step() reads found_inf on the host, a sync per minibatch) -- DESIGN.md §8
        fused = self.device.type == "cuda" and os.environ.get("MS_FOREACH_ADAMW", "0") == "0"  # (A/B knob)
        self.opt = AdamW(self.model.parameters(), lr=cfg.lr, fused=fused)
        self.sched = CosineAnnealingLR(self.opt, T_max=cfg.total_updates)
        self.amp_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[amp]
        self.scaler = torch.amp.GradScaler("cuda") if amp == "fp16" else None
        # one flat gradient bucket for the data-parallel all-reduce; one rank needs none, and without
        # it autograd hands each gradient over instead of adding it into zeroed views (the same
        # values: 0 + g = g; ~44 fewer add kernels a minibatch)
        self.flat = FlatGrads(self.model.parameters()) if self.info.world > 1 else None
        self.ppo_cfg = PPOConfig(clip_eps=cfg.clip_eps, clip_eps_v=cfg.clip_eps_v, vf_coef=cfg.vf_coef,
                                 ent_coef=cfg.ent_coef, aux_mine_weight=cfg.aux_mine_weight,
                                 aux_mine_calib_weight=cfg.aux_mine_calib_weight,
                                 max_grad_norm=cfg.max_grad_norm,
                                 beta_l2=float(training.get("beta_l2", 0.0)))
        (self.aux_base, self.aux_warm_w, self.aux_final_w, self.aux_warm_u,
         self.aux_power) = aux_schedule_params(cfg, training)
        self.buffer: RolloutBuffer | None = None
        self.seed = seed
        # minibatches are stratified over S stripes of the global env list (RolloutBuffer.
        # get_stratified_minibatches): with S a multiple of the world size, rank r's minibatch k
        # is its part of the unsharded run's minibatch k, so training does not depend on world
        # (minibatch_strata: 1 at world 1 is the reference's single randperm over the buffer).
        # A requested S that does not divide num_envs or is not a multiple of the world size
        # falls back to S = world, which divides num_envs (checked above): every rank then
        # holds num_envs / S envs per stripe and the same number of rows and minibatches.
        S = int(training.get("minibatch_strata", 8))
        if S <= 0 or cfg.num_envs % S or S % self.info.world:
            S = self.info.world
        assert cfg.num_envs % S == 0 and S % self.info.world == 0
        self.strata = S
        self.stripes_local = S // self.info.world
        self.stripe_begin = self.info.rank * self.stripes_local

    def update(self, update: int, profile: bool = False) -> Dict[str, float]:
        """One PPO update. ``profile`` synchronises between phases and adds
        rollout_s / gae_s / ppo_s wall times to the stats."""
        cfg, pc = self.cfg, self.ppo_cfg
        tick = [time.perf_counter()]

        def mark():
            if profile:
                torch.cuda.synchronize(self.device)
                tick.append(time.perf_counter())
        pc.ent_coef = ent_coef_at(cfg, update)
        pc.aux_mine_weight = aux_weight_at(update, cfg.total_updates, self.aux_base, self.aux_warm_w,
                                           self.aux_final_w, self.aux_warm_u, self.aux_power)
        self.model.train()
        with prange("update/rollout"):
            self.buffer, aux = collect_rollout(
                self.vec, self.model, cfg.steps_per_env, self.device, pc.aux_mine_weight,
                pc.aux_mine_calib_weight, amp_dtype=self.amp_dtype, buffer=self.buffer,
                sample_seed=self.seed * 7919 + 17, sample_counter=update << 20, obs_codes=self.obs_codes,
                timing=profile)
        mark()
        with prange("update/gae"):
            self.buffer.compute_gae(aux["last_values"], gamma=cfg.gamma, lam=cfg.gae_lambda)
        mark()
        acc: Dict[str, torch.Tensor] = {}
        n = 0
        group = self.info.group if self.info.world > 1 else None
        dseed = mix_seed(self.seed * 7919 + 17, MINIBATCH)
        for epoch in range(cfg.ppo_epochs):
            mbs = self.buffer.get_stratified_minibatches(cfg.mini_batches, self.stripes_local, self.stripe_begin,
                                                         seed=(self.seed * 1000003 + update) * 64 + epoch)
            for k, batch in enumerate(mbs):
                # Dropout2d masks keyed by (update, epoch, minibatch, global sample id)
                with prange("update/minibatch"), \
                        keyed_dropout(self.model, batch.rows, dseed, (((update << 8) + epoch) << 16) + k):
                    st = ppo_update(self.model, self.opt, batch, pc, self.scaler, amp_dtype=self.amp_dtype,
                                    group=group, flat_grads=self.flat, sync_stats=False)
                for name, v in st.items():
                    acc[name] = acc[name] + v if name in acc else v
                n += 1
        self.sched.step()
        keys = sorted(acc)
        vals = torch.stack([acc[k] for k in keys]).div(max(1, n)).tolist() if keys else []
        out = dict(zip(keys, vals))
        out["aux_weight"] = pc.aux_mine_weight
        out["ent_coef"] = pc.ent_coef
        if profile:
            mark()
            out["rollout_s"], out["gae_s"], out["ppo_s"] = (tick[1] - tick[0], tick[2] - tick[1],
                                                           tick[3] - tick[2])
            for key, v in aux["timings"].items():  # the reference's rollout buckets (train_rl.py:278-288)
                if key.endswith("_total_s"):
                    out["rollout_" + key] = v
        return out

    def checkpoint(self, path: str, metric=None) -> None:
        payload = {"model": {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                   "cfg": asdict(self.cfg), "model_meta": self.model_meta}
        if metric is not None:
            payload["metric"] = metric
        torch.save(payload, path)

    def load_init(self, path: str) -> None:  # train_rl.py:401-413 (weights only, strict=False)
        state = torch.load(path, map_location=self.device, weights_only=True)
        sd = state["model"] if isinstance(state, dict) and "model" in state else state
        self.model.load_state_dict(strip_compile_prefix(sd), strict=False)
        broadcast_module(self.model, self.info)


def quick_eval_score(metrics: Dict[str, float]) -> float:
    """train_rl.py:434-455: win rate plus small guess / AUROC bonuses (keys this build does
    not compute are NaN and contribute nothing, as in the reference)."""
    def _f(v):
        try:
            return float(v)
        except (TypeError, ValueError):
            return float("nan")
    score = _f(metrics.get("win_rate"))
    ge, gs, au = _f(metrics.get("guesses_per_episode")), _f(metrics.get("guess_success_rate")), \
        _f(metrics.get("belief_auroc"))
    if math.isfinite(ge):
        score -= max(0.0, ge - 1.5) * 0.01
        score += max(0.0, 1.5 - ge) * 0.005
    if math.isfinite(gs):
        score += max(0.0, gs - 0.75) * 0.05
    if math.isfinite(au):
        score += max(0.0, au - 0.93) * 0.02
    return score


def evaluate_model(model, env_cfg, *, episodes: int, num_envs: int, seed: int, pairs: int = 1,
                   amp_dtype=None) -> Dict[str, float]:
    """train_rl.py:49-69: ``pairs`` evaluations with seeds seed, seed+1, ... averaged."""
    from .eval import evaluate_vec
    runs = [evaluate_vec(model, env_cfg, episodes=episodes, seed=seed + i, num_envs=num_envs, amp_dtype=amp_dtype)
            for i in range(max(1, pairs))]
    keys = runs[0].keys()
    return {k: float(np.mean([r[k] for r in runs])) for k in keys}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=str, default=None)
    ap.add_argument("--model", type=str, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", type=str, default="runs/ppo")
    ap.add_argument("--updates", type=int, default=None)
    ap.add_argument("--init_ckpt", type=str, default=None)
    ap.add_argument("--save_every", type=int, default=50)
    ap.add_argument("--amp", choices=["bf16", "fp16", "fp32"], default="fp16",
                    help="autocast type: fp16 + GradScaler as the reference (train_rl.py:415-420), bf16 (no scaler) or fp32")
    # evaluation flags of train_rl.py:297-305 (on-device greedy eval, ms_amd/eval.py)
    ap.add_argument("--eval_episodes", type=int, default=2048)
    ap.add_argument("--eval_num_envs", type=int, default=64)
    ap.add_argument("--eval_quick_episodes", type=int, default=512)
    ap.add_argument("--quick_eval_pairs", type=int, default=2)
    ap.add_argument("--quick_eval_interval", type=int, default=10)
    ap.add_argument("--eval_pairs", type=int, default=1)
    ap.add_argument("--eval_amp", choices=["fp32", "bf16", "fp16"], default="fp32",
                    help="evaluation precision (the reference evaluates in fp32)")
    ap.add_argument("--skip_final_eval", action="store_true")
    ap.add_argument("--grad_checkpoint", action="store_true")
    ap.add_argument("--flash_attention", choices=["auto", "on", "off"], default="auto")
    args = ap.parse_args(argv)
    from . import exact_fp32_convs
    exact_fp32_convs()  # before any convolution (the fp32 / eval paths use MIOpen)

    info = init_from_env()
    cfg, env_d, model_d, extras = load_config(args.config)
    if args.updates is not None:
        cfg.total_updates = int(args.updates)
    training = extras.get("training", {}) if isinstance(extras, dict) else {}
    patience = early_stop_patience(training)
    logging.basicConfig(level=logging.INFO if info.is_main else logging.WARNING,
                        format="[%(asctime)s] %(message)s", datefmt="%H:%M:%S")
    log = logging.getLogger("ms_amd.train")
    device = torch.device("cuda", info.local_rank if info.world > 1 else torch.cuda.current_device())
    torch.cuda.set_device(device)
    tr = Trainer(cfg, env_d, model_d, extras, seed=args.seed, model_name=args.model, info=info, amp=args.amp,
                 device=device)
    env_cfg = tr.vec.cfg
    eval_amp = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.eval_amp)
    if args.init_ckpt:
        tr.load_init(args.init_ckpt)
    if info.is_main:
        os.makedirs(args.out, exist_ok=True)
        n_params = sum(p.numel() for p in tr.model.parameters())
        log.info(f"Model: {tr.model_name} | params={n_params / 1e6:.2f}M | world={info.world} | "
                 f"envs/rank={tr.vec.num_envs}")
    rows = []
    best_score, best_metrics, best_update, best_ckpt = float("-inf"), None, -1, None
    stopped_early = False
    quick_eps = max(0, min(args.eval_quick_episodes, args.eval_episodes))
    for update in range(cfg.total_updates):
        t0 = time.time()
        st = tr.update(update)
        dt = time.time() - t0
        row = {"update": update + 1, "seconds": dt, "steps": cfg.num_envs * cfg.steps_per_env, **st}
        for k in ("quick_win_rate", "quick_guesses_per_ep", "quick_guess_success", "quick_belief_auroc",
                  "quick_belief_ece", "quick_forced_guess_rate", "quick_safe_option_pick_rate", "quick_score"):
            row[k] = None
        rows.append(row)
        stop = False
        if info.is_main:
            extra = "".join(f" {k}={st[k]:.4f}" for k in ("aux_bce", "aux_calib") if k in st)
            log.info(f"upd {update + 1}/{cfg.total_updates} | {dt:.2f}s | steps={row['steps']} | "
                     f"pi={st.get('policy_loss', float('nan')):.4f} v={st.get('value_loss', float('nan')):.4f} "
                     f"ent={st.get('entropy', float('nan')):.4f}{extra} ent_coef={st['ent_coef']:.4f}")
            if (update + 1) % max(1, args.save_every) == 0:
                tr.checkpoint(os.path.join(args.out, "ckpt_latest.pt"))
            if quick_eps > 0 and args.quick_eval_interval > 0 and (update + 1) % args.quick_eval_interval == 0:
                mq = evaluate_model(tr.model, env_cfg, episodes=quick_eps,
                                    seed=args.seed * 1000 + (update + 1) * 7,
                                    num_envs=min(args.eval_num_envs, max(1, quick_eps // 8)),
                                    pairs=args.quick_eval_pairs, amp_dtype=eval_amp)
                score = quick_eval_score(mq)
                row.update(quick_win_rate=mq["win_rate"], quick_belief_auroc=mq["belief_auroc"],
                           quick_belief_ece=mq["belief_ece"], quick_forced_guess_rate=mq["forced_guess_rate"],
                           quick_safe_option_pick_rate=mq["safe_option_pick_rate"], quick_score=score)
                log.info("quick eval upd %d: win_rate=%.3f avg_steps=%.2f auroc=%.3f score=%.3f", update + 1,
                         mq["win_rate"], mq["avg_steps"], mq["belief_auroc"], score)
                if score > best_score or best_update < 0:
                    best_score, best_metrics, best_update = score, mq, update + 1
                    best_ckpt = os.path.join(args.out, "ckpt_best.pt")
                    tr.checkpoint(best_ckpt, metric=mq)
                if patience is not None and best_update >= 0 and (update + 1) - best_update >= patience:
                    log.info("Early stopping at update %d (best score %.3f at update %d, patience=%d)",
                             update + 1, best_score, best_update, patience)
                    stop = True
        if info.world > 1:  # every rank leaves the loop together
            flag = torch.tensor([1.0 if stop else 0.0], device=device)
            torch.distributed.all_reduce(flag, group=info.group)
            stop = bool(flag.item() > 0)
        if stop:
            stopped_early = True
            break
    if info.is_main:
        keys = sorted(set().union(*rows)) if rows else []
        with open(os.path.join(args.out, "train_metrics.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            for r in rows:
                w.writerow(r)
        final = os.path.join(args.out, "ckpt_final.pt")
        tr.checkpoint(final)
        last = final
        if best_ckpt and os.path.exists(best_ckpt):  # evaluate the best weights (train_rl.py:703-718)
            state = torch.load(best_ckpt, map_location=device, weights_only=True)
            tr.model.load_state_dict(strip_compile_prefix(state["model"]), strict=False)
            last = best_ckpt
        metrics_raw = None
        if not args.skip_final_eval and args.eval_episodes > 0 and args.eval_num_envs > 0:
            eps = max(1, args.eval_episodes)
            metrics_raw = evaluate_model(tr.model, env_cfg, episodes=eps, seed=args.seed * 17,
                                         num_envs=min(args.eval_num_envs, eps), pairs=args.eval_pairs,
                                         amp_dtype=eval_amp)
            log.info("final eval: %s", {k: round(v, 4) for k, v in metrics_raw.items() if math.isfinite(v)})
        with open(os.path.join(args.out, "summary.json"), "w") as f:
            json.dump({"checkpoint": os.path.basename(last), "metrics_raw": metrics_raw, "model": tr.model_meta,
                       "seed": args.seed, "quick_eval_pairs": args.quick_eval_pairs,
                       "quick_eval_interval": args.quick_eval_interval, "eval_pairs": args.eval_pairs,
                       "best_quick_metrics": best_metrics,
                       "best_quick_score": best_score if math.isfinite(best_score) else None,
                       "best_checkpoint": os.path.basename(best_ckpt) if best_ckpt else None,
                       "best_update": best_update, "stopped_early": stopped_early,
                       "early_stop_patience": patience, "world_size": info.world}, f)
    if info.world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
