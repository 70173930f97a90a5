"""Greedy evaluation on device: win rate + Wilson CI, steps, progress, invalid-action
rate, belief AUROC / ECE over unknown cells.

Reference: eval.py:265-511 (``evaluate_vec``), AUROC eval.py:54-66, ECE eval.py:69-90,
Wilson interval eval.py:447-458, CLI eval.py:526-640. The episode bookkeeping follows
the reference loop exactly (a batch of ``num_envs`` envs; each env's current episode
is counted once; the env stream is NOT reset between batches; envs past
``batch_size`` in a final partial batch still count, as in the reference), but every
per-env quantity is a device tensor: one host sync per step (the loop condition).

Not computed here: the avoidability / forced-move diagnostics (``forced_guess_*``,
``safe_option_*``, component sizes; eval.py:356-398 via avoidability.py / rules.py).
They are host-side rule solvers outside the hot path (SURVEY.md §8f rank 1 note);
their keys are returned as NaN so callers that print the reference's summary work.
"""
from __future__ import annotations

import argparse
import math
import os
from typing import Callable, Dict, Optional

import numpy as np
import torch

from .env import EnvConfig, VecMinesweeper

NAN = float("nan")
_HOST_ONLY_KEYS = ("forced_guess_rate", "forced_guess_success_rate", "forced_guess_episode_rate",
                   "safe_option_rate", "safe_option_miss_rate", "safe_option_pick_rate",
                   "avg_safe_options_per_turn", "avg_frontier_component_size", "avg_selected_component_size")


def wilson_interval(successes: int, total: int, z: float = 1.96) -> tuple:
    """95 % Wilson score interval (eval.py:447-458)."""
    if total <= 0:
        return NAN, NAN
    phat = successes / float(total)
    denom = 1.0 + (z * z) / total
    center = phat + (z * z) / (2.0 * total)
    rad = z * math.sqrt((phat * (1.0 - phat) / total) + (z * z) / (4.0 * total * total))
    return float((center - rad) / denom), float((center + rad) / denom)


def compute_auroc(labels: torch.Tensor, scores: torch.Tensor) -> float:
    """Rank-sum AUROC (eval.py:54-66): ranks 1..n by ascending score, no tie averaging."""
    labels = labels.reshape(-1)
    scores = scores.reshape(-1).to(torch.float64)
    pos = float((labels == 1).sum())
    neg = float((labels == 0).sum())
    if pos == 0 or neg == 0:
        return NAN
    order = torch.argsort(scores, stable=True)
    ranks = torch.empty_like(scores)
    ranks[order] = torch.arange(1, scores.numel() + 1, dtype=torch.float64, device=scores.device)
    pos_rank_sum = float(ranks[labels == 1].sum())
    return float((pos_rank_sum - pos * (pos + 1.0) / 2.0) / (pos * neg))


def compute_ece(probs: torch.Tensor, labels: torch.Tensor, bins: int = 15) -> float:
    """Expected calibration error with equal-width bins (eval.py:69-90): bin i holds
    [i/bins, (i+1)/bins), the last bin is closed."""
    probs = probs.reshape(-1).to(torch.float64)
    labels = labels.reshape(-1).to(torch.float64)
    total = probs.numel()
    if total == 0:
        return NAN
    edges = torch.linspace(0.0, 1.0, bins + 1, dtype=torch.float64, device=probs.device)
    idx = torch.bucketize(probs, edges[1:-1], right=True)  # probs in [e_i, e_{i+1}) -> i
    idx = torch.where(probs >= edges[-1], torch.full_like(idx, bins - 1), idx)
    inside = (probs >= 0.0) & (probs <= 1.0)
    idx, p, lab = idx[inside], probs[inside], labels[inside]
    count = torch.zeros(bins, dtype=torch.float64, device=probs.device).index_add_(0, idx, torch.ones_like(p))
    acc = torch.zeros_like(count).index_add_(0, idx, lab)
    conf = torch.zeros_like(count).index_add_(0, idx, p)
    nz = count > 0
    ece = ((count[nz] / total) * (acc[nz] / count[nz] - conf[nz] / count[nz]).abs()).sum()
    return float(ece)


@torch.no_grad()
def evaluate_vec(model: torch.nn.Module, env_cfg: EnvConfig, episodes: int = 1000, seed: int = 0,
                 num_envs: int = 256, progress_every: int = 0,
                 print_fn: Optional[Callable[[str], None]] = None, reveal_only: bool = False,
                 max_steps_per_episode: int = 512, reveal_fallback_every: int = 0,
                 device: Optional[torch.device] = None, amp_dtype: Optional[torch.dtype] = None,
                 vec: Optional[VecMinesweeper] = None) -> Dict[str, float]:
    """Greedy (argmax over valid cells) evaluation, reference semantics (eval.py:265-511).

    ``amp_dtype`` None runs the model in fp32 like the reference; torch.bfloat16 uses
    the fused MFMA trunk. ``vec`` may be passed to evaluate on an existing env stream."""
    device = device or next(model.parameters()).device
    train_mode = model.training
    model.eval()
    if print_fn is None:
        def print_fn(msg: str):
            print(msg, flush=True)
    if vec is None:
        vec = VecMinesweeper(num_envs, env_cfg, seed=seed, device=device)
    num_envs = vec.num_envs
    batch = vec.reset()
    H, W = env_cfg.H, env_cfg.W
    reveal_count = H * W
    ar = torch.arange(num_envs, device=device)

    remaining = episodes
    processed = 0
    wins = torch.zeros((), dtype=torch.int64, device=device)
    total_steps = torch.zeros((), dtype=torch.int64, device=device)
    total_progress = torch.zeros((), dtype=torch.float64, device=device)
    invalids = torch.zeros((), dtype=torch.int64, device=device)
    belief_p, belief_l = [], []
    while remaining > 0:
        batch_size = min(num_envs, remaining)
        counted = torch.zeros(num_envs, dtype=torch.bool, device=device)
        step_counters = torch.zeros(num_envs, dtype=torch.int32, device=device)
        finished = 0
        tick = 0
        last_reported = 0
        while finished < batch_size:
            obs = batch["obs"]
            mask = batch["action_mask"].clone()
            if reveal_only or (reveal_fallback_every and tick % reveal_fallback_every == 0):
                mask[:, reveal_count:] = False  # the action space is reveal-only: a no-op here
            empty = ~mask.any(dim=1)
            mask[empty] = True
            with torch.autocast("cuda", dtype=amp_dtype or torch.bfloat16, enabled=amp_dtype is not None):
                logits, _, mine_logits = model(obs, return_mine=True)
            logits = logits.float().reshape(num_envs, -1)
            actions = logits.masked_fill(~mask, -1e9).argmax(dim=-1)
            invalids += (~mask[ar, actions]).sum()
            # belief over unknown (= not revealed; flags are never set) cells of the
            # envs whose episode is still being counted, captured before the step
            labels, _ = vec.mine_labels()  # mine_mask (all 0 before the first click)
            unknown = obs[:, 0] == 0
            live = (~counted) & (ar < batch_size)
            sel = unknown & live[:, None, None]
            belief_p.append(torch.sigmoid(mine_logits.float()).reshape(num_envs, H, W)[sel])
            belief_l.append(labels[sel])

            batch, _, dones, infos = vec.step(actions)
            t = infos.tensors
            step_counters += 1
            open_ = ~counted
            total_progress += (t["last_new_reveals"].to(torch.float64) * open_).sum() / float(H * W)
            fin = open_ & dones
            wins += (fin & (t["outcome"] == 1)).sum()
            total_steps += (step_counters.to(torch.int64) * fin).sum()
            step_counters = torch.where(fin, torch.zeros_like(step_counters), step_counters)
            counted = counted | fin
            if max_steps_per_episode > 0:
                cut = (~counted) & (step_counters >= max_steps_per_episode)
                total_steps += (step_counters.to(torch.int64) * cut).sum()
                step_counters = torch.where(cut, torch.zeros_like(step_counters), step_counters)
                counted = counted | cut
            finished = int(counted.sum())  # the reference counts envs past batch_size too
            tick += 1
            if progress_every:
                if finished - last_reported >= min(progress_every, batch_size):
                    print_fn(f"eval progress: {processed + finished}/{episodes} episodes")
                    last_reported = finished
                elif tick % 50 == 0:
                    print_fn(f"eval progress: {processed + finished}/{episodes} episodes (running)")
        remaining -= batch_size
        processed += batch_size
        if progress_every and processed % progress_every == 0:
            print_fn(f"eval progress: {processed}/{episodes} episodes")
    if train_mode:
        model.train()

    wins_i = int(wins)
    lo, hi = wilson_interval(wins_i, max(1, episodes))
    if belief_p:
        probs = torch.cat(belief_p)
        labs = torch.cat(belief_l)
        auroc = compute_auroc(labs, probs) if probs.numel() else NAN
        ece = compute_ece(probs, labs) if probs.numel() else NAN
    else:
        auroc = ece = NAN
    ts = int(total_steps)
    out = {
        "win_rate": wins_i / max(1, episodes),
        "win_ci_low": lo,
        "win_ci_high": hi,
        "avg_steps": ts / max(1, episodes),
        "avg_progress": float(total_progress) / max(1, episodes),
        "invalid_rate": int(invalids) / max(1, ts),
        "belief_auroc": auroc,
        "belief_ece": ece,
        "wins": float(wins_i),
        "episodes": float(episodes),
    }
    out.update({k: NAN for k in _HOST_ONLY_KEYS})
    return out


def main(argv=None) -> None:
    """CLI with the reference's flags (eval.py:526-536)."""
    import yaml

    from .models import build_model, strip_compile_prefix
    ap = argparse.ArgumentParser(description="Evaluate a Minesweeper RL checkpoint on device")
    ap.add_argument("--run_dir", type=str, default=None)
    ap.add_argument("--ckpt", type=str, default=None)
    ap.add_argument("--episodes", type=int, default=64)
    ap.add_argument("--config", type=str, required=True)
    ap.add_argument("--model", type=str, default=None)
    ap.add_argument("--num_envs", type=int, default=128)
    ap.add_argument("--progress", action="store_true")
    ap.add_argument("--reveal_only", action="store_true")
    ap.add_argument("--debug_eval", action="store_true", help="accepted; not implemented on device")
    ap.add_argument("--amp", choices=["fp32", "bf16", "fp16"], default="fp32")
    args = ap.parse_args(argv)
    from . import exact_fp32_convs
    exact_fp32_convs()
    device = torch.device("cuda")
    if args.ckpt:
        ckpt = args.ckpt
    else:
        if not args.run_dir:
            raise SystemExit("Provide either --ckpt or --run_dir")
        import glob
        import re
        paths = glob.glob(os.path.join(args.run_dir, "ckpt_*.pt"))
        if not paths:
            raise FileNotFoundError(f"No checkpoints found in {args.run_dir}")
        num = lambda p: int(m.group(1)) if (m := re.search(r"ckpt_(\d+)\.pt$", os.path.basename(p))) else -1  # noqa: E731
        ckpt = max(paths, key=num)
    with open(args.config) as f:
        cfg = yaml.safe_load(f)
    env_d = dict(cfg["env"] if "env" in cfg else cfg)
    env_d.pop("include_frontier_channel", None)
    env_cfg = EnvConfig(**env_d)
    state = torch.load(ckpt, map_location=device, weights_only=True)
    meta = state.get("model_meta", {}) if isinstance(state, dict) else {}
    mcfg = dict((meta or {}).get("config", {}))
    mcfg.pop("name", None)
    name = args.model or (meta or {}).get("name", "cnn")
    model = build_model(name, obs_shape=(10, env_cfg.H, env_cfg.W), model_cfg=mcfg).to(device)
    sd = strip_compile_prefix(dict(state["model"]) if isinstance(state, dict) and "model" in state else state)
    ms = model.state_dict()
    model.load_state_dict({k: v for k, v in sd.items() if k in ms and ms[k].shape == v.shape}, strict=False)
    metrics = evaluate_vec(model, env_cfg, episodes=args.episodes, seed=0,
                           num_envs=min(args.num_envs, args.episodes),
                           progress_every=(max(1, args.episodes // 4) if args.progress else 0),
                           reveal_only=args.reveal_only,
                           amp_dtype={"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.amp))
    summary = {"checkpoint": os.path.basename(ckpt), "model": name, **metrics}
    for k, v in summary.items():
        print(f"{k}: {v:.3f}" if isinstance(v, float) and np.isfinite(v) else f"{k}: {v}")


if __name__ == "__main__":
    main()
