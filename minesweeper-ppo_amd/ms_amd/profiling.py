"""Profiler ranges and event-timed phase buckets ("profiler ranges around env-step /
forward / GAE / update").

``prange(name)`` is a roctx range (torch.cuda.nvtx maps to roctx on ROCm builds of PyTorch), seen
by ``rocprofv3 --marker-trace``; it costs one host call and never synchronises.

``PhaseTimer`` attributes GPU time to named buckets with HIP events recorded on the current
stream: ``split(bucket)`` records an event and charges the interval since the previous one to
``bucket``. Nothing waits on the device until ``totals()`` is called, so a rollout loop keeps its
launch queue full (the reference times its phases with ``time.perf_counter`` around host calls
that synchronise, train_rl.py:194-289).
"""
from __future__ import annotations

import contextlib
from collections.abc import Mapping
from typing import Dict, Iterator, List, Optional, Tuple

import torch


@contextlib.contextmanager
def prange(name: str):
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class PhaseTimer:
    """GPU time per bucket from consecutive events on one stream (no host sync until read)."""

    def __init__(self, device: torch.device, enabled: bool = True):
        self.enabled = enabled and torch.device(device).type == "cuda"
        self.dev = torch.device(device).index or 0
        self._marks: List[Tuple[torch.cuda.Event, Optional[str]]] = []
        self._pool: List[torch.cuda.Event] = []  # reused after totals()
        self._used = 0
        self._totals: Optional[Dict[str, float]] = None

    def _event(self) -> torch.cuda.Event:
        if self._used == len(self._pool):
            self._pool.append(torch.cuda.Event(enable_timing=True))
        ev = self._pool[self._used]
        self._used += 1
        return ev

    def start(self) -> None:
        if self.enabled:
            ev = self._event()
            ev.record()
            self._marks.append((ev, None))

    def split(self, bucket: str) -> None:
        """Charge the GPU time since the previous mark to ``bucket``."""
        if self.enabled:
            ev = self._event()
            ev.record()
            self._marks.append((ev, bucket))

    def totals(self) -> Dict[str, float]:
        """Seconds per bucket (synchronises on the last event once)."""
        if self._totals is None:
            tot: Dict[str, float] = {}
            if self._marks:
                self._marks[-1][0].synchronize()
                for (a, _), (b, name) in zip(self._marks, self._marks[1:]):
                    if name is not None:
                        tot[name] = tot.get(name, 0.0) + a.elapsed_time(b) / 1e3
            self._totals = tot
            self._marks = []
            self._used = 0  # the pool's events are free again
        return self._totals


class RolloutTimings(Mapping):
    """The reference's ``timings`` dict of collect_rollout (train_rl.py:278-288): steps and, per
    bucket (tensor_bridge, mine_label_copy, env_step, model_forward), ``<bucket>_total_s`` and
    ``<bucket>_per_step_ms``, measured on the GPU by a PhaseTimer and resolved on first read;
    plus ``enqueue_total_s``, the host time the loop took to enqueue. With timing disabled
    (``collect_rollout(timing=False)``) no events exist and only ``steps`` and
    ``enqueue_total_s`` are present. ``to_dict()`` gives a plain dict (json-serialisable).

    On this path the buckets mean: tensor_bridge = the device-side hand-offs that replace the
    reference's PCIe copies (obs -> cell codes, values -> buffer), mine_label_copy = ms_labels,
    env_step = ms_step, model_forward = the policy forward plus the masked sampling."""

    BUCKETS = ("tensor_bridge", "mine_label_copy", "env_step", "model_forward")

    def __init__(self, steps: int, timer: PhaseTimer, enqueue_s: float):
        self._steps, self._timer, self._enqueue = steps, timer, enqueue_s
        self._d: Optional[Dict[str, float]] = None

    def _resolve(self) -> Dict[str, float]:
        if self._d is None:
            tot = self._timer.totals()
            d: Dict[str, float] = {"steps": self._steps}
            for b in (self.BUCKETS if self._timer.enabled else ()):
                s = tot.get(b, 0.0)
                d[f"{b}_total_s"] = s
                d[f"{b}_per_step_ms"] = (s / self._steps) * 1000.0 if self._steps else 0.0
            d["enqueue_total_s"] = self._enqueue
            self._d = d
        return self._d

    def __getitem__(self, k):
        return self._resolve()[k]

    def __iter__(self) -> Iterator[str]:
        return iter(self._resolve())

    def __len__(self) -> int:
        return len(self._resolve())

    def __repr__(self) -> str:
        return repr(self._resolve())

    def to_dict(self) -> Dict[str, float]:
        return dict(self._resolve())


__all__ = ["prange", "PhaseTimer", "RolloutTimings"]
