"""RolloutBuffer.get_minibatches (reference buffers.py:96-116):
every row of the T*N buffer appears exactly once per epoch, minibatches are
slices of ``batch_size`` of one permutation (a short tail when B is not a
multiple), and every field of a minibatch row comes from the same buffer row."""
from __future__ import annotations

import pytest
import torch


def _filled(dev, N=12, T=5, H=3, W=4, labels=True):
    from ms_amd.buffers import RolloutBuffer
    buf = RolloutBuffer(N, T, (10, H, W), H * W, dev, with_mine_labels=labels)
    B = N * T
    r = torch.arange(B, device=dev)
    buf.obs.copy_(r.float().view(B, 1, 1, 1).expand_as(buf.obs))
    buf.action_mask.copy_(((r.view(B, 1) + torch.arange(H * W, device=dev)) % 3 == 0))
    buf.actions.copy_(r)
    for name in ("logp", "rewards", "values", "advantages", "returns"):
        getattr(buf, name).copy_(r.float() + {"logp": 0.25, "rewards": 0.5, "values": 0.75,
                                              "advantages": 1.25, "returns": 1.5}[name])
    buf.dones.copy_(r % 2 == 1)
    if labels:
        buf.mine_labels.copy_((r % 7).float().view(B, 1, 1).expand_as(buf.mine_labels))
        buf.mine_valid.copy_((r % 5 != 0).view(B, 1, 1).expand_as(buf.mine_valid))
    return buf, B, H * W


def _check_epoch(buf, B, A, mb, gen=None, labels=True):
    seen = []
    sizes = []
    for b in buf.get_minibatches(mb, generator=gen):
        rows = b.actions
        sizes.append(rows.numel())
        seen.append(rows)
        f = rows.float()
        assert torch.equal(b.obs.amax(dim=(1, 2, 3)), f) and torch.equal(b.obs.amin(dim=(1, 2, 3)), f)
        assert torch.equal(b.action_mask, (rows.view(-1, 1) + torch.arange(A, device=rows.device)) % 3 == 0)
        assert torch.equal(b.old_logp, f + 0.25) and torch.equal(b.rewards, f + 0.5)
        assert torch.equal(b.values, f + 0.75) and torch.equal(b.advantages, f + 1.25)
        assert torch.equal(b.returns, f + 1.5) and torch.equal(b.dones, rows % 2 == 1)
        if labels:
            assert torch.equal(b.mine_labels[:, 0, 0], (rows % 7).float())
            assert torch.equal(b.mine_valid.all(dim=(1, 2)), rows % 5 != 0)
        else:
            assert not hasattr(b, "mine_labels")
    allrows = torch.cat(seen)
    assert torch.equal(allrows.sort().values, torch.arange(B, device=allrows.device))
    want = [mb] * (B // mb) + ([B % mb] if B % mb else [])
    assert sizes == want
    return allrows


def _devices():
    return ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("mb", [60, 15, 7, 1])
def test_minibatches_cover_each_row_once(dev, mb):
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.fail("gpu test without a HIP device")
    buf, B, A = _filled(torch.device(dev))
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    perms = [_check_epoch(buf, B, A, mb, g) for _ in range(3)]  # 3 epochs, fresh permutation each
    if mb < B:
        assert not torch.equal(perms[0], perms[1])


@pytest.mark.parametrize("dev", _devices())
def test_minibatches_without_labels(dev):
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.fail("gpu test without a HIP device")
    buf, B, A = _filled(torch.device(dev), labels=False)
    _check_epoch(buf, B, A, 16, labels=False)


def test_minibatches_seeded_generator_is_reproducible():
    buf, B, A = _filled(torch.device("cpu"))
    runs = []
    for _ in range(2):
        g = torch.Generator()
        g.manual_seed(11)
        runs.append(torch.cat([b.actions for b in buf.get_minibatches(8, generator=g)]))
    assert torch.equal(runs[0], runs[1])


def _tagged(N, T, env_begin, dev="cpu"):
    """Buffer whose actions hold the GLOBAL (t, env) id t*1000 + env of each row."""
    from ms_amd.buffers import RolloutBuffer
    buf = RolloutBuffer(N, T, (10, 2, 2), 4, torch.device(dev))
    t = torch.arange(T).view(T, 1)
    e = torch.arange(N).view(1, N) + env_begin
    buf.actions.copy_((t * 1000 + e).reshape(-1))
    return buf


@pytest.mark.parametrize("world", [2, 4])
def test_stratified_minibatches_are_world_invariant(world):
    """Rank r's minibatch k (its stripes of the global env list) is exactly its part of
    minibatch k of the unsharded buffer with the same seed; sizes are equal across ranks."""
    N, T, S, mbs = 16, 6, 4, 3
    full = [set(b.actions.tolist()) for b in _tagged(N, T, 0).get_stratified_minibatches(mbs, S, 0, seed=77)]
    n = N // world
    parts = []
    for r in range(world):
        buf = _tagged(n, T, r * n)
        parts.append([b.actions.tolist() for b in buf.get_stratified_minibatches(mbs, S // world, r * S // world,
                                                                                 seed=77)])
    assert len(full) == mbs and all(len(p) == mbs for p in parts)
    for k in range(mbs):
        sizes = {len(p[k]) for p in parts}
        assert len(sizes) == 1
        union = set().union(*(set(p[k]) for p in parts))
        assert union == full[k] and sum(len(p[k]) for p in parts) == len(full[k])
    allrows = sorted(x for k in range(mbs) for x in full[k])
    assert allrows == sorted(t * 1000 + e for t in range(T) for e in range(N))
    # a different epoch seed permutes differently
    other = [set(b.actions.tolist()) for b in _tagged(N, T, 0).get_stratified_minibatches(mbs, S, 0, seed=78)]
    assert other != full


def test_obs_codes_buffer_layout_and_cpu_guard():
    """The u8-code buffer (the Trainer's layout) stores [B, H, W] bytes and is HIP-only: the
    encode is a device kernel, so a CPU buffer in that mode is refused up front."""
    from ms_amd import _lib as L
    from ms_amd.buffers import RolloutBuffer
    with pytest.raises(L.MsEnvError):
        RolloutBuffer(4, 2, (10, 3, 3), 9, torch.device("cpu"), obs_codes=True)
    with pytest.raises(ValueError):
        RolloutBuffer(4, 2, (11, 3, 3), 9, torch.device("cpu"), obs_codes=True)
    b = RolloutBuffer(4, 2, (10, 3, 3), 9, torch.device("cpu"))
    assert b.obs.shape == (8, 10, 3, 3) and b.obs.dtype == torch.float32 and not b.obs_codes
