"""Policy parity (CPU, fp32, eval mode) against outputs captured from the
reference models (tests/golden/model_*.npz): logits/values/mine within 1e-5,
and bit-identical seeded initialisation (state_dict sha256)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest
import torch

from conftest import golden


def _sha(model):
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


@pytest.fixture(autouse=True)
def _fp32():
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    yield
    torch.set_float32_matmul_precision(prev)


def test_small_model_outputs_from_golden_weights():
    from ms_amd.models import build_model
    z = golden("model_small.npz")
    m = build_model("cnn_residual", obs_shape=(10, 16, 16),
                    model_cfg=dict(stem_channels=16, blocks=2, dropout=0.05, value_hidden=32)).eval()
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w::")}
    missing, unexpected = m.load_state_dict(sd, strict=True), None
    with torch.no_grad():
        lg, v, mine = m(torch.from_numpy(z["obs"]), return_mine=True)
    np.testing.assert_allclose(lg.numpy(), z["logits"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(v.numpy(), z["value"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(mine.numpy(), z["mine"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("H,W", [(16, 16), (9, 9), (30, 16)])
def test_full_model_seeded_init_and_outputs(H, W):
    from ms_amd.models import build_model
    z = golden(f"model_full_{H}x{W}.npz")
    torch.manual_seed(0)
    m = build_model("cnn_residual", obs_shape=(10, H, W),
                    model_cfg=dict(stem_channels=96, blocks=5, dropout=0.05, value_hidden=256)).eval()
    assert sum(p.numel() for p in m.parameters()) == int(z["n_params"]) == 950947
    assert _sha(m) == z["sha256"].item().decode()
    with torch.no_grad():
        lg, v, mine = m(torch.from_numpy(z["obs"]), return_mine=True)
    np.testing.assert_allclose(lg.numpy(), z["logits"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(v.numpy(), z["value"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(mine.numpy(), z["mine"], rtol=0, atol=1e-5)


def test_cnn_policy_seeded_init_and_outputs():
    from ms_amd.models import build_model
    z = golden("model_cnn_9x9.npz")
    torch.manual_seed(0)
    m = build_model("cnn", obs_shape=(10, 9, 9), model_cfg=dict(hidden=64)).eval()
    assert _sha(m) == z["sha256"].item().decode()
    with torch.no_grad():
        lg, v, mine = m(torch.from_numpy(z["obs"]), return_mine=True)
    np.testing.assert_allclose(lg.numpy(), z["logits"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(v.numpy(), z["value"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(mine.numpy(), z["mine"], rtol=0, atol=1e-5)


def test_build_model_names_and_errors():
    from ms_amd.models import CNNPolicy, CNNResidualPolicy, build_model, strip_compile_prefix
    assert isinstance(build_model("cnn_large", obs_shape=(10, 8, 8)), CNNResidualPolicy)
    assert isinstance(build_model("cnn", obs_shape=(10, 8, 8)), CNNPolicy)
    with pytest.raises(ValueError):
        build_model("transformer", obs_shape=(10, 8, 8))
    with pytest.raises(ValueError):
        CNNResidualPolicy(10, stem_channels=0)
    sd = {"_orig_mod.stem.0.weight": 1, "_orig_mod.stem.0.bias": 2}
    assert set(strip_compile_prefix(sd)) == {"stem.0.weight", "stem.0.bias"}


def test_models_take_cell_codes_on_cpu():
    """The Trainer's rollout buffer holds u8 cell codes [N, H, W] (ms_amd.fused.obs_encode):
    codes_to_obs decodes them to the env's one-hot planes (0 = hidden -> all zero, 1 + k = revealed
    with k adjacent mines -> planes 0 and 1 + k), and both models give the same outputs on codes as
    on the decoded obs (the PyTorch path; the fused path is tested on the GPU)."""
    from ms_amd.fused import codes_to_obs
    from ms_amd.models import build_model
    codes = torch.arange(10, dtype=torch.uint8).view(1, 2, 5)
    obs = codes_to_obs(codes)
    assert obs.shape == (1, 10, 2, 5) and obs.dtype == torch.float32
    for i in range(10):
        r, c = divmod(i, 5)
        want = torch.zeros(10)
        if i > 0:
            want[0] = 1.0
            want[i] = 1.0
        assert torch.equal(obs[0, :, r, c], want), i
    g = torch.Generator().manual_seed(2)
    codes = torch.randint(0, 10, (6, 9, 9), dtype=torch.uint8, generator=g)
    for name, cfg in (("cnn", {}), ("cnn_residual", dict(stem_channels=16, blocks=1, dropout=0.0, value_hidden=16))):
        torch.manual_seed(0)
        m = build_model(name, obs_shape=(10, 9, 9), model_cfg=cfg).eval()
        with torch.no_grad():
            a = m(codes, return_mine=True)
            b = m(codes_to_obs(codes), return_mine=True)
        for x, y in zip(a, b):
            assert torch.equal(x, y), name


def test_model_constructors_select_exact_fp32_convs(monkeypatch):
    """Building CNNResidualPolicy / CNNPolicy directly (as the reference's code does, without
    build_model) turns MIOpen's fp32 Winograd convolutions off too."""
    from ms_amd.models import CNNPolicy, CNNResidualPolicy
    for ctor in (lambda: CNNResidualPolicy(10, stem_channels=16, blocks=1, value_hidden=8), lambda: CNNPolicy(10)):
        monkeypatch.delenv("MIOPEN_DEBUG_CONV_WINOGRAD", raising=False)
        ctor()
        import os
        assert os.environ.get("MIOPEN_DEBUG_CONV_WINOGRAD") == "0"
