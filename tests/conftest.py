"""Shared pytest setup: paths, the `gpu` marker, golden-fixture loading."""
from __future__ import annotations

import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "minesweeper-ppo_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
# exact fp32 convolutions for the fp32 parity tests (ms_amd.exact_fp32_convs), set before MIOpen
# runs anything; spawned test workers inherit it
os.environ.setdefault("MIOPEN_DEBUG_CONV_WINOGRAD", "0")
# the fp32 reference convolutions of the production-size parity tests run once per shape: MIOpen's
# heuristic (immediate) find instead of an exhaustive search per new shape
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def golden(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_files(pattern: str):
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, pattern)))


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.fail("gpu-marked test ran without a HIP device (run with -m 'not gpu' on CPU)")
    import torch
    return torch.device("cuda:0")
