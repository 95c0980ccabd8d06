"""Shared pytest setup: the `gpu` marker, package/oracle loaders and golden fixtures."""
from __future__ import annotations

import hashlib
import importlib.util
import json
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"
PKG_DIR = ROOT / "real-time-sdr_amd"

if str(ROOT / "oracle") not in sys.path:
    sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def load_pkg():
    """Import the product package `real-time-sdr_amd/` as `real_time_sdr_amd`."""
    if "real_time_sdr_amd" in sys.modules:
        return sys.modules["real_time_sdr_amd"]
    spec = importlib.util.spec_from_file_location(
        "real_time_sdr_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["real_time_sdr_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc
    orc.lib()
    return orc


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(GOLD / "golden_mode0.npz"))


@pytest.fixture(scope="session")
def golden_long():
    return json.loads((GOLD / "golden_mode0_long.json").read_text())


@pytest.fixture(scope="session")
def synth(pkg):
    import real_time_sdr_amd.synth as s
    return s


_INPUT_CACHE: dict = {}


def channel_input(synth_mod, ch: int, nblocks: int, expect_sha: str | None = None) -> np.ndarray:
    key = (ch, nblocks)
    if key not in _INPUT_CACHE:
        src = synth_mod.FMMultiplexSource(ch)
        _INPUT_CACHE[key] = np.stack([src.next_block() for _ in range(nblocks)])
    iq = _INPUT_CACHE[key]
    if expect_sha is not None:
        assert sha(iq) == expect_sha, "synthetic input drifted from the one the golden vectors were made on"
    return iq
