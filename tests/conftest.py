"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def load_npz(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def params_from_array(arr) -> dict:
    from mpc_ros_amd.params import KEYS

    d = {k: float(v) for k, v in zip(KEYS, arr)}
    d["STEPS"] = int(d["STEPS"])
    return d


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle

    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def infinity_golden():
    return load_npz("infinity_N20.npz")


@pytest.fixture(scope="session")
def variants_golden():
    z = load_npz("variants.npz")
    out = {}
    for k, v in z.items():
        if "__" in k:
            name, field = k.split("__", 1)
            out.setdefault(name, {})[field] = v
    return out


@pytest.fixture(scope="session")
def bicycle_golden():
    """Kinematic-bicycle variant (tests/golden/bicycle_N25.npz): params dict includes MODEL/LF."""
    g = load_npz("bicycle_N25.npz")
    P = params_from_array(g["params"])
    P["MODEL"] = int(g["model"])
    P["LF"] = float(g["lf"])
    g["P"] = P
    return g


@pytest.fixture(scope="session")
def features_golden():
    """tests/golden/ipopt_features.npz split by set (N20, N40, bicycle, budget); each set
    carries its parameter dict as "P"."""
    z = load_npz("ipopt_features.npz")
    out = {}
    for k, v in z.items():
        if "__" in k:
            name, field = k.split("__", 1)
            out.setdefault(name, {})[field] = v
    for name, g in out.items():
        P = params_from_array(g["params"])
        if name == "bicycle":
            P.update(MODEL=1, LF=0.5)
        g["P"] = P
    return out


@pytest.fixture(scope="session")
def libmpcg():
    from mpc_ros_amd import build, _lib

    build.build()
    return _lib.lib()
