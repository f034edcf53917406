"""The bench line's contract on the GPU: `python bench.py` (a short run) prints one JSON line
with BASELINE.json's metric and the fields the driver and the judge read -- value, unit,
n_gpus, steps, warmup, ms_per_step, higher_is_better, scaling, vs_baseline, dtype, data,
config.workload, and the roofline and cpu_baseline objects (ROUND contract, item ④)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_line_contract():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--cpu-seconds", "1"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"] and d["unit"] == "solves/s"
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["dtype"] == "f64" and "synthetic" in d["data"] and d["config"]["workload"]
    # value = whole-job solves / s over the timed steps
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - 65536 / (d["ms_per_step"] * 1e-3)) <= 0.02 * d["value"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"])
    assert rf["traffic"] is None or rf["traffic"] > 0
    assert rf["kernel_ms"] <= d["ms_per_step"] * 1.01  # (the kernel inside the step)
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["value"] > 0 and cb["cores"] >= 1
