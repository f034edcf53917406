"""The measurement scripts the bench line's figures come from (CPU, synthetic inputs): the PMC
summary that bench.py reads roofline.traffic from, the static ISA census and the kernel-trace
timeline.  No GPU: the inputs are hand-made rocprofv3 CSVs and an assembly snippet in the
formats those tools read."""
from __future__ import annotations

import csv
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

TOOLS = os.path.join(ROOT, "tools")


def _write_pass(root, name, rows):
    d = os.path.join(root, name, "host", "")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "1_counter_collection.csv")
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value",
                                          "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _dispatch(did, kernel, counters, t0, ms):
    return [dict(Dispatch_Id=did, Kernel_Name=kernel, Counter_Name=c, Counter_Value=v, Start_Timestamp=t0,
                 End_Timestamp=t0 + int(ms * 1e6)) for c, v in counters.items()]


def test_pmc_summary_keeps_the_batch_instance(tmp_path):
    """configs[2] launches two instances of k_solve_wide (the fp32 batch and the fp64 head of 64
    problems): the summary averages only the one with the most GPU time, per pass."""
    batch = "void mpcg::k_solve_wide<0, false, float, 1, false, 3>(mpcg::WideArgs)"
    head = "void mpcg::k_solve_wide<0, false, double, 1, true, 2>(mpcg::WideArgs)"
    root = str(tmp_path / "pmc")
    _write_pass(root, "write", _dispatch(1, head, {"WRITE_SIZE": 100.0}, 0, 5.0) +
                _dispatch(2, batch, {"WRITE_SIZE": 1000.0}, 0, 25.0) +
                _dispatch(3, "mpcg::k_reset_ws(int*)", {"WRITE_SIZE": 7.0}, 0, 0.01))
    _write_pass(root, "fetch", _dispatch(1, head, {"FETCH_SIZE": 10.0}, 0, 5.0) +
                _dispatch(2, batch, {"FETCH_SIZE": 40.0}, 0, 25.0))
    _write_pass(root, "lds", _dispatch(1, head, {"SQ_WAVES": 64.0, "SQ_LDS_BANK_CONFLICT": 1.0,
                                                 "SQ_LDS_IDX_ACTIVE": 2.0}, 0, 5.0) +
                _dispatch(2, batch, {"SQ_WAVES": 65472.0, "SQ_LDS_BANK_CONFLICT": 30.0,
                                     "SQ_LDS_IDX_ACTIVE": 200.0}, 0, 25.0))
    out = str(tmp_path / "summary.json")
    subprocess.run([sys.executable, os.path.join(TOOLS, "pmc_summary.py"), root, out, "--batch", "65536"], check=True,
                   capture_output=True)
    d = json.load(open(out))
    c = d["counters_per_dispatch"]
    assert c["WRITE_SIZE"] == 1000.0 and c["FETCH_SIZE"] == 40.0 and c["SQ_WAVES"] == 65472.0
    assert d["write_bytes"] == 1000.0 * 1024 and d["fetch_bytes_corrected"] == 2 * 40.0 * 1024
    assert d["hbm_bytes_per_launch"] == 2 * 40.0 * 1024 + 1000.0 * 1024
    assert d["lds_bank_conflict_frac"] == pytest.approx(0.15)
    assert d["dispatch_s"] == pytest.approx(0.025)


def test_isa_census_separates_spill_reloads(tmp_path):
    """Lane reads out of the VGPRs that v_writelane fills (the SGPR spills) are counted apart from
    the solver's own v_readlane broadcasts."""
    sym = "_ZN4mpcg12k_solve_wideTEST"
    asm = "\n".join([
        f"{sym}:",
        "\tv_writelane_b32 v200, s4, 0",
        "\tv_writelane_b32 v200, s5, 1",
        "\tv_fma_f64 v[0:1], v[2:3], v[4:5], v[6:7]",
        "\tv_readlane_b32 s4, v200, 0",
        "\tv_readlane_b32 s5, v200, 1",
        "\tv_readlane_b32 s6, v7, 3",
        "\tv_mov_b32_dpp v1, v2 row_shr:1 row_mask:0xf bank_mask:0xf",
        "\tv_mov_b64 v[8:9], v[10:11]",
        "\tds_read_b128 v[0:3], v4",
        "\ts_endpgm",
        ".Lfunc_end0:",
        "",
    ])
    p = tmp_path / "k.s"
    p.write_text(asm)
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "isa_census.py"), str(p), sym], check=True,
                       capture_output=True, text=True).stdout
    assert "8 VALU instructions" in r
    assert "2 spill writes, 2 reloads; 1 other v_readlane" in r
    assert "fp64 arithmetic" in r and "dpp" in r and "LDS" in r


def test_trace_timeline_orders_dispatches(tmp_path):
    """The kernel-trace timeline: every dispatch from 2 ms before the last fp32 batch launch to the
    end of the fp64 phase after it, in ms relative to the batch launch's start."""
    path = tmp_path / "kernel_trace.csv"
    rows = [("mpcg::k_reset_ws(int*)", 999_000_000, 999_010_000),
            ("mpcg::k_reset_ws(int*)", 990_000_000, 990_010_000),  # (before the window: left out)
            ("void mpcg::k_solve_wide<0, false, float, 1, false, 3>(mpcg::WideArgs)", 1_000_000_000, 1_025_000_000),
            ("void mpcg::k_solve_wide<0, false, double, 1, true, 2>(mpcg::WideArgs)", 999_990_000, 1_005_000_000),
            ("void mpcg::k_warm_wide<0, false, double, 1, true, 2>(mpcg::WideArgs)", 1_025_100_000, 1_033_600_000)]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Queue_Id"])
        for n, s, e in rows:
            w.writerow([n, s, e, 64, 1])
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "trace_timeline.py"), str(path)], check=True,
                       capture_output=True, text=True).stdout.strip().split("\n")
    assert len(r) == 4
    assert r[0].split()[0] == "-1.000" and "k_reset_ws" in r[0]
    assert r[2].split()[:2] == ["0.000", "25.000"] and "float" in r[2]
    assert "k_warm_wide" in r[3] and r[3].split()[2] == "8.500"
