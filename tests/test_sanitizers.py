"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the
oracle's C restatement (tests/native/oracle_san_check.c) and the solver core's host
emulation (tests/native/wide_host_check.cpp, the code the HIP kernel runs) on small
problems.  GPU sanitizers are not available on this pool; the device code's host
emulation is what runs here.  Any sanitizer report fails the run (halt_on_error)."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_san")
    src = [os.path.join(ROOT, "oracle", f) for f in ("ldlt.c", "ipm.c", "nlp_mpc.c", "nlp_hs071.c", "preprocess.c")]
    subprocess.check_call(["gcc", "-std=c11", "-D_DEFAULT_SOURCE", *SAN, f"-I{os.path.join(ROOT, 'oracle')}", "-o", exe,
                           os.path.join(ROOT, "tests", "native", "oracle_san_check.c"), *src, "-lm"])
    r = subprocess.run([exe], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert r.stdout.count("status 1 ") >= 5


def test_wide_core_host_emulation_under_asan_ubsan(tmp_path, variants_golden):
    from test_core_host import compare, run_harness

    from conftest import params_from_array

    exe = str(tmp_path / "whc_san")
    subprocess.check_call(["g++", "-std=c++20", "-w", "-pthread", *SAN, "-o", exe,
                           os.path.join(ROOT, "tests", "native", "wide_host_check.cpp")])
    g = variants_golden["N3"]
    sub = {k: g[k][:2] for k in ("state", "coeffs", "u0", "traj", "obj", "status", "iters", "diag")}
    old = dict(os.environ)
    os.environ.update(ASAN_OPTIONS=ENV["ASAN_OPTIONS"], UBSAN_OPTIONS=ENV["UBSAN_OPTIONS"])
    try:
        r = run_harness(exe, params_from_array(g["params"]), sub["state"], sub["coeffs"])
    finally:
        os.environ.clear()
        os.environ.update(old)
    compare(r, sub, atol=1e-9)
