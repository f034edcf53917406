"""Algorithm check of the device solver core on the CPU (no GPU needed).

tests/native/ipm_host_check.cpp compiles mpc_ros_amd/csrc/ipm_core.h -- the exact
code the HIP kernel runs per lane -- for the host, into a temporary directory (it is
never part of the product).  Its results must equal the oracle's fixtures: the
structured Riccati IPM follows the dense Ipopt restatement iterate for iterate.
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, params_from_array


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("hc") / "ipm_host_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-w", "-o", exe,
                           os.path.join(ROOT, "tests", "native", "ipm_host_check.cpp")])
    return exe


def run_harness(exe, P, state, coeffs, tol=1e-8, max_iter=3000):
    N = int(P["STEPS"])
    hdr = (f"{N} {P['DT']!r} {P['REF_CTE']!r} {P['REF_ETHETA']!r} {P['REF_V']!r} {P['W_CTE']!r} {P['W_EPSI']!r} "
           f"{P['W_V']!r} {P['W_ANGVEL']!r} {P['W_A']!r} {P['W_DANGVEL']!r} {P['W_DA']!r} {P['ANGVEL']!r} "
           f"{P['MAXTHR']!r} {P['BOUND']!r} {tol!r} {max_iter}\n{int(P.get('MODEL', 0))} {float(P.get('LF', 0.5))!r}\n"
           f"{len(state)}\n")
    body = "\n".join(" ".join(repr(float(v)) for v in np.concatenate([state[b], coeffs[b]]))
                     for b in range(len(state)))
    out = subprocess.run([exe], input=hdr + body + "\n", capture_output=True, text=True, check=True).stdout
    rows = np.array([r.split() for r in out.strip().split("\n")], dtype=np.float64)
    return dict(status=rows[:, 0].astype(int), iters=rows[:, 1].astype(int), obj=rows[:, 2], u0=rows[:, 3:5],
                traj=rows[:, 5:].reshape(len(state), 3, N))


def compare(r, g, atol=1e-9):
    np.testing.assert_array_equal(r["status"], g["status"])
    np.testing.assert_array_equal(r["iters"], g["iters"])
    np.testing.assert_allclose(r["u0"], g["u0"], rtol=0, atol=atol)
    np.testing.assert_allclose(r["traj"], g["traj"], rtol=0, atol=atol)
    np.testing.assert_allclose(r["obj"], g["obj"], rtol=1e-10, atol=1e-9)


def test_core_matches_oracle_infinity_set(harness, infinity_golden):
    g = infinity_golden
    r = run_harness(harness, params_from_array(g["params"]), g["state"], g["coeffs"])
    compare(r, g)


@pytest.mark.parametrize("name", ["class_defaults", "no_rate", "rate_w", "N40", "N3", "small_bound"])
def test_core_matches_oracle_variants(harness, variants_golden, name):
    g = variants_golden[name]
    r = run_harness(harness, params_from_array(g["params"]), g["state"], g["coeffs"])
    compare(r, g)


# ---------------------------------------------------------------- wavefront solver
# tests/native/wide_host_check.cpp runs mpc_ros_amd/csrc/wide_core.h (one problem per
# wavefront: stage-parallel sweeps, 64-lane Riccati) with 64 host threads standing in
# for the lanes.  Summation orders differ from the oracle's (tree reductions), so the
# comparison is to rounding: same status and iteration count, controls within 1e-9.
@pytest.fixture(scope="module")
def wide_harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("whc") / "wide_host_check")
    subprocess.check_call(["g++", "-O2", "-std=c++20", "-w", "-pthread", "-o", exe,
                           os.path.join(ROOT, "tests", "native", "wide_host_check.cpp")])
    return exe


def test_wide_core_matches_oracle_infinity_subset(wide_harness, infinity_golden):
    g = infinity_golden
    sel = np.r_[0:24, 256:264]  # course samples + edge cases
    sub = {k: g[k][sel] for k in ("state", "coeffs", "u0", "traj", "obj", "status", "iters")}
    r = run_harness(wide_harness, params_from_array(g["params"]), sub["state"], sub["coeffs"])
    compare(r, sub, atol=1e-9)


@pytest.mark.parametrize("name", ["class_defaults", "rate_w", "N40", "N3", "small_bound"])
def test_wide_core_matches_oracle_variants(wide_harness, variants_golden, name):
    g = variants_golden[name]
    n = 6
    sub = {k: g[k][:n] for k in ("state", "coeffs", "u0", "traj", "obj", "status", "iters")}
    r = run_harness(wide_harness, params_from_array(g["params"]), sub["state"], sub["coeffs"])
    compare(r, sub, atol=1e-9)


def test_wide_core_bicycle_matches_oracle(wide_harness, bicycle_golden):
    """Kinematic-bicycle variant (N = 25) through the wavefront solver."""
    g = bicycle_golden
    n = 12
    sub = {k: g[k][:n] for k in ("state", "coeffs", "u0", "traj", "obj", "status", "iters")}
    r = run_harness(wide_harness, g["P"], sub["state"], sub["coeffs"])
    compare(r, sub, atol=1e-9)


def _oracle_run(oracle, P, state, coeffs):
    return oracle.mpc_solve_batch(P, state, coeffs, opts=oracle.ipm_opts(tol=1e-8), nthreads=4)


def test_wide_core_full_width_N64(wide_harness, oracle):
    """STEPS = 64, the widest horizon the wavefront strategy takes (one stage per
    lane, every lane active), against the oracle on benchmark scenarios."""
    from mpc_ros_amd import infinity, params

    P = dict(params.PLUGIN_DEFAULTS, STEPS=64)
    sc = infinity.draw_scenarios(np.arange(200, 206))
    px, py, yaw, plan = infinity.scenario_poses(sc)
    st, cf = infinity.find_best_path(px, py, yaw, sc["v"], sc["w_prev"], sc["a_prev"], P["DT"], plan, True)
    g = _oracle_run(oracle, P, st, cf)
    r = run_harness(wide_harness, P, st, cf)
    compare(r, g, atol=1e-9)


def nonfinite_inputs():
    """NaN / inf in the state or the path polynomial, and a huge finite state."""
    st = np.tile(np.array([0.05, 0.0, 0.02, 0.4, 0.1, 0.05]), (6, 1))
    cf = np.tile(np.array([0.1, 0.02, -0.01, 0.001]), (6, 1))
    st[0, 3] = np.nan
    cf[1, 2] = np.inf
    st[2, 0] = 1e300
    cf[3, 0] = -np.inf
    st[4, 5] = np.nan
    return st, cf


def test_nonfinite_inputs_stop_with_invalid_number(harness, wide_harness, oracle):
    """A non-finite f or g at the starting point ends the solve before the first
    iteration with Ipopt's INVALID_NUMBER_DETECTED (11) -- no hang, no iterations --
    in the oracle and in both device cores; finite rows are unaffected."""
    from mpc_ros_amd import params

    P = params.PLUGIN_DEFAULTS
    st, cf = nonfinite_inputs()
    g = _oracle_run(oracle, P, st, cf)
    np.testing.assert_array_equal(g["status"][[0, 1, 3, 4]], 11)
    np.testing.assert_array_equal(g["iters"][[0, 1, 3, 4]], 0)
    assert g["status"][5] == 1
    for exe in (harness, wide_harness):
        r = run_harness(exe, P, st, cf)
        np.testing.assert_array_equal(r["status"], g["status"])
        np.testing.assert_array_equal(r["iters"], g["iters"])
        np.testing.assert_allclose(r["u0"], g["u0"], rtol=0, atol=1e-9)
