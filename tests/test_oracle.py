"""The oracle itself: pinned against the reference's known answer and the
reference's own AD library, and self-consistent with the committed fixtures."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_npz, params_from_array


def test_ldlt_solve_and_inertia(oracle):
    rng = np.random.default_rng(3)
    for _ in range(200):
        n = int(rng.integers(2, 40))
        A = rng.standard_normal((n, n))
        A = A + A.T
        z = int(rng.integers(0, n // 2 + 1))
        A[:z, :z] = 0.0
        ev = np.linalg.eigvalsh(A)
        if np.min(np.abs(ev)) < 1e-6 * np.max(np.abs(ev)):
            continue
        fac, ipiv, inertia = oracle.ldlt(A)
        b = rng.standard_normal(n)
        x = oracle.ldlt_solve(fac, ipiv, b)
        assert np.abs(A @ x - b).max() <= 1e-9 * (1 + np.abs(x).max())
        assert inertia == (int((ev > 0).sum()), int((ev < 0).sum()), 0)


def test_hs071_known_answer(oracle):
    """The reference's only known-answer test (assets/document/example/CppAD_Ipopt.cpp:146-150)."""
    with open(os.path.join(GOLDEN, "hs071.json")) as f:
        ka = json.load(f)
    r = oracle.hs071()
    assert r["status"] == 1
    for key in ("x", "zl", "zu"):
        np.testing.assert_allclose(r[key], ka[key], rtol=ka["rel_tol"], atol=ka["abs_tol"])
    assert r["iters"] == 8  # Ipopt's own HS071 iteration count


@pytest.mark.parametrize("N", [6, 20])
def test_nlp_derivatives_match_reference_cppad(oracle, N):
    """f, g, grad f, J_g and the Lagrangian Hessian of the restated FG_eval equal the
    values the reference's vendored CppAD computes for the same NLP."""
    z = load_npz("cppad_derivs.npz")
    P = params_from_array(z[f"N{N}_params"])
    for k in range(z[f"N{N}_x"].shape[0]):
        c, x = z[f"N{N}_coeffs"][k], z[f"N{N}_x"][k]
        sig, lam = z[f"N{N}_sigma"][k], z[f"N{N}_lambda"][k]
        fg = oracle.mpc_fg(P, c, x)
        np.testing.assert_allclose(fg, z[f"N{N}_fg"][k], rtol=1e-13, atol=1e-11)
        gf, J, H = oracle.mpc_derivs(P, c, x, 1.0, np.zeros(6 * N))
        np.testing.assert_allclose(gf, z[f"N{N}_jac"][k][0], rtol=1e-13, atol=1e-11)
        np.testing.assert_allclose(J, z[f"N{N}_jac"][k][1:], rtol=1e-13, atol=1e-11)
        # CppAD's Hessian weight vector is [sigma, lambda] (fg[0] is the objective)
        _, _, H = oracle.mpc_derivs(P, c, x, sig, lam)
        np.testing.assert_allclose(H, z[f"N{N}_hess"][k], rtol=1e-12, atol=1e-9)


def test_oracle_reproduces_fixtures(oracle, infinity_golden):
    g = infinity_golden
    P = params_from_array(g["params"])
    sel = np.r_[0:24, 256:264]
    r = oracle.mpc_solve_batch(P, g["state"][sel], g["coeffs"][sel], opts=oracle.ref_opts(int(P["STEPS"])))
    np.testing.assert_array_equal(r["status"], g["status"][sel])
    np.testing.assert_array_equal(r["iters"], g["iters"][sel])
    np.testing.assert_allclose(r["u0"], g["u0"][sel], rtol=0, atol=1e-12)
    np.testing.assert_allclose(r["traj"], g["traj"][sel], rtol=0, atol=1e-12)


def test_golden_solutions_are_kkt_points(oracle, infinity_golden):
    """Independent first-order certificate of the committed solutions."""
    g = infinity_golden
    P = params_from_array(g["params"])
    N = P["STEPS"]
    for b in range(0, 288, 9):
        if g["status"][b] != 1:
            continue
        # rebuild the full primal vector from the trajectory by integrating the dynamics
        x = full_primal(oracle, P, g["state"][b], g["coeffs"][b], g["traj"][b], g["u0"][b])
        if x is None:
            continue
        res = oracle.mpc_kkt_residual(P, g["state"][b], g["coeffs"][b], x)
        assert res["primal"] < 1e-8 and res["bound"] <= 1e-12


def full_primal(oracle, P, state, coeffs, traj, u0):
    r = oracle.mpc_solve(P, state, coeffs, opts=oracle.ref_opts(int(P["STEPS"])), full=True)
    if np.abs(r["traj"] - traj).max() > 1e-12:
        return None
    return r["x"]


def test_oracle_tight_tolerance_converges(oracle, infinity_golden):
    """At tol 1e-12 the oracle converges to the same local solution as at Ipopt's 1e-8."""
    g = infinity_golden
    P = params_from_array(g["params"])
    sel = np.arange(0, 64, 4)
    r = oracle.mpc_solve_batch(P, g["state"][sel], g["coeffs"][sel], opts=oracle.ipm_opts(tol=1e-12))
    ok = (g["status"][sel] == 1) & (r["status"] == 1)
    assert np.abs(r["u0"][ok] - g["u0"][sel][ok]).max() < 1e-6


def test_preprocess_restatement(oracle):
    z = load_npz("preprocess.npz")
    for b in range(z["pose"].shape[0]):
        px, py, yaw = z["pose"][b]
        v, w, a = z["vel"][b]
        rc, st, cf = oracle.find_best_path(px, py, yaw, v, w, a, float(z["dt"]), z["plan"][b], True)
        assert rc == 0
        np.testing.assert_allclose(st, z["state"][b], atol=1e-13)
        np.testing.assert_allclose(cf, z["coeffs"][b], atol=1e-13)
    rc, _, _ = oracle.find_best_path(0, 0, 0, 0, 0, 0, 0.1, np.zeros((0, 2)), True)
    assert rc == -1  # empty plan (driving_state.cpp:182-185)


@pytest.mark.parametrize("M", [64, 65, 300])
def test_preprocess_long_plans(oracle, M):
    """findBestPath takes any plan length: the oracle's QR beyond 64 waypoints (heap arrays)
    against a least-squares fit of the same vehicle-frame points (numpy lstsq)."""
    rng = np.random.default_rng(M)
    px, py, yaw = 0.3, -0.2, 0.4
    s = np.linspace(0.0, 4.0, M)
    hd = yaw + 0.2 * s
    plan = np.stack([px + np.cumsum(np.cos(hd)) * s[1], py + np.cumsum(np.sin(hd)) * s[1]], axis=1)
    plan += rng.normal(0, 1e-3, plan.shape)
    rc, st, cf = oracle.find_best_path(px, py, yaw, 0.5, 0.1, 0.2, 0.1, plan, False)
    assert rc == 0
    dx, dy = plan[:, 0] - px, plan[:, 1] - py
    xv = dx * np.cos(yaw) + dy * np.sin(yaw)
    yv = dy * np.cos(yaw) - dx * np.sin(yaw)
    ref = np.linalg.lstsq(np.vander(xv, 4, increasing=True), yv, rcond=None)[0]
    np.testing.assert_allclose(cf, ref, rtol=1e-8, atol=1e-9)
    assert st[4] == cf[0]  # cte = polyeval(c, 0) (no delay)


# --------------------------------------------------------- kinematic bicycle (model 1)
# No reference implementation exists: the NLP is pinned by its own
# derivative consistency (analytic vs central differences of fg) and by the KKT
# certificate of the committed solutions; parity unpinned against Ipopt.
def test_bicycle_derivatives_match_finite_differences(oracle, bicycle_golden):
    P = dict(bicycle_golden["P"], STEPS=6)
    N = 6
    nx, ng = 8 * N - 2, 6 * N
    rng = np.random.default_rng(3)
    c = bicycle_golden["coeffs"][0]
    x = rng.normal(scale=0.5, size=nx)
    lam = rng.normal(scale=5.0, size=ng)
    gf, J, H = oracle.mpc_derivs(P, c, x, 0.7, lam)
    h = 1e-6
    Jfd = np.zeros((1 + ng, nx))
    for i in range(nx):
        e = np.zeros(nx)
        e[i] = h
        Jfd[:, i] = (oracle.mpc_fg(P, c, x + e) - oracle.mpc_fg(P, c, x - e)) / (2 * h)
    np.testing.assert_allclose(gf, Jfd[0], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(J, Jfd[1:], rtol=1e-6, atol=1e-6)
    # Hessian of the Lagrangian by differences of the analytic gradients
    def grad_l(xx):
        g0, JJ, _ = oracle.mpc_derivs(P, c, xx, 0.7, lam)
        return 0.7 * g0 + JJ.T @ lam
    Hfd = np.zeros((nx, nx))
    for i in range(nx):
        e = np.zeros(nx)
        e[i] = h
        Hfd[:, i] = (grad_l(x + e) - grad_l(x - e)) / (2 * h)
    np.testing.assert_allclose(H, Hfd, rtol=1e-5, atol=1e-4)


def test_bicycle_fixtures_reproduce_and_certify(oracle, bicycle_golden):
    g = bicycle_golden
    P = g["P"]
    sel = np.arange(0, 64, 4)
    r = oracle.mpc_solve_batch(P, g["state"][sel], g["coeffs"][sel], opts=oracle.ref_opts(int(P["STEPS"])))
    np.testing.assert_array_equal(r["status"], g["status"][sel])
    np.testing.assert_array_equal(r["iters"], g["iters"][sel])
    np.testing.assert_allclose(r["u0"], g["u0"][sel], rtol=0, atol=1e-12)
    for b in sel[:6]:
        if g["status"][b] != 1:
            continue
        full = oracle.mpc_solve(P, g["state"][b], g["coeffs"][b], opts=oracle.ref_opts(int(P["STEPS"])), full=True)
        res = oracle.mpc_kkt_residual(P, g["state"][b], g["coeffs"][b], full["x"])
        assert res["primal"] < 1e-8 and res["bound"] <= 1e-12


def test_oracle_ipopt_mechanisms_fire_and_reproduce(oracle, features_golden):
    """The fixture of Ipopt's mechanisms (second-order corrections, watchdog, soft
    restoration, restoration phase) reproduces, and every mechanism acts on some problem;
    the results of problems that went through the restoration phase are KKT points."""
    seen = np.zeros(4, bool)
    for name in ("N20", "N40", "bicycle"):
        g = features_golden[name]
        P = g["P"]
        r = oracle.mpc_solve_batch(P, g["state"], g["coeffs"], opts=oracle.ref_opts(int(P["STEPS"])), diag=True)
        np.testing.assert_array_equal(r["status"], g["status"])
        np.testing.assert_array_equal(r["iters"], g["iters"])
        np.testing.assert_array_equal(r["diag"][:, :5], g["diag"])  # (the fixtures: the first five)
        np.testing.assert_allclose(r["u0"], g["u0"], rtol=0, atol=1e-12)
        seen |= (g["diag"][:, :4] > 0).any(0)
        for b in np.where(g["diag"][:, 3] > 0)[0][:3]:
            full = oracle.mpc_solve(P, g["state"][b], g["coeffs"][b], opts=oracle.ref_opts(int(P["STEPS"])), full=True)
            res = oracle.mpc_kkt_residual(P, g["state"][b], g["coeffs"][b], full["x"])
            assert res["primal"] < 1e-8 and res["dual"] < 1e-5
    assert seen.all(), seen


def test_oracle_cpu_time_budget(oracle, features_golden):
    """max_cpu_time 0.5 s (mpc_planner.cpp:368) as an iteration budget: > max_iter-free
    problems stop with unknown (14) once iter exceeds it (solve_callback.hpp:1165-1167)."""
    # CppAD's derivatives + Ipopt's own iteration (profiles/r3/cpu_iter_cost.json): 0.5 s is
    # 1520 iterations at N = 20, 737 at N = 40
    assert oracle.cpu_iter_budget(0.5, 20) == 1520 and oracle.cpu_iter_budget(0.5, 40) == 737
    assert oracle.cpu_iter_budget(1e6, 20) == -1
    g = features_golden["budget"]
    r = oracle.mpc_solve_batch(g["P"], g["state"], g["coeffs"],
                               opts=oracle.ref_opts(20, cpu_iter_budget=int(g["iter_budget"])))
    np.testing.assert_array_equal(r["status"], g["status"])
    assert set(np.unique(r["status"])) == {1, 14}
    assert r["iters"][r["status"] == 14].min() == int(g["iter_budget"]) + 1


def test_structured_kkt_same_iterates(oracle, infinity_golden):
    """kkt_structured (the CPU baseline's linear algebra: KKT rows in stage order, envelope
    Bunch-Kaufman) follows the checker's iterates: same statuses and iteration counts,
    controls to rounding (a different pivot order)."""
    g = infinity_golden
    sel = np.r_[0:24, 256:264]
    P = params_from_array(g["params"])
    o = oracle.ref_opts(20)
    o.kkt_structured = 1
    r = oracle.mpc_solve_batch(P, g["state"][sel], g["coeffs"][sel], opts=o, nthreads=4)
    np.testing.assert_array_equal(r["status"], g["status"][sel])
    np.testing.assert_array_equal(r["iters"], g["iters"][sel])
    ok = g["status"][sel] == 1
    np.testing.assert_allclose(r["u0"][ok], g["u0"][sel][ok], rtol=0, atol=1e-12)


def test_iterative_refinement_changes_no_fixture_row(oracle, infinity_golden, features_golden):
    """Ipopt refines every KKT solve at least once (PDFullSpaceSolver, min_refinement_steps 1,
    residual_ratio_max 1e-10); the oracle's fixtures and the device solve without it.  With the
    refinement restated (ora_ipm_opts.refine_steps = 1) the infinity set and every Ipopt-feature
    set (SOC, watchdog, soft restoration, the restoration phase at N = 20 and 40, the bicycle)
    keep every status, iteration count and restoration count, and u0 moves by rounding only
    (measured: <= 3.2e-15): the dense factorisation is accurate without it.  (The locally
    infeasible small_bound variant, 5-13 restoration phases at condition numbers up to ~1e20, is
    the exception: one row of 16 takes 68 iterations instead of 67, u0 within 1e-11.)  The
    device's reduced restoration solve is not that accurate and refines every restoration step
    (wide_core.h refine_resto; tests/test_core_host.py SMALL_BOUND_ITERS_EXACT)."""
    sets = [("infinity", infinity_golden, 20, slice(0, 96))]
    for name in ("N20", "N40", "bicycle", "resto_N20", "resto_N40"):
        g = features_golden[name]
        sets.append((name, g, int(g["P"]["STEPS"]), slice(None)))
    for name, g, N, sl in sets:
        P = g["P"] if "P" in g else params_from_array(g["params"])
        r = oracle.mpc_solve_batch(P, g["state"][sl], g["coeffs"][sl], opts=oracle.ref_opts(N, refine_steps=1),
                                   nthreads=8, diag=True)
        np.testing.assert_array_equal(r["status"], g["status"][sl], err_msg=name)
        np.testing.assert_array_equal(r["iters"], g["iters"][sl], err_msg=name)
        np.testing.assert_array_equal(r["diag"][:, 3], g["diag"][sl, 3], err_msg=name)
        np.testing.assert_allclose(r["u0"], g["u0"][sl], rtol=0, atol=1e-13, err_msg=name)


def test_unrestated_ipopt_paths_never_reached(oracle, infinity_golden, features_golden, variants_golden):
    """Two parts of Ipopt 3.12 are not restated (oracle/ipm.c header), and this shows no fixture
    row reaches them:
    - the slack move (IpoptCalculatedQuantities::CalculateSafeSlack, then AcceptTrialPoint's
      AdjustedTrialSlacks bound relaxation) acts on a slack below eps * min(1, mu); the oracle
      records the smallest slack / (eps min(1, mu)) of every point whose barrier it evaluates,
      original and restoration problem: no point falls below 1 (measured: >= 1e8 on every set but
      the locally infeasible small_bound, 1e3 there);
    - the restoration phase of the restoration problem (RestoRestorationPhase) runs only where the
      restoration problem's line search fails, which is where the oracle (and the device) return
      RESTORATION_FAILURE (9): no row ends with 9."""
    sets = [("infinity", infinity_golden, None)]
    for name in ("N20", "N40", "bicycle", "resto_N20", "resto_N40"):
        sets.append((name, features_golden[name], None))
    for name in ("class_defaults", "no_rate", "rate_w", "N40", "N3", "small_bound", "N80", "N100"):
        sets.append((name, variants_golden[name], None))
    worst = []
    for name, g, _ in sets:
        P = g["P"] if "P" in g else params_from_array(g["params"])
        r = oracle.mpc_solve_batch(P, g["state"], g["coeffs"], opts=oracle.ref_opts(int(P["STEPS"])), nthreads=8,
                                   diag=True)
        np.testing.assert_array_equal(r["status"], g["status"], err_msg=name)
        assert (r["diag"][:, 5] == 0).all(), (name, np.flatnonzero(r["diag"][:, 5]))
        assert (r["status"] != 9).all(), name
        worst.append((name, int(r["diag"][:, 6].min())))
    print("floor(log10(smallest slack margin)) per set:", worst)
    assert min(w for _, w in worst) >= 0


def test_small_bound_iteration_counts_depend_on_the_linear_algebra(oracle, variants_golden):
    """On the locally infeasible small_bound set (BOUND = 0.4: 5-13 restoration phases per row,
    restoration Newton systems at condition numbers up to ~1e20) the iteration count is not fixed
    by the algorithm alone.  The oracle under two restatements of Ipopt's linear algebra that are
    equally faithful to it -- the KKT matrix in stage order (kkt_structured, another pivot order
    for the Bunch-Kaufman factorisation, as MUMPS' ordering is neither) and Ipopt's own iterative
    refinement of every solve (refine_steps = 1: PDFullSpaceSolver's min_refinement_steps default)
    -- keeps every status, restoration count and control (1e-10) and ends row 8 one iteration
    later than the fixture (68 against 67); an FMA-contracted build of the same C does too.  The
    device's reduced restoration solve differs from all of them in the same last digits, more so
    where its refinement contracts slowly (tests/test_core_host.py SMALL_BOUND_ITERS_*)."""
    g = variants_golden["small_bound"]
    P = params_from_array(g["params"])
    iters = {}
    for name, kw in (("dense", {}), ("structured", {"kkt_structured": 1}), ("refined", {"refine_steps": 1})):
        r = oracle.mpc_solve_batch(P, g["state"], g["coeffs"], opts=oracle.ref_opts(20, **kw), nthreads=8, diag=True)
        np.testing.assert_array_equal(r["status"], g["status"], err_msg=name)
        np.testing.assert_array_equal(r["diag"][:, 3], g["diag"][:, 3], err_msg=name)
        np.testing.assert_allclose(r["u0"], g["u0"], rtol=0, atol=1e-10, err_msg=name)
        iters[name] = r["iters"]
    np.testing.assert_array_equal(iters["dense"], g["iters"])
    spread = np.abs(np.stack(list(iters.values())) - g["iters"]).max(0)
    print("iteration-count spread per row across the oracle's variants:", spread.tolist())
    assert spread.max() >= 1 and spread.max() <= 1
    assert int(np.flatnonzero(spread)[0]) == 8
