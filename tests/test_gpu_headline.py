"""GPU parity of the kernel instances the benchmark and the BASELINE configurations time.

The dispatcher picks an instance by batch size (mpcg_wide.hip wide_kernel): the benchmark
configuration (N = 20, default Ipopt options) runs k_solve_wide<0,true,double,1,true,2>
with the expected-longest-first solve order for B > 4,096, and the 512-VGPR
k_solve_wide<0,true,double,1,true,1> for smaller batches -- the one every fixture-sized
test exercises.  Here every default-option N = 20 fixture row (infinity set, Ipopt-feature
set, restoration set) goes through the large-batch instance inside a batch of 8,192, padded
with fresh problems that are checked against the oracle as well; mpcg_last_kernel() says which
instance ran.  The same for the bicycle (configs[4]) and the fp32 solver (configs[2]) at
B > 4,096.  Reference call: mpc_ros/src/mpc_planner.cpp:373-401.

Tolerance as tests/test_gpu_parity.py: same status, iteration count and restoration count on
every row, u0 / trajectory within 1e-7.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

from conftest import params_from_array
from test_gpu_parity import ATOL, check_against, oracle_ref

pytestmark = pytest.mark.gpu

HEADLINE = "k_solve_wide<0,true,double,1,true,2>"
LONE = "k_solve_wide<0,true,double,1,true,1>"
B_BIG = 8192


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    return torch


def _solver(P, **kw):
    from mpc_ros_amd.solver import BatchSolver

    return BatchSolver(0, P, **kw)


def _fixture_rows(infinity_golden, features_golden):
    """Every default-option N = 20 fixture row: (state, coeffs, expected dict)."""
    sets = [infinity_golden, features_golden["N20"], features_golden["resto_N20"]]
    exp = {}
    for k in ("u0", "traj", "status", "iters", "obj"):
        exp[k] = np.concatenate([g[k] for g in sets])
    exp["diag"] = np.concatenate([g["diag"] for g in sets])
    st = np.concatenate([g["state"] for g in sets])
    cf = np.concatenate([g["coeffs"] for g in sets])
    return st, cf, exp


def _padded(st, cf, B, seed, base):
    """The fixture rows scattered over a batch of B, the rest fresh infinity-set problems."""
    from mpc_ros_amd import infinity

    rng = np.random.default_rng(seed)
    pos = np.sort(rng.choice(B, len(st), replace=False))
    rest = np.setdiff1d(np.arange(B), pos)
    fst, fcf = infinity.make_problems(base + np.arange(len(rest)))
    S = np.empty((B, 6))
    C = np.empty((B, 4))
    S[pos], C[pos] = st, cf
    S[rest], C[rest] = fst, fcf
    return S, C, pos, rest


def _sub(r, idx):
    return {k: r[k][idx] for k in ("u0", "traj", "status", "obj", "iters", "diag")}


def test_headline_instance_every_fixture_row(torch_cuda, infinity_golden, features_golden, oracle):
    """All 302 default-option N = 20 fixture rows (and 7,890 fresh problems against the
    oracle) through the benchmark's instance, in its solve order."""
    from mpc_ros_amd import params

    P = params.PLUGIN_DEFAULTS
    assert params_from_array(infinity_golden["params"]) == P
    st, cf, exp = _fixture_rows(infinity_golden, features_golden)
    S, C, pos, rest = _padded(st, cf, B_BIG, 4, 2_000_000)
    s = _solver(P)
    r = s.solve(S, C)
    assert s.last_kernel == HEADLINE
    check_against(_sub(r, pos), exp)
    assert (r["diag"][pos, 0] >= 1).sum() == (exp["diag"][:, 3] >= 1).sum() >= 5  # (restoration rows)
    ref = oracle_ref(oracle, P, S[rest], C[rest])
    check_against(_sub(r, rest), ref)


@pytest.mark.parametrize("B", [4096, 2049])
def test_configs1_dispatch_every_fixture_row(torch_cuda, infinity_golden, features_golden, oracle, B):
    """BASELINE configs[1] (B = 4,096, N = 20, fp64) exactly as dispatched: the 512-VGPR
    instance with the expected-longest-first solve order (B > 2,048).  All 302 default-option
    N = 20 fixture rows inside the batch and every fresh problem of it against the oracle; the
    same at B = 2,049, the smallest batch that is ordered."""
    from mpc_ros_amd import params

    P = params.PLUGIN_DEFAULTS
    st, cf, exp = _fixture_rows(infinity_golden, features_golden)
    S, C, pos, rest = _padded(st, cf, B, 9, 7_000_000 + B)
    s = _solver(P)
    r = s.solve(S, C)
    assert s.last_kernel == LONE and s.last_solve_order
    check_against(_sub(r, pos), exp)
    check_against(_sub(r, rest), oracle_ref(oracle, P, S[rest], C[rest]))
    # (results do not depend on the order: an unordered solve of the fixture rows alone)
    alone = s.solve(st, cf)
    assert not s.last_solve_order
    np.testing.assert_array_equal(alone["u0"], r["u0"][pos])


def test_small_batches_run_the_lone_instance(torch_cuda, infinity_golden):
    """B <= 4,096 runs the 512-VGPR instance (the fixture-sized tests' instance)."""
    g = infinity_golden
    s = _solver(params_from_array(g["params"]))
    s.solve(g["state"][:64], g["coeffs"][:64])
    assert s.last_kernel == LONE and not s.last_solve_order


def test_bicycle_instance_at_large_batch(torch_cuda, bicycle_golden, features_golden, oracle):
    """configs[4] (bicycle, N = 25) at B = 8,192: every bicycle fixture row inside the batch."""
    g, f = bicycle_golden, features_golden["bicycle"]
    st = np.concatenate([g["state"], f["state"]])
    cf = np.concatenate([g["coeffs"], f["coeffs"]])
    exp = {k: np.concatenate([g[k], f[k]]) for k in ("u0", "traj", "status", "iters", "obj", "diag")}
    S, C, pos, rest = _padded(st, cf, B_BIG, 5, 3_000_000)
    s = _solver(g["P"])
    r = s.solve(S, C)
    assert s.last_kernel == "k_solve_wide<1,true,double,1,true,2>"
    check_against(_sub(r, pos), exp)
    sample = rest[:: len(rest) // 256][:256]
    check_against(_sub(r, sample), oracle_ref(oracle, g["P"], S[sample], C[sample]))


def test_fp32_instance_at_large_batch(torch_cuda, variants_golden):
    """configs[2]'s instance (fp32, N = 40, then the fp64 phase) at B = 8,192: the N = 40 fixtures
    inside the batch, within the tolerance of tests/test_gpu_fp32.py (every row); the rows equal a
    solo solve of them (results do not depend on batch position)."""
    g = variants_golden["N40"]
    P = params_from_array(g["params"])
    S, C, pos, _ = _padded(g["state"], g["coeffs"], B_BIG, 6, 4_000_000)
    s = _solver(P, dtype="fp32")
    r = s.solve(S, C)
    assert s.last_kernel == "k_solve_wide<0,false,float,1,false,3>"
    alone = s.solve(g["state"], g["coeffs"])
    np.testing.assert_array_equal(r["u0"][pos], alone["u0"])
    np.testing.assert_array_equal(r["status"][pos], alone["status"])
    du = np.abs(r["u0"][pos] - g["u0"]).max(1)
    assert du.max() <= 1e-3 and np.isin(r["status"], (1, 4)).all()


def test_park_area_overflow_matches_oracle(torch_cuda, features_golden, infinity_golden):
    """A park area of one entry: the restoration rows beyond it go to the overflow list and are
    solved again from the start after the drain (diag[:, 2] == 2); results equal the fixtures
    (Ipopt runs the restoration phase for every one of them)."""
    st, cf, exp = _fixture_rows(infinity_golden, features_golden)
    S, C, pos, _ = _padded(st, cf, B_BIG, 7, 5_000_000)
    from mpc_ros_amd import params

    s = _solver(params.PLUGIN_DEFAULTS)
    s.set_park_capacity(1)
    r = s.solve(S, C)
    check_against(_sub(r, pos), exp)
    d2 = r["diag"][:, 2]
    assert (d2 == 1).sum() <= 1 and (d2 == 2).sum() >= 4
    assert ((d2 > 0) == (r["diag"][:, 0] > 0)).all()
    s.set_park_capacity(0)
    r2 = s.solve(S, C)
    np.testing.assert_array_equal(r2["u0"], r["u0"])
    assert (r2["diag"][:, 2] == 2).sum() == 0


def test_graph_capture_and_replay(torch_cuda, infinity_golden, features_golden):
    """The solve (solve order, batch kernel, resume workers forked on the aux stream, drain) is
    captured in a HIP graph and replayed: the same results as a direct solve, and a replay takes
    about as long (a graph executor that runs the forked workers before the batch kernel would
    have them exit after ~2 ms instead of spinning)."""
    torch = torch_cuda
    from mpc_ros_amd import params

    P = params.PLUGIN_DEFAULTS
    st, cf, exp = _fixture_rows(infinity_golden, features_golden)
    S, C, pos, _ = _padded(st, cf, B_BIG, 8, 6_000_000)
    dev = torch.device("cuda:0")
    s = _solver(P)
    s.reserve(B_BIG)
    tst, tcf = torch.from_numpy(S).to(dev), torch.from_numpy(C).to(dev)
    u0 = torch.empty((B_BIG, 2), dtype=torch.float64, device=dev)
    status = torch.empty(B_BIG, dtype=torch.int32, device=dev)
    iters = torch.empty(B_BIG, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        s.solve_device(tst, tcf, u0, status=status, iters=iters)  # (warm-up on the capture stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        s.solve_device(tst, tcf, u0, status=status, iters=iters)
    torch.cuda.synchronize()
    direct_s = time.perf_counter() - t0
    ref = (u0.cpu().numpy().copy(), status.cpu().numpy().copy(), iters.cpu().numpy().copy())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):  # (the handle's previous stream: no cross-stream wait)
        s.solve_device(tst, tcf, u0, status=status, iters=iters)
    for _ in range(2):
        u0.zero_()
        status.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        replay_s = time.perf_counter() - t0
        np.testing.assert_array_equal(u0.cpu().numpy(), ref[0])
        np.testing.assert_array_equal(status.cpu().numpy(), ref[1])
        np.testing.assert_array_equal(iters.cpu().numpy(), ref[2])
        assert replay_s < max(0.5, 3 * direct_s), (replay_s, direct_s)
    np.testing.assert_allclose(ref[0][pos], exp["u0"], rtol=0, atol=ATOL)
    np.testing.assert_array_equal(ref[1][pos], exp["status"])
