"""Generate the committed golden fixtures under tests/golden/.

Run in the development container (needs /root/reference for the CppAD part):

    python tests/golden/make_goldens.py

Fixtures (data only -- inputs and expected outputs):
  cppad_derivs.npz   f, g, grad f, J_g, Lagrangian Hessian of the reference NLP at
                     seeded points, computed by the reference's vendored CppAD
                     (oracle/ref_probe/cppad_fg.cpp -> oracle/_ref/cppad_fg)
  hs071.json         the reference's known answer (assets/document/example/CppAD_Ipopt.cpp:146-150)
  infinity_N20.npz   256 infinity-set problems + 32 edge cases, plugin defaults,
                     solved by the oracle (Ipopt restatement, Ipopt default options)
  variants.npz       other parameter sets (class defaults, W_DA = 0, rate penalty on w,
                     N = 40, N = 3, small BOUND with active state bounds, N = 80, N = 100)
  preprocess.npz     findBestPath inputs (poses, waypoints) and the oracle's outputs
  bicycle_N25.npz    the kinematic-bicycle variant (BASELINE configs[4]; no reference
                     implementation exists, so this pins the build's own restatement):
                     64 infinity-set problems, N = 25, MODEL = 1, LF = 0.5, ANGVEL = 0.5
  ipopt_features.npz problems of the infinity set on which Ipopt's second-order
                     corrections, watchdog, soft restoration and restoration phase act
                     (found by scanning with the oracle's diagnostics), the problems the
                     round-1 advisor named for the bounded filter (16101, 1887), and the
                     max_cpu_time iteration budget forced low; per problem the parameter
                     set (N20 / N40 / bicycle), the oracle's diagnostics and results

All solves use the reference's options (oracle.pyoracle.ref_opts: Ipopt 3.12 defaults,
max_cpu_time 0.5 s as its iteration budget).

    python tests/golden/make_goldens.py [set ...]     (default: all sets)
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as O  # noqa: E402
from mpc_ros_amd import infinity, params  # noqa: E402

PLUGIN = params.PLUGIN_DEFAULTS


def cppad_derivs():
    probe = os.path.join(ROOT, "oracle", "_ref", "cppad_fg")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    rng = np.random.default_rng(7)
    out = {}
    for N, K in ((6, 8), (20, 2)):
        P = dict(PLUGIN, STEPS=N, W_DANGVEL=30.0)
        nx, ng = 8 * N - 2, 6 * N
        st, cf = infinity.make_problems(np.arange(100, 100 + K))
        X = rng.normal(scale=0.6, size=(K, nx))
        SIG = rng.uniform(0.2, 2.0, size=K)
        LAM = rng.normal(scale=50.0, size=(K, ng))
        hdr = (f"{N} {P['DT']} {P['REF_CTE']} {P['REF_ETHETA']} {P['REF_V']} {P['W_CTE']} {P['W_EPSI']} "
               f"{P['W_V']} {P['W_ANGVEL']} {P['W_A']} {P['W_DANGVEL']} {P['W_DA']}\n{K}\n")
        body = []
        for k in range(K):
            body.append(" ".join(repr(float(v)) for v in np.concatenate([cf[k], X[k], [SIG[k]], LAM[k]])))
        res = subprocess.run([probe], input=hdr + "\n".join(body) + "\n", capture_output=True, text=True,
                             check=True).stdout.split()
        vals = np.array(res, dtype=np.float64).reshape(K, -1)
        o = 0
        fg = vals[:, o:o + 1 + ng]; o += 1 + ng
        jac = vals[:, o:o + (1 + ng) * nx].reshape(K, 1 + ng, nx); o += (1 + ng) * nx
        hes = vals[:, o:o + nx * nx].reshape(K, nx, nx)
        out[f"N{N}_params"] = np.array([P[k] for k in params.KEYS])
        out[f"N{N}_coeffs"] = cf
        out[f"N{N}_x"] = X
        out[f"N{N}_sigma"] = SIG
        out[f"N{N}_lambda"] = LAM
        out[f"N{N}_fg"] = fg
        out[f"N{N}_jac"] = jac
        out[f"N{N}_hess"] = hes
    out["keys"] = np.array(params.KEYS)
    np.savez_compressed(os.path.join(HERE, "cppad_derivs.npz"), **out)


def solve_set(P, st, cf, opts=None):
    r = O.mpc_solve_batch(P, st, cf, opts=opts or O.ref_opts(int(P["STEPS"])), nthreads=os.cpu_count() or 8,
                          diag=True)
    return dict(state=st, coeffs=cf, u0=r["u0"], traj=r["traj"], obj=r["obj"], status=r["status"],
                iters=r["iters"], diag=r["diag"], params=np.array([P[k] for k in params.KEYS]))


def infinity_set():
    st, cf = infinity.make_problems(np.arange(256))
    est, ecf = infinity.problems_from_scenarios(infinity.edge_scenarios())
    st = np.concatenate([st, est])
    cf = np.concatenate([cf, ecf])
    d = solve_set(PLUGIN, st, cf)
    d["index"] = np.concatenate([np.arange(256), -1 - np.arange(32)])
    np.savez_compressed(os.path.join(HERE, "infinity_N20.npz"), **d)
    print("infinity_N20 status:", np.unique(d["status"], return_counts=True), "iters mean", d["iters"].mean())


VARIANTS = {
    "class_defaults": (params.CLASS_DEFAULTS, 64, 1000),
    "no_rate": (dict(PLUGIN, W_DA=0.0), 64, 2000),
    "rate_w": (dict(PLUGIN, W_DANGVEL=50.0), 32, 3000),
    "N40": (dict(PLUGIN, STEPS=40), 24, 4000),
    "N3": (dict(PLUGIN, STEPS=3), 16, 5000),
    "small_bound": (dict(PLUGIN, BOUND=0.4), 16, 6000),
    # the cfg's STEPS range reaches 100 (MPCPlanner.cfg:22): two stage blocks per wavefront
    "N80": (dict(PLUGIN, STEPS=80), 8, 8000),
    "N100": (dict(PLUGIN, STEPS=100), 8, 9000),
}


def variants():
    out = {}
    for name, (P, n, off) in VARIANTS.items():
        st, cf = infinity.make_problems(np.arange(off, off + n))
        d = solve_set(P, st, cf)
        for k, v in d.items():
            out[f"{name}__{k}"] = v
        print(name, "status:", np.unique(d["status"], return_counts=True), "iters mean", d["iters"].mean())
    out["keys"] = np.array(params.KEYS)
    np.savez_compressed(os.path.join(HERE, "variants.npz"), **out)


def preprocess():
    idx = np.arange(64)
    sc = infinity.draw_scenarios(idx)
    px, py, yaw, plan = infinity.scenario_poses(sc)
    st = np.zeros((len(idx), 6))
    cf = np.zeros((len(idx), 4))
    for b in range(len(idx)):
        rc, st[b], cf[b] = O.find_best_path(px[b], py[b], yaw[b], sc["v"][b], sc["w_prev"][b], sc["a_prev"][b],
                                            0.1, plan[b], True)
        assert rc == 0
    np.savez_compressed(os.path.join(HERE, "preprocess.npz"), pose=np.stack([px, py, yaw], 1),
                        vel=np.stack([sc["v"], sc["w_prev"], sc["a_prev"]], 1), plan=plan, dt=0.1, state=st,
                        coeffs=cf)


BICYCLE = dict(PLUGIN, STEPS=25, MODEL=1, LF=0.5, ANGVEL=0.5)


def bicycle():
    st, cf = infinity.make_problems(np.arange(7000, 7064))
    d = solve_set(BICYCLE, st, cf)
    d["model"] = np.int32(1)
    d["lf"] = np.float64(BICYCLE["LF"])
    np.savez_compressed(os.path.join(HERE, "bicycle_N25.npz"), **d)
    print("bicycle_N25 status:", np.unique(d["status"], return_counts=True), "iters mean", d["iters"].mean())


FEATURE_SETS = {
    # name: (params, problem indices of the infinity set)
    # N20: second-order corrections (7, 11, 25, 932: different local minimum without them;
    # 2571: two corrections), soft restoration (5045, 8938), restoration phase (1443),
    # round-1 advisor's filter-size problems (1887, 16101)
    "N20": (PLUGIN, [7, 11, 25, 932, 2571, 5045, 8938, 1443, 1887, 16101]),
    # N40: watchdog (88: six activations, 460, 842, 2012, 2094), soft restoration (422, 429,
    # 1431), restoration phase (69, 1167, 1204, 2956, 3441)
    "N40": (dict(PLUGIN, STEPS=40), [88, 460, 842, 2012, 2094, 422, 429, 1431, 69, 1167, 1204, 2956, 3441]),
    # bicycle N25: watchdog (3308), soft restoration (1292), corrections (18, 23)
    "bicycle": (BICYCLE, [3308, 1292, 18, 23]),
    # the feasibility-restoration phase (round 3, found by scanning problems 0..131071 at
    # N = 20 and 0..32767 at N = 40 with the oracle's diagnostics): every problem of those
    # ranges on which Ipopt enters it
    "resto_N20": (PLUGIN, [1443, 40852, 74511, 84582]),
    "resto_N40": (dict(PLUGIN, STEPS=40), [69, 1167, 1204, 2956, 3441, 4626, 8420, 9871, 18581, 18819, 19148,
                                            19304, 23287, 25150, 25384, 28303, 30285, 31014, 31746]),
}


def ipopt_features():
    out = {}
    for name, (P, idx) in FEATURE_SETS.items():
        st, cf = infinity.make_problems(np.array(idx))
        d = solve_set(P, st, cf)
        d["index"] = np.array(idx)
        for k, v in d.items():
            out[f"{name}__{k}"] = v
        print(name, "status", d["status"].tolist(), "iters", d["iters"].tolist())
        print("   diag (soc, watchdog, soft, resto, resto iters):", d["diag"].tolist())
    # the max_cpu_time budget forced low: 0.005 s -> ora_cpu_iter_budget iterations at N = 20
    P = PLUGIN
    st, cf = infinity.make_problems(np.arange(0, 32))
    budget = O.cpu_iter_budget(0.005, 20)
    d = solve_set(P, st, cf, opts=O.ref_opts(20, cpu_iter_budget=budget))
    for k, v in d.items():
        out[f"budget__{k}"] = v
    out["budget__max_cpu_time"] = np.float64(0.005)
    out["budget__iter_budget"] = np.int32(budget)
    print("budget", budget, "status", np.unique(d["status"], return_counts=True))
    out["keys"] = np.array(params.KEYS)
    np.savez_compressed(os.path.join(HERE, "ipopt_features.npz"), **out)


def hs071():
    with open(os.path.join(HERE, "hs071.json"), "w") as f:
        json.dump({"source": "assets/document/example/CppAD_Ipopt.cpp:146-150",
                   "x": [1.000000, 4.743000, 3.82115, 1.379408], "zl": [1.087871, 0.0, 0.0, 0.0],
                   "zu": [0.0, 0.0, 0.0, 0.0], "rel_tol": 1e-6, "abs_tol": 1e-6}, f, indent=1)


if __name__ == "__main__":
    O.build(force=True)
    sets = set(sys.argv[1:]) or {"hs071", "preprocess", "infinity", "variants", "bicycle", "features", "cppad"}
    if "hs071" in sets:
        hs071()
    if "preprocess" in sets:
        preprocess()
    if "infinity" in sets:
        infinity_set()
    if "variants" in sets:
        variants()
    if "bicycle" in sets:
        bicycle()
    if "features" in sets:
        ipopt_features()
    if "cppad" in sets:
        if os.path.isdir("/root/reference/mpc_ros/include/cppad"):
            cppad_derivs()
        else:
            print("reference tree absent: cppad_derivs.npz not regenerated")
