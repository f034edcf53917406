"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package mpc_ros_amd/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")


class MpcParams(C.Structure):
    _fields_ = [
        ("steps", C.c_int),
        ("dt", C.c_double), ("ref_cte", C.c_double), ("ref_etheta", C.c_double), ("ref_v", C.c_double),
        ("w_cte", C.c_double), ("w_etheta", C.c_double), ("w_v", C.c_double), ("w_angvel", C.c_double),
        ("w_accel", C.c_double), ("w_angvel_d", C.c_double), ("w_accel_d", C.c_double),
        ("max_angvel", C.c_double), ("max_throttle", C.c_double), ("bound", C.c_double),
        ("model", C.c_int), ("lf", C.c_double),
    ]


class IpmOpts(C.Structure):
    _fields_ = [
        ("tol", C.c_double), ("max_iter", C.c_int), ("bound_relax_factor", C.c_double),
        ("honor_original_bounds", C.c_int), ("mu_init", C.c_double), ("print_level", C.c_int),
        ("acceptable_tol", C.c_double), ("acceptable_iter", C.c_int), ("acceptable_dual_inf_tol", C.c_double),
        ("acceptable_constr_viol_tol", C.c_double), ("acceptable_compl_inf_tol", C.c_double),
        ("acceptable_obj_change_tol", C.c_double), ("max_soc", C.c_int), ("kappa_soc", C.c_double),
        ("watchdog_shortened_iter_trigger", C.c_int), ("watchdog_trial_iter_max", C.c_int),
        ("soft_resto_pderror_reduction_factor", C.c_double), ("max_soft_resto_iters", C.c_int),
        ("restoration", C.c_int), ("obj_max_inc", C.c_double), ("max_filter_resets", C.c_int),
        ("filter_reset_trigger", C.c_int), ("tiny_step_tol", C.c_double), ("tiny_step_y_tol", C.c_double),
        ("cpu_iter_budget", C.c_int), ("dual_inf_tol", C.c_double), ("constr_viol_tol", C.c_double),
        ("compl_inf_tol", C.c_double), ("kkt_structured", C.c_int), ("refine_steps", C.c_int),
    ]


_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int)
        L.ora_ldlt_factor.argtypes = [C.c_int, dp, ip, C.c_double, ip, ip, ip]
        L.ora_ldlt_solve.argtypes = [C.c_int, dp, ip, dp]
        L.ora_ipm_default_opts.argtypes = [C.POINTER(IpmOpts)]
        L.ora_mpc_nx.argtypes = [C.c_int]
        L.ora_mpc_ng.argtypes = [C.c_int]
        for fn in ("ora_mpc_fg", "ora_mpc_grad_f", "ora_mpc_jac_g"):
            getattr(L, fn).argtypes = [C.POINTER(MpcParams), dp, dp, dp]
        L.ora_mpc_hess.argtypes = [C.POINTER(MpcParams), dp, dp, C.c_double, dp, dp]
        L.ora_mpc_bounds.argtypes = [C.POINTER(MpcParams), dp, dp, dp, dp, dp, dp]
        L.ora_mpc_solve.argtypes = [C.POINTER(MpcParams), C.POINTER(IpmOpts), dp, dp, dp, dp, dp, ip, dp, dp]
        L.ora_mpc_solve_batch_diag.argtypes = [C.POINTER(MpcParams), C.POINTER(IpmOpts), C.c_int64, dp, dp, dp, dp,
                                               dp, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                               C.POINTER(C.c_int32), C.c_int]
        L.ora_cpu_iter_budget.argtypes = [C.c_double, C.c_int]
        L.ora_mpc_solve_batch.argtypes = [C.POINTER(MpcParams), C.POINTER(IpmOpts), C.c_int64, dp, dp, dp, dp,
                                          dp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int]
        L.ora_mpc_kkt_residual.argtypes = [C.POINTER(MpcParams), dp, dp, dp, dp, dp, dp]
        L.ora_mpc_kkt_residual.restype = C.c_double
        L.ora_hs071_solve.argtypes = [C.POINTER(IpmOpts), dp, dp, dp, ip]
        L.ora_find_best_path.argtypes = [C.c_double] * 7 + [C.c_int, dp, C.c_int, dp, dp]
        L.ora_polyfit.argtypes = [C.c_int, dp, dp, C.c_int, dp]
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_double))


def params_from_dict(d: dict) -> MpcParams:
    p = MpcParams()
    p.steps = int(d["STEPS"])
    p.dt = d["DT"]
    p.ref_cte = d["REF_CTE"]
    p.ref_etheta = d["REF_ETHETA"]
    p.ref_v = d["REF_V"]
    p.w_cte = d["W_CTE"]
    p.w_etheta = d["W_EPSI"]
    p.w_v = d["W_V"]
    p.w_angvel = d["W_ANGVEL"]
    p.w_accel = d["W_A"]
    p.w_angvel_d = d["W_DANGVEL"]
    p.w_accel_d = d["W_DA"]
    p.max_angvel = d["ANGVEL"]
    p.max_throttle = d["MAXTHR"]
    p.bound = d["BOUND"]
    p.model = int(d.get("MODEL", 0))  # extension keys (not in the reference map): kinematic bicycle
    p.lf = float(d.get("LF", 0.5))
    return p


def ipm_opts(tol: float = 1e-10, max_iter: int = 3000, bound_relax_factor: float = 1e-8,
             honor_original_bounds: int = 1, print_level: int = 0, **kw) -> IpmOpts:
    """Ipopt 3.12 defaults (oracle/ipm.c ora_ipm_default_opts) with the given overrides;
    keyword arguments are further IpmOpts fields (e.g. max_soc=0, cpu_iter_budget=40)."""
    o = IpmOpts()
    lib().ora_ipm_default_opts(C.byref(o))
    o.tol = tol
    o.max_iter = max_iter
    o.bound_relax_factor = bound_relax_factor
    o.honor_original_bounds = honor_original_bounds
    o.print_level = print_level
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(k)
        setattr(o, k, v)
    return o


def ref_opts(steps: int, **kw) -> IpmOpts:
    """The reference's solver options (mpc_planner.cpp:356-368): Ipopt 3.12 defaults with
    max_cpu_time 0.5 s applied as its iteration budget at this horizon."""
    kw.setdefault("cpu_iter_budget", cpu_iter_budget(0.5, steps))
    return ipm_opts(tol=1e-8, **kw)


def cpu_iter_budget(max_cpu_time: float, steps: int) -> int:
    """Iterations equivalent to max_cpu_time seconds of the reference's Solve (ora.h)."""
    return int(lib().ora_cpu_iter_budget(float(max_cpu_time), int(steps)))


def mpc_solve(params: dict, state, coeffs, opts: IpmOpts | None = None, full: bool = False):
    L = lib()
    p = params_from_dict(params)
    o = opts or ipm_opts()
    N = p.steps
    st = np.ascontiguousarray(state, dtype=np.float64)
    cf = np.ascontiguousarray(coeffs, dtype=np.float64)
    u0 = np.zeros(2)
    traj = np.zeros(3 * N)
    obj = C.c_double()
    it = C.c_int()
    kkt = C.c_double()
    xfull = np.zeros(L.ora_mpc_nx(N))
    status = L.ora_mpc_solve(C.byref(p), C.byref(o), _dp(st), _dp(cf), _dp(u0), _dp(traj), C.byref(obj),
                             C.byref(it), C.byref(kkt), _dp(xfull))
    out = dict(u0=u0, traj=traj.reshape(3, N), obj=obj.value, iters=it.value, status=status, kkt=kkt.value)
    if full:
        out["x"] = xfull
    return out


def mpc_solve_batch(params: dict, state: np.ndarray, coeffs: np.ndarray, opts: IpmOpts | None = None,
                    nthreads: int = 0, diag: bool = False):
    L = lib()
    p = params_from_dict(params)
    o = opts or ipm_opts()
    N = p.steps
    B = state.shape[0]
    st = np.ascontiguousarray(state, dtype=np.float64)
    cf = np.ascontiguousarray(coeffs, dtype=np.float64)
    u0 = np.zeros((B, 2))
    traj = np.zeros((B, 3, N))
    obj = np.zeros(B)
    status = np.zeros(B, dtype=np.int32)
    iters = np.zeros(B, dtype=np.int32)
    dg = np.zeros((B, 7), dtype=np.int32)
    L.ora_mpc_solve_batch_diag(C.byref(p), C.byref(o), B, _dp(st), _dp(cf), _dp(u0), _dp(traj), _dp(obj),
                               status.ctypes.data_as(C.POINTER(C.c_int32)), iters.ctypes.data_as(C.POINTER(C.c_int32)),
                               dg.ctypes.data_as(C.POINTER(C.c_int32)), int(nthreads))
    out = dict(u0=u0, traj=traj, obj=obj, status=status, iters=iters)
    if diag:  # per problem: n_soc, n_watchdog, n_soft_resto, n_resto, resto_iters, slack moves
        # (never restated: must be 0), floor(log10(smallest slack / (eps min(1, mu))))
        out["diag"] = dg
    return out


def mpc_fg(params: dict, coeffs, vars_):
    L = lib()
    p = params_from_dict(params)
    ng = L.ora_mpc_ng(p.steps)
    fg = np.zeros(ng + 1)
    L.ora_mpc_fg(C.byref(p), _dp(np.ascontiguousarray(coeffs, float)), _dp(np.ascontiguousarray(vars_, float)),
                 _dp(fg))
    return fg


def mpc_derivs(params: dict, coeffs, vars_, sigma: float, lam):
    L = lib()
    p = params_from_dict(params)
    nx, ng = L.ora_mpc_nx(p.steps), L.ora_mpc_ng(p.steps)
    c = np.ascontiguousarray(coeffs, float)
    x = np.ascontiguousarray(vars_, float)
    lm = np.ascontiguousarray(lam, float)
    gf = np.zeros(nx)
    J = np.zeros((ng, nx))
    H = np.zeros((nx, nx))
    L.ora_mpc_grad_f(C.byref(p), _dp(c), _dp(x), _dp(gf))
    L.ora_mpc_jac_g(C.byref(p), _dp(c), _dp(x), _dp(J))
    L.ora_mpc_hess(C.byref(p), _dp(c), _dp(x), sigma, _dp(lm), _dp(H))
    return gf, J, H


def mpc_kkt_residual(params: dict, state, coeffs, x):
    L = lib()
    p = params_from_dict(params)
    d, pr, b = C.c_double(), C.c_double(), C.c_double()
    r = L.ora_mpc_kkt_residual(C.byref(p), _dp(np.ascontiguousarray(state, float)),
                               _dp(np.ascontiguousarray(coeffs, float)), _dp(np.ascontiguousarray(x, float)),
                               C.byref(d), C.byref(pr), C.byref(b))
    return dict(max=r, dual=d.value, primal=pr.value, bound=b.value)


def hs071(opts: IpmOpts | None = None):
    L = lib()
    o = opts or ipm_opts(tol=1e-8)
    x = np.zeros(4)
    zl = np.zeros(4)
    zu = np.zeros(4)
    it = C.c_int()
    st = L.ora_hs071_solve(C.byref(o), _dp(x), _dp(zl), _dp(zu), C.byref(it))
    return dict(x=x, zl=zl, zu=zu, status=st, iters=it.value)


def ldlt(a: np.ndarray, tiny: float = 1e-300):
    """Factor a symmetric matrix; returns (factor, ipiv, inertia)."""
    L = lib()
    n = a.shape[0]
    f = np.asfortranarray(a.astype(np.float64)).copy(order="F")
    buf = np.ascontiguousarray(f.T).ravel()  # column-major storage as a flat C array
    ipiv = np.zeros(n, dtype=np.int32)
    npos, nneg, nz = C.c_int(), C.c_int(), C.c_int()
    L.ora_ldlt_factor(n, _dp(buf), ipiv.ctypes.data_as(C.POINTER(C.c_int)), tiny, C.byref(npos), C.byref(nneg),
                      C.byref(nz))
    return buf, ipiv, (npos.value, nneg.value, nz.value)


def ldlt_solve(fac, ipiv, b):
    L = lib()
    n = ipiv.shape[0]
    x = np.ascontiguousarray(b, dtype=np.float64).copy()
    L.ora_ldlt_solve(n, _dp(fac), ipiv.ctypes.data_as(C.POINTER(C.c_int)), _dp(x))
    return x


def find_best_path(px, py, yaw, v, w, throttle, dt, plan_xy, delay_mode=True):
    L = lib()
    plan = np.ascontiguousarray(plan_xy, dtype=np.float64).reshape(-1)
    M = plan.shape[0] // 2
    st = np.zeros(6)
    cf = np.zeros(4)
    rc = L.ora_find_best_path(px, py, yaw, v, w, throttle, dt, M, _dp(plan), int(delay_mode), _dp(st), _dp(cf))
    return rc, st, cf
