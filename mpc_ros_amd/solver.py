"""Batched NMPC solver on one MI355X (wrapper of the C-ABI in include/mpcg.h).

``BatchSolver`` owns one ``mpcg_handle`` (one GPU).  ``solve`` takes host numpy
arrays; ``solve_device`` takes torch tensors already resident in HBM and queues
the kernel on the current torch stream without any host synchronisation.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .params import PLUGIN_DEFAULTS

# Ipopt options of the reference's solve (mpc_planner.cpp:356-368: max_cpu_time 0.5, the
# rest Ipopt 3.12 defaults); any mpcg_params field can be overridden by keyword
IPOPT_DEFAULTS = dict(tol=1e-8, max_iter=3000, filter_cap=64, bound_relax_factor=1e-8, mu_init=0.1, max_cpu_time=0.5)
# the fp32 configuration (precision 1, BASELINE configs[2]) runs two phases (mpcg_wide.hip):
# (1) the fp32 solver on the whole batch with tolerances a float iterate can meet -- the scaled
#     dual infeasibility of an fp32 iterate stalls near 1e-4 (multipliers ~1e3 times
#     FLT_EPSILON) and mu_min = min(tol, compl_inf_tol) / 11 must stay above float resolution;
#     it stops at tol 1e-3 (acceptable termination at 1e-3 and a 300-iteration cap end stalls);
# (2) the fp64 solver with the reference's Ipopt options on the whole batch again: from the fp32
#     iterate where the fp32 solve converged (status 1 or 4: a few fp64 iterations to Ipopt's
#     tolerance, diag[:, 2] == 4), else from the start (its line search failed at a float
#     iterate's noise floor where Ipopt would enter the restoration phase, a tiny step, the
#     iteration limit: diag[:, 2] == 3, bitwise the fp64 solver's result).
# (B > 2048: the B / 1024 problems the solve order ranks longest are solved by the fp64 solver from
# the start, diag[:, 2] == 3, while the fp32 phase runs the others.)
# The returned controls are the fp64 solver's (within 1e-6 of the reference's double-precision
# solve where they converge to the same local minimum).  no_restoration = 1 runs the fp32 phase
# alone and keeps its ending (status 9, 3 or 2 where it cannot finish).
FP32_OPTIONS = dict(precision=1, tol=1e-3, compl_inf_tol=1e-2, tiny_step_tol=10 * 1.1920928955078125e-07,
                    acceptable_tol=1e-3, max_iter=300, no_restoration=0)


class BatchSolver:
    def __init__(self, device: int = 0, params: dict | None = None, strategy: str = "wave", dtype: str = "fp64",
                 **ipopt):
        """dtype "fp32": the fp32 solver with FP32_OPTIONS (overridable by keyword)."""
        if dtype == "fp32":
            ipopt = dict(FP32_OPTIONS, **ipopt)
        elif dtype != "fp64":
            raise ValueError("dtype must be 'fp64' or 'fp32'")
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.mpcg_create(int(device), C.byref(h)), "mpcg_create")
        self._h = h
        self.device = device
        self.set_params(params if params is not None else PLUGIN_DEFAULTS, **ipopt)
        self.set_strategy(strategy)

    def set_strategy(self, strategy: str = "wave"):
        """'wave' (= 'auto'): one problem per wavefront, LDS-resident (the only kernel strategy)."""
        _lib.check(_lib.lib().mpcg_set_strategy(self._h, _lib.STRATEGY[strategy]), "mpcg_set_strategy")

    @property
    def strategy(self) -> str:
        v = _lib.lib().mpcg_get_strategy(self._h)
        return {v2: k for k, v2 in _lib.STRATEGY.items()}[v]

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().mpcg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ parameters
    def set_params(self, params: dict, base: str = "plugin", **ipopt):
        p = _lib.params_from_map(params, base)
        opts = dict(IPOPT_DEFAULTS)
        opts.update(ipopt)
        for k, v in opts.items():
            if not hasattr(p, k):
                raise AttributeError(f"mpcg_params has no field {k!r}")
            setattr(p, k, v)
        _lib.check(_lib.lib().mpcg_set_params(self._h, C.byref(p)), "mpcg_set_params")
        self.params = p
        self.N = p.steps

    def set_park_capacity(self, cap: int = 0):
        """Park-area entries (0: the default max(256, B / 128)); results do not depend on it."""
        _lib.check(_lib.lib().mpcg_set_park_capacity(self._h, int(cap)), "mpcg_set_park_capacity")

    @property
    def last_kernel(self) -> str:
        """The solver kernel instance the last solve launched ("k_solve_wide<...>")."""
        return _lib.lib().mpcg_last_kernel(self._h).decode()

    @property
    def last_solve_order(self) -> bool:
        """True if the last solve ran its problems expected-longest first (B > 2048)."""
        return bool(_lib.lib().mpcg_last_solve_order(self._h))

    def reserve(self, B: int):
        _lib.check(_lib.lib().mpcg_reserve(self._h, int(B)), "mpcg_reserve")

    def workspace_bytes(self, B: int) -> int:
        """What reserve(B) allocates (the handle's park capacity and device included)."""
        return int(_lib.lib().mpcg_handle_workspace_bytes(self._h, int(B)))

    # ----------------------------------------------------------------- solve
    def solve(self, state: np.ndarray, coeffs: np.ndarray, want_traj: bool = True) -> dict:
        state = np.ascontiguousarray(state, dtype=np.float64)
        coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
        B = state.shape[0]
        assert state.shape == (B, 6) and coeffs.shape == (B, 4), "state [B,6], coeffs [B,4]"
        N = self.N
        u0 = np.zeros((B, 2))
        traj = np.zeros((B, 3, N)) if want_traj else None
        status = np.zeros(B, dtype=np.int32)
        iters = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        diag = np.zeros((B, 4), dtype=np.int32)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int32)
        _lib.check(_lib.lib().mpcg_solve_ex(
            self._h, B, state.ctypes.data_as(dp), coeffs.ctypes.data_as(dp), u0.ctypes.data_as(dp),
            traj.ctypes.data_as(dp) if traj is not None else None, status.ctypes.data_as(ip),
            obj.ctypes.data_as(dp), iters.ctypes.data_as(ip), diag.ctypes.data_as(ip)), "mpcg_solve_ex")
        # diag columns: restoration phases, filter entries dropped beyond its capacity, parked,
        # most filter entries held at once
        return dict(u0=u0, traj=traj, status=status, obj=obj, iters=iters, diag=diag)

    def solve_device(self, state, coeffs, u0, traj=None, status=None, obj=None, iters=None, stream=None, diag=None):
        """All arguments are torch tensors on this handle's GPU (float64 / int32, contiguous);
        diag [B, 4] int32: restoration phases, filter overflows, parked, filter peak."""
        import torch

        B = state.shape[0]
        for t, shape, dt in ((state, (B, 6), torch.float64), (coeffs, (B, 4), torch.float64),
                             (u0, (B, 2), torch.float64)):
            assert t.is_cuda and t.dtype == dt and t.is_contiguous() and tuple(t.shape) == shape
        if traj is not None:
            assert traj.dtype == torch.float64 and traj.is_contiguous() and traj.numel() == B * 3 * self.N
        for t in (status, iters):
            assert t is None or (t.dtype == torch.int32 and t.numel() == B)
        assert diag is None or (diag.dtype == torch.int32 and diag.numel() == 4 * B and diag.is_contiguous())
        if stream is None:
            stream = torch.cuda.current_stream(state.device)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        _lib.check(_lib.lib().mpcg_solve_device_ex(
            self._h, B, ptr(state), ptr(coeffs), ptr(u0), ptr(traj), ptr(status), ptr(obj), ptr(iters), ptr(diag),
            C.c_void_p(stream.cuda_stream)), "mpcg_solve_device_ex")

    # ------------------------------------------------ the benchmark's synthetic robots
    def synth_infinity_device(self, start: int, B: int, M: int = 11, seed: int | None = None, stream=None):
        """Robots start .. start + B - 1 of the infinity set generated on this GPU from (seed,
        global index) (mpcg_synth_infinity_device): torch tensors pose [B,3], vel [B,3], plan [B,M,2]."""
        import torch

        from . import infinity

        dev = torch.device("cuda", self.device)
        pose = torch.empty((B, 3), dtype=torch.float64, device=dev)
        vel = torch.empty((B, 3), dtype=torch.float64, device=dev)
        plan = torch.empty((B, M, 2), dtype=torch.float64, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        _lib.check(_lib.lib().mpcg_synth_infinity_device(
            self._h, int(infinity.SEED if seed is None else seed), int(start), int(B), int(M), C.c_void_p(pose.data_ptr()),
            C.c_void_p(vel.data_ptr()), C.c_void_p(plan.data_ptr()), C.c_void_p(stream.cuda_stream)),
            "mpcg_synth_infinity_device")
        return pose, vel, plan

    # ------------------------------------------------ the caller side on the device
    def preprocess_device(self, pose, vel, plan, state, coeffs, delay_mode: bool = True, stream=None):
        """Tracking::findBestPath's preprocessing (driving_state.cpp:175-256) for B robots.

        pose [B,3] (x, y, yaw), vel [B,3] (v feedback, previous w, previous throttle),
        plan [B,M,2] -> state [B,6], coeffs [B,4]; torch float64 tensors on this GPU."""
        import torch

        B, M = plan.shape[0], plan.shape[1]
        for t, shape in ((pose, (B, 3)), (vel, (B, 3)), (plan, (B, M, 2)), (state, (B, 6)), (coeffs, (B, 4))):
            assert t.is_cuda and t.dtype == torch.float64 and t.is_contiguous() and tuple(t.shape) == shape
        if stream is None:
            stream = torch.cuda.current_stream(pose.device)
        ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mpcg_preprocess_device(
            self._h, B, M, ptr(pose), ptr(vel), ptr(plan), int(bool(delay_mode)), ptr(state), ptr(coeffs),
            C.c_void_p(stream.cuda_stream)), "mpcg_preprocess_device")

    def track_device(self, pose, vel, plan, cmd, traj=None, status=None, delay_mode: bool = True, stream=None):
        """One control tick for B robots: preprocessing, solve, post-processing
        (driving_state.cpp:175-269).  cmd [B,3] = (speed, w, throttle)."""
        import torch

        B, M = plan.shape[0], plan.shape[1]
        for t, shape in ((pose, (B, 3)), (vel, (B, 3)), (plan, (B, M, 2)), (cmd, (B, 3))):
            assert t.is_cuda and t.dtype == torch.float64 and t.is_contiguous() and tuple(t.shape) == shape
        if traj is not None:
            assert traj.dtype == torch.float64 and traj.is_contiguous() and traj.numel() == B * 3 * self.N
        assert status is None or (status.dtype == torch.int32 and status.numel() == B)
        if stream is None:
            stream = torch.cuda.current_stream(pose.device)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        _lib.check(_lib.lib().mpcg_track_device(
            self._h, B, M, ptr(pose), ptr(vel), ptr(plan), int(bool(delay_mode)), ptr(cmd), ptr(traj), ptr(status),
            C.c_void_p(stream.cuda_stream)), "mpcg_track_device")


def _params_struct(params, dtype, ipopt):
    if dtype == "fp32":
        ipopt = dict(FP32_OPTIONS, **ipopt)
    p = _lib.params_from_map(params if params is not None else PLUGIN_DEFAULTS)
    opts = dict(IPOPT_DEFAULTS)
    opts.update(ipopt)
    for k, v in opts.items():
        if not hasattr(p, k):
            raise AttributeError(f"mpcg_params has no field {k!r}")
        setattr(p, k, v)
    return p


class MultiSolver:
    """mpcg_multi: a persistent multi-GPU context (communicator, per-GPU handles, streams and
    buffers for batches of up to B_max problems, created once); ``solve`` shards a host batch
    over the GPUs and gathers the results to devices[0] by RCCL (include/mpcg.h)."""

    def __init__(self, devices, B_max: int, params: dict | None = None, dtype: str = "fp64", **ipopt):
        self.p = _params_struct(params, dtype, ipopt)
        self.N = self.p.steps
        self.B_max = int(B_max)
        dev = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        _lib.check(_lib.lib().mpcg_multi_create(len(devices), dev, C.byref(self.p), self.B_max, C.byref(h)),
                   "mpcg_multi_create")
        self._h = h

    def solve(self, state, coeffs) -> dict:
        state = np.ascontiguousarray(state, dtype=np.float64)
        coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
        B = state.shape[0]
        assert state.shape == (B, 6) and coeffs.shape == (B, 4), "state [B,6], coeffs [B,4]"
        N = self.N
        u0 = np.zeros((B, 2))
        traj = np.zeros((B, 3, N))
        status = np.zeros(B, dtype=np.int32)
        iters = np.zeros(B, dtype=np.int32)
        obj = np.zeros(B)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int32)
        _lib.check(_lib.lib().mpcg_multi_solve(
            self._h, B, state.ctypes.data_as(dp), coeffs.ctypes.data_as(dp), u0.ctypes.data_as(dp),
            traj.ctypes.data_as(dp), status.ctypes.data_as(ip), obj.ctypes.data_as(dp), iters.ctypes.data_as(ip)),
            "mpcg_multi_solve")
        return dict(u0=u0, traj=traj, status=status, obj=obj, iters=iters)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().mpcg_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_multi(devices, params: dict | None = None, state=None, coeffs=None, dtype: str = "fp64", **ipopt) -> dict:
    """mpcg_solve_multi: one process, the batch sharded over `devices`, results gathered to
    devices[0] by RCCL (include/mpcg.h).  Only ngpu = 1 has run on hardware (the GPU boxes
    this was developed on hold one MI355X); the shard and gather arithmetic for ngpu > 1 is
    unit-tested on the CPU (tests/test_abi.py)."""
    state = np.ascontiguousarray(state, dtype=np.float64)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    B = state.shape[0]
    assert state.shape == (B, 6) and coeffs.shape == (B, 4), "state [B,6], coeffs [B,4]"
    if dtype == "fp32":
        ipopt = dict(FP32_OPTIONS, **ipopt)
    p = _lib.params_from_map(params if params is not None else PLUGIN_DEFAULTS)
    opts = dict(IPOPT_DEFAULTS)
    opts.update(ipopt)
    for k, v in opts.items():
        if not hasattr(p, k):
            raise AttributeError(f"mpcg_params has no field {k!r}")
        setattr(p, k, v)
    N = p.steps
    u0 = np.zeros((B, 2))
    traj = np.zeros((B, 3, N))
    status = np.zeros(B, dtype=np.int32)
    iters = np.zeros(B, dtype=np.int32)
    obj = np.zeros(B)
    dev = (C.c_int * len(devices))(*devices)
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int32)
    _lib.check(_lib.lib().mpcg_solve_multi(
        len(devices), dev, C.byref(p), B, state.ctypes.data_as(dp), coeffs.ctypes.data_as(dp), u0.ctypes.data_as(dp),
        traj.ctypes.data_as(dp), status.ctypes.data_as(ip), obj.ctypes.data_as(dp), iters.ctypes.data_as(ip)),
        "mpcg_solve_multi")
    return dict(u0=u0, traj=traj, status=status, obj=obj, iters=iters)
