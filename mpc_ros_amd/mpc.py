"""Python mirror of the reference's ``class MPC`` (mpc_ros/include/mpc_planner.h:26-47).

Same names, argument meaning and behaviour as the C++ class, backed by the GPU
solver (one problem per call; ``solve_batch`` for many):

* ``MPC()``                           -- MPC::MPC() defaults (mpc_planner.cpp:223-241)
* ``LoadParams(params: dict)``        -- MPC::LoadParams (:243-262).  The map is stored;
  STEPS / ANGVEL / MAXTHR / BOUND keep their previous value when absent, while the
  FG_eval keys (DT, REF_*, W_*) fall back to the FG_eval constructor defaults
  (:42-68) when absent, because the reference builds a fresh FG_eval per Solve.
* ``Solve(state, coeffs) -> [w0, a0]`` -- MPC::Solve (:265-402); fills ``mpc_x``,
  ``mpc_y``, ``mpc_theta`` (N entries each).  As in the reference, the solver status
  is not raised (:378); it is exposed as ``last_status``.
"""
from __future__ import annotations

import numpy as np

from .params import CLASS_DEFAULTS

_FG_KEYS = ("DT", "REF_CTE", "REF_ETHETA", "REF_V", "W_CTE", "W_EPSI", "W_V", "W_ANGVEL", "W_A", "W_DANGVEL",
            "W_DA")


class MPC:
    def __init__(self, device: int = 0):
        self.device = device
        self._mpc_steps = 20
        self._max_angvel = 3.0
        self._max_throttle = 1.0
        self._bound_value = 1.0e3
        self._params: dict = {}
        self.mpc_x: list = []
        self.mpc_y: list = []
        self.mpc_theta: list = []
        self.last_status = 0
        self.last_iters = 0
        self.last_obj = float("nan")
        self._solver = None

    def LoadParams(self, params: dict):  # noqa: N802 (reference name)
        self._params = dict(params)
        if "STEPS" in params:
            self._mpc_steps = int(params["STEPS"])  # double -> int truncation (mpc_planner.cpp:247)
        if "ANGVEL" in params:
            self._max_angvel = float(params["ANGVEL"])
        if "MAXTHR" in params:
            self._max_throttle = float(params["MAXTHR"])
        if "BOUND" in params:
            self._bound_value = float(params["BOUND"])

    def effective_params(self) -> dict:
        """The parameter set a reference Solve would use right now."""
        p = {k: CLASS_DEFAULTS[k] for k in _FG_KEYS}
        for k in _FG_KEYS:
            if k in self._params:
                p[k] = float(self._params[k])
        p.update(STEPS=self._mpc_steps, ANGVEL=self._max_angvel, MAXTHR=self._max_throttle,
                 BOUND=self._bound_value)
        return p

    def _ensure_solver(self):
        from .solver import BatchSolver

        if self._solver is None:
            self._solver = BatchSolver(self.device, self.effective_params(), base="class")
        else:
            self._solver.set_params(self.effective_params(), base="class")
        return self._solver

    def Solve(self, state, coeffs):  # noqa: N802 (reference name)
        st = np.asarray(state, dtype=np.float64).reshape(1, 6)
        cf = np.asarray(coeffs, dtype=np.float64).reshape(1, 4)
        out = self._ensure_solver().solve(st, cf)
        N = self._mpc_steps
        traj = out["traj"][0]
        self.mpc_x = list(traj[0, :N])
        self.mpc_y = list(traj[1, :N])
        self.mpc_theta = list(traj[2, :N])
        self.last_status = int(out["status"][0])
        self.last_iters = int(out["iters"][0])
        self.last_obj = float(out["obj"][0])
        return [float(out["u0"][0, 0]), float(out["u0"][0, 1])]

    def solve_batch(self, state: np.ndarray, coeffs: np.ndarray) -> dict:
        """Extension: B problems with the current parameters in one GPU launch."""
        return self._ensure_solver().solve(state, coeffs)
