"""Parameter sets of the reference, by name.

The reference keeps MPC parameters in a ``std::map<string,double>`` with 15 keys
(built in DrivingStateContext::updateMpcConfigs, mpc_ros/src/driving_state.cpp:65-79,
consumed by MPC::LoadParams, mpc_ros/src/mpc_planner.cpp:243-262, and
FG_eval::LoadParams, :71-97).  Two default sets exist in the reference:

* ``CLASS_DEFAULTS``  -- what an ``MPC`` object holds before any LoadParams:
  MPC::MPC() (:223-241: STEPS 20, ANGVEL 3.0, MAXTHR 1.0, BOUND 1e3) plus the
  FG_eval constructor defaults (:42-68).  FG_eval's own default STEPS is 40, which
  would index past the 20-step variable vector the MPC sizes; the shared STEPS of
  the MPC object is used instead (documented deviation).
* ``PLUGIN_DEFAULTS`` -- what the move_base plugin actually loads: the
  dynamic_reconfigure defaults of mpc_ros/cfg/MPCPlanner.cfg:22-37 with
  DT = 1/controller_frequency = 0.1 (driving_state.cpp:28).  The benchmark and the
  golden fixtures use these.
"""
from __future__ import annotations

KEYS = ("DT", "STEPS", "REF_CTE", "REF_ETHETA", "REF_V", "W_CTE", "W_EPSI", "W_V", "W_ANGVEL", "W_A",
        "W_DANGVEL", "W_DA", "ANGVEL", "MAXTHR", "BOUND")

CLASS_DEFAULTS = {
    "DT": 0.1, "STEPS": 20, "REF_CTE": 0.0, "REF_ETHETA": 0.0, "REF_V": 0.5,
    "W_CTE": 100.0, "W_EPSI": 100.0, "W_V": 1.0, "W_ANGVEL": 100.0, "W_A": 50.0,
    "W_DANGVEL": 0.0, "W_DA": 0.0, "ANGVEL": 3.0, "MAXTHR": 1.0, "BOUND": 1.0e3,
}

PLUGIN_DEFAULTS = {
    "DT": 0.1, "STEPS": 20, "REF_CTE": 0.0, "REF_ETHETA": 0.0, "REF_V": 1.0,
    "W_CTE": 1000.0, "W_EPSI": 1000.0, "W_V": 100.0, "W_ANGVEL": 100.0, "W_A": 50.0,
    "W_DANGVEL": 0.0, "W_DA": 10.0, "ANGVEL": 1.0, "MAXTHR": 1.0, "BOUND": 1000.0,
}


def merged(base: dict, overrides: dict | None) -> dict:
    """LoadParams semantics: keys present in ``overrides`` replace, others keep the
    previous value (the ``params.find(k) != end() ? at(k) : old`` pattern of
    mpc_planner.cpp:73-85, 247-250).  Unknown keys are kept but ignored."""
    out = dict(base)
    if overrides:
        for k, v in overrides.items():
            out[k] = float(v)
    return out
