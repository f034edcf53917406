"""Closed-loop single robot on the infinity course (BASELINE configs[0]).

The reference's tracking loop (mpc_ros/src/driving_state.cpp:175-269): every control
tick the robot's pose and feedback speed, the previous command (_w, _throttle) and the
next waypoints of the plan go through findBestPath's preprocessing and MPC::Solve; the
post-processing turns (w0, a0) into the command speed = min(v + a0 dt, REF_V), and the
command is fed back (driving_state.cpp:191-193, 262-269).  Here the "robot" is the
unicycle the NLP models, integrated over one control period per tick, and the plan is
the next 5 m of the lemniscate (infinity.py), so the whole loop is reproducible.

`step_fn(pose[3], vel[3], plan[M,2]) -> cmd[3]` is one control tick (the GPU's
mpcg_track_device at B = 1, or a checker's restatement).
"""
from __future__ import annotations

import numpy as np

from . import infinity


def nearest_t(px: float, py: float, t_prev: float, window: float = 0.6, n: int = 601) -> float:
    """Path parameter of the closest lemniscate point near the previous one (forward search)."""
    arc = infinity._arc()
    ts = t_prev + np.linspace(-0.1 * window, window, n)
    x, y = arc.point(ts)
    return float(ts[np.argmin((x - px) ** 2 + (y - py) ** 2)])


def plan_from(t: float) -> np.ndarray:
    """The next PATH_LENGTH metres of the course from parameter t: [M, 2] waypoints."""
    arc = infinity._arc()
    s0 = float(np.interp(t % (4.0 * np.pi), arc.t, arc.s))
    ds = infinity.PATH_LENGTH / (infinity.N_WAYPOINTS - 1)
    tj = arc.t_at(s0 + ds * np.arange(infinity.N_WAYPOINTS))
    wx, wy = arc.point(tj)
    return np.stack([wx, wy], axis=-1)


def run(step_fn, ticks: int = 200, dt: float = 0.1, t0: float = 0.3, lateral: float = 0.15,
        heading_err: float = 0.2) -> dict:
    """Drive `ticks` control periods from a pose offset from the course; returns the
    per-tick pose, feedback and command arrays."""
    arc = infinity._arc()
    x, y = arc.point(t0)
    hd = float(arc.heading(t0))
    x, y = float(x - np.sin(hd) * lateral), float(y + np.cos(hd) * lateral)
    yaw = hd + heading_err
    v, w_prev, a_prev, t = 0.0, 0.0, 0.0, t0
    poses, cmds, cte = [], [], []
    for _ in range(ticks):
        t = nearest_t(x, y, t)
        plan = plan_from(t)
        pose = np.array([x, y, np.arctan2(np.sin(yaw), np.cos(yaw))])
        vel = np.array([v, w_prev, a_prev])
        cmd = np.asarray(step_fn(pose, vel, plan), dtype=np.float64)  # speed, w, throttle
        poses.append(pose)
        cmds.append(cmd)
        px, py = arc.point(t)
        cte.append(float(np.hypot(px - x, py - y)))
        speed, w, a = float(cmd[0]), float(cmd[1]), float(cmd[2])
        # the unicycle over one control period with the commanded speed and turn rate
        x += speed * np.cos(yaw) * dt
        y += speed * np.sin(yaw) * dt
        yaw += w * dt
        v, w_prev, a_prev = speed, w, a
    return dict(pose=np.array(poses), cmd=np.array(cmds), dist=np.array(cte))
