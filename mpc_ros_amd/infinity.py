"""Synthetic "infinity set" of NMPC problems.

The reference's ref_trajectory_tracking node and its infinity course are absent
from this fork, so the problem set is synthesised: a robot near a
lemniscate of Gerono p(t) = (A sin t, A sin t cos t), A = 3 m, with pose and
velocity ranges taken from the reference's closed-loop log (assets/mpc.csv:
cte in [-0.47, 0.28], etheta in [-0.85, 1.12], v <= 0.8, |w| <= 1).

Every problem is a pure function of (seed, global index), via a counter-based
hash, so a shard on any rank regenerates exactly its own slice.

Each problem is pre-processed exactly as Tracking::findBestPath does
(mpc_ros/src/driving_state.cpp:175-256, delay_mode = true per
mpc_ros/cfg/MPCPlanner.cfg:14): waypoints -> vehicle frame, cubic polyfit,
cte = c0, heading error from the first int(0.3 M) waypoint increments,
kinematic delay compensation.  Output: state[B, 6] = (x, y, theta, v, cte, etheta)
and coeffs[B, 4], the two arguments of MPC::Solve (mpc_planner.cpp:265).
"""
from __future__ import annotations

import numpy as np

SEED = 20251015
LEMNISCATE_A = 3.0
N_WAYPOINTS = 11
PATH_LENGTH = 5.0  # path_length, MPCPlanner.cfg:19

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniforms(idx: np.ndarray, k: int, seed: int = SEED) -> np.ndarray:
    """U[0,1) draw number k of problem idx (counter-based, shard independent)."""
    with np.errstate(over="ignore"):
        z = np.asarray(idx, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03)
        z = z ^ (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)) ^ (np.uint64(k + 1) * np.uint64(0xA24BAED4963EE407))
        z = _splitmix64(_splitmix64(z))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


class _Arc:
    """Arc-length table of the lemniscate over t in [0, 4 pi)."""

    def __init__(self, A: float = LEMNISCATE_A, n: int = 200001):
        t = np.linspace(0.0, 4.0 * np.pi, n)
        dx = A * np.cos(t)
        dy = A * np.cos(2.0 * t)
        sp = np.hypot(dx, dy)
        s = np.concatenate([[0.0], np.cumsum(0.5 * (sp[1:] + sp[:-1]) * np.diff(t))])
        self.t, self.s, self.A = t, s, A

    def point(self, t):
        return self.A * np.sin(t), self.A * np.sin(t) * np.cos(t)

    def heading(self, t):
        return np.arctan2(self.A * np.cos(2.0 * t), self.A * np.cos(t))

    def t_at(self, s):
        return np.interp(s, self.s, self.t)

    def s_at(self, t):
        return np.interp(t, self.t, self.s)


_ARC = None


def _arc() -> _Arc:
    global _ARC
    if _ARC is None:
        _ARC = _Arc()
    return _ARC


def draw_scenarios(idx: np.ndarray, seed: int = SEED) -> dict:
    """Per-problem scenario parameters (SURVEY.md §8d ranges)."""
    idx = np.asarray(idx, dtype=np.int64)
    return dict(
        t=2.0 * np.pi * uniforms(idx, 0, seed),
        lateral=-0.45 + 0.75 * uniforms(idx, 1, seed),
        heading_err=-0.85 + 1.95 * uniforms(idx, 2, seed),
        v=0.8 * uniforms(idx, 3, seed),
        w_prev=-1.0 + 2.0 * uniforms(idx, 4, seed),
        a_prev=-1.0 + 2.0 * uniforms(idx, 5, seed),
    )


def scenario_poses(sc: dict):
    """Robot pose + reference waypoints for scenarios (arrays of length B)."""
    arc = _arc()
    t = np.asarray(sc["t"], dtype=np.float64)
    px, py = arc.point(t)
    hd = arc.heading(t)
    px = px - np.sin(hd) * sc["lateral"]
    py = py + np.cos(hd) * sc["lateral"]
    yaw = hd + sc["heading_err"]
    yaw = np.arctan2(np.sin(yaw), np.cos(yaw))  # tf2::getYaw range
    s0 = arc.s_at(t)
    ds = PATH_LENGTH / (N_WAYPOINTS - 1)
    sj = s0[:, None] + ds * np.arange(N_WAYPOINTS)[None, :]
    tj = arc.t_at(sj)
    wx, wy = arc.point(tj)
    plan = np.stack([wx, wy], axis=-1)  # [B, M, 2]
    return px, py, yaw, plan


def find_best_path(px, py, yaw, v, w, throttle, dt, plan, delay_mode: bool = True):
    """Vectorised Tracking::findBestPath (driving_state.cpp:175-256) for B problems.

    plan: [B, M, 2] waypoints.  Returns state [B, 6], coeffs [B, 4]."""
    px, py, yaw, v, w, throttle = (np.asarray(a, dtype=np.float64) for a in (px, py, yaw, v, w, throttle))
    B, M, _ = plan.shape
    ct, st = np.cos(yaw)[:, None], np.sin(yaw)[:, None]
    dx = plan[:, :, 0] - px[:, None]
    dy = plan[:, :, 1] - py[:, None]
    xv = dx * ct + dy * st
    yv = dy * ct - dx * st
    V = np.ones((B, M, 4))
    for j in range(3):
        V[:, :, j + 1] = V[:, :, j] * xv
    q, r = np.linalg.qr(V)  # Householder QR least squares, as Eigen householderQr().solve
    coeffs = np.linalg.solve(r, np.einsum("bmk,bm->bk", q, yv)[..., None])[..., 0]
    cte = coeffs[:, 0]
    nsample = int(M * 0.3)
    gx = np.zeros(B)
    gy = np.zeros(B)
    for i in range(1, nsample):
        gx += plan[:, i, 0] - plan[:, i - 1, 0]
        gy += plan[:, i, 1] - plan[:, i - 1, 1]
    temp = yaw.copy()
    traj = np.arctan2(gy, gx)
    temp = np.where(temp <= -np.pi + traj, temp + 2.0 * np.pi, temp)
    ok = (gx != 0.0) & (gy != 0.0) & (temp - traj < 1.8 * np.pi)
    eth = np.where(ok, temp - traj, 0.0)
    state = np.zeros((B, 6))
    if delay_mode:
        theta_act = w * dt
        state[:, 0] = v * dt
        state[:, 1] = 0.0
        state[:, 2] = theta_act
        state[:, 3] = v + throttle * dt
        state[:, 4] = cte + v * np.sin(eth) * dt
        state[:, 5] = eth - theta_act
    else:
        state[:, 3] = v
        state[:, 4] = cte
        state[:, 5] = eth
    return state, coeffs


def make_problems(idx, dt: float = 0.1, seed: int = SEED, delay_mode: bool = True):
    """(state [B,6], coeffs [B,4]) for global problem indices idx."""
    sc = draw_scenarios(np.asarray(idx), seed)
    return problems_from_scenarios(sc, dt, delay_mode)


def problems_from_scenarios(sc: dict, dt: float = 0.1, delay_mode: bool = True):
    px, py, yaw, plan = scenario_poses(sc)
    return find_best_path(px, py, yaw, sc["v"], sc["w_prev"], sc["a_prev"], dt, plan, delay_mode)


def edge_scenarios() -> dict:
    """32 hand-picked cases: saturated turns, saturated throttle, path crossing point,
    wrap-around headings, standstill, maximum speed, extreme lateral offsets."""
    rows = []
    for t in (0.0, np.pi / 2, np.pi, 3 * np.pi / 2):
        for he in (-0.85, 1.10):
            rows.append((t, 0.0, he, 0.4, 0.0, 0.0))
    for lat in (-0.45, 0.30):
        for v in (0.0, 0.8):
            for w in (-1.0, 1.0):
                rows.append((0.7, lat, 0.3, v, w, 1.0 if v == 0.0 else -1.0))
    for t in (0.05, 2.9, 3.3, 6.2):
        rows.append((t, 0.1, -0.6, 0.8, 1.0, 1.0))
        rows.append((t, -0.2, 0.9, 0.0, -1.0, -1.0))
    while len(rows) < 32:
        k = len(rows)
        rows.append((0.37 * k, 0.02 * (k % 7) - 0.06, 0.05 * (k % 9) - 0.2, 0.1 * (k % 8), 0.0, 0.0))
    a = np.array(rows[:32], dtype=np.float64)
    return dict(t=a[:, 0], lateral=a[:, 1], heading_err=a[:, 2], v=a[:, 3], w_prev=a[:, 4], a_prev=a[:, 5])
