"""Closed-loop single robot on the infinity course (BASELINE configs[0]; the reference's
loop driving_state.cpp:175-269 with the command fed back, mpc_ros_amd/closed_loop.py).

CPU: the checker's loop (oracle preprocessing + oracle solve + post-processing) tracks the
course.  GPU: the device loop (mpcg_track_device at B = 1) drives the robot for 200 ticks;
at every tick the checker's command for the same inputs (pose, feedback, previous
command, plan) must agree within 1e-6.  (Two loops closed separately drift apart at
rounding level, 1e-13 per tick, until a tick near a local-minimum boundary sends them to
different minima -- so the comparison is made on the device loop's inputs.)  The share
of ticks with a saturated turn rate is reported beside the reference's log
(assets/mpc.csv: 103 of 365 ticks, 28 %).
"""
from __future__ import annotations

import numpy as np
import pytest

DT = 0.1


def oracle_step(oracle, P):
    def step(pose, vel, plan):
        rc, st, cf = oracle.find_best_path(pose[0], pose[1], pose[2], vel[0], vel[1], vel[2], DT, plan, True)
        assert rc == 0
        r = oracle.mpc_solve(P, st, cf, opts=oracle.ref_opts(int(P["STEPS"])))
        w0, a0 = r["u0"]
        return np.array([min(vel[0] + a0 * DT, P["REF_V"]), w0, a0])

    return step


def test_oracle_closed_loop_tracks_course(oracle):
    from mpc_ros_amd import closed_loop, params

    P = params.PLUGIN_DEFAULTS
    r = closed_loop.run(oracle_step(oracle, P), ticks=80)
    assert r["dist"][-40:].max() < 0.3  # converged onto the course
    assert r["cmd"][:, 0].max() <= P["REF_V"] + 1e-12


@pytest.mark.gpu
def test_gpu_closed_loop_matches_oracle_loop(oracle):
    import torch

    from mpc_ros_amd import closed_loop, params
    from mpc_ros_amd.solver import BatchSolver

    P = params.PLUGIN_DEFAULTS
    s = BatchSolver(0, P)
    dev = torch.device("cuda:0")

    def gpu_step(pose, vel, plan):
        tp = torch.from_numpy(np.ascontiguousarray(pose[None])).to(dev)
        tv = torch.from_numpy(np.ascontiguousarray(vel[None])).to(dev)
        tpl = torch.from_numpy(np.ascontiguousarray(plan[None])).to(dev)
        cmd = torch.empty((1, 3), dtype=torch.float64, device=dev)
        s.track_device(tp, tv, tpl, cmd)
        torch.cuda.synchronize()
        return cmd[0].cpu().numpy()

    ticks = 200
    seen = []
    ostep = oracle_step(oracle, P)

    def both(pose, vel, plan):
        c = gpu_step(pose, vel, plan)
        seen.append(ostep(pose, vel, plan))
        return c

    g = closed_loop.run(both, ticks=ticks)
    diff = np.abs(g["cmd"] - np.array(seen)).max(1)
    assert diff.max() <= 1e-6, (diff.argmax(), diff.max())
    sat = np.mean(np.abs(g["cmd"][:, 1]) >= P["ANGVEL"] - 1e-6)
    print(f"closed loop: {ticks} ticks, max |dcmd| {diff.max():.2e}, |w| saturated on {100 * sat:.1f} % of ticks "
          f"(reference log assets/mpc.csv: 28.2 %)")
    assert g["dist"][-100:].max() < 0.3
