"""Host-side logic of the product package (no GPU): parameter semantics of the
reference's MPC / LoadParams, the synthetic problem generator, sharding."""
from __future__ import annotations

import os

import numpy as np
import pytest

from mpc_ros_amd import dist, infinity, params
from mpc_ros_amd.mpc import MPC


def test_mpc_defaults_match_reference_constructor():
    m = MPC()
    p = m.effective_params()
    # MPC::MPC() mpc_planner.cpp:226-230 and FG_eval ctor :47-57
    assert p["STEPS"] == 20 and p["ANGVEL"] == 3.0 and p["MAXTHR"] == 1.0 and p["BOUND"] == 1e3
    assert p["DT"] == 0.1 and p["REF_V"] == 0.5 and p["W_CTE"] == 100 and p["W_V"] == 1 and p["W_DA"] == 0


def test_load_params_semantics():
    m = MPC()
    m.LoadParams(dict(params.PLUGIN_DEFAULTS, STEPS=25.9))
    p = m.effective_params()
    assert p["STEPS"] == 25  # double -> int truncation (mpc_planner.cpp:247)
    assert p["W_CTE"] == 1000 and p["ANGVEL"] == 1.0
    # a later map without some keys: MPC-level keys keep their value, FG keys revert
    m.LoadParams({"W_V": 7.0})
    p = m.effective_params()
    assert p["STEPS"] == 25 and p["ANGVEL"] == 1.0 and p["BOUND"] == 1000
    assert p["W_V"] == 7.0 and p["W_CTE"] == 100.0 and p["REF_V"] == 0.5


def test_generator_is_shard_independent():
    a_st, a_cf = infinity.make_problems(np.arange(0, 300))
    b_st, b_cf = infinity.make_problems(np.arange(137, 300))
    np.testing.assert_array_equal(a_st[137:], b_st)
    np.testing.assert_array_equal(a_cf[137:], b_cf)


def test_generator_ranges():
    sc = infinity.draw_scenarios(np.arange(20000))
    assert sc["lateral"].min() >= -0.45 and sc["lateral"].max() <= 0.30
    assert sc["heading_err"].min() >= -0.85 and sc["heading_err"].max() <= 1.10
    assert sc["v"].min() >= 0 and sc["v"].max() <= 0.8
    st, cf = infinity.make_problems(np.arange(4096))
    assert np.isfinite(st).all() and np.isfinite(cf).all()
    # delay-mode prediction (driving_state.cpp:242-256): y_act = 0, x_act = v dt >= 0
    assert (st[:, 1] == 0).all() and (st[:, 0] >= 0).all()


def test_generator_matches_golden_preprocess():
    from conftest import load_npz

    z = load_npz("preprocess.npz")
    st, cf = infinity.find_best_path(z["pose"][:, 0], z["pose"][:, 1], z["pose"][:, 2], z["vel"][:, 0],
                                     z["vel"][:, 1], z["vel"][:, 2], float(z["dt"]), z["plan"])
    np.testing.assert_allclose(st, z["state"], atol=1e-11)
    np.testing.assert_allclose(cf, z["coeffs"], atol=1e-9, rtol=1e-9)


@pytest.mark.parametrize("total,world", [(10, 3), (524288, 8), (5, 8), (64, 1)])
def test_shard_covers_exactly(total, world):
    seen = []
    for r in range(world):
        s, c = dist.shard(total, r, world)
        seen.extend(range(s, s + c))
        assert c <= dist.max_shard(total, world)
    assert seen == list(range(total))


def test_build_reads_kernel_resource_remarks():
    """build.kernel_resources parses hipcc's kernel-resource-usage remarks; the build
    refuses a solve kernel whose LDS is not all dynamic (static LDS would overlap the
    solver's layout, which starts at address 0)."""
    from mpc_ros_amd import build

    text = "\n".join([
        "x.hip:39:1: remark: Function Name: _ZN4mpcg12k_solve_wideILi0ELb1EdLi1ELb1EEEvNS_8WideArgsE [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:39:1: remark:     VGPRs: 256 [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:39:1: remark:     ScratchSize [bytes/lane]: 128 [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:39:1: remark:     Occupancy [waves/SIMD]: 2 [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:39:1: remark:     SGPRs Spill: 341 [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:39:1: remark:     LDS Size [bytes/block]: 4096 [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:80:1: remark: Function Name: _ZN4mpcg11k_sched_keyElPKdPfPi [-Rpass-analysis=kernel-resource-usage]",
        "x.hip:80:1: remark:     VGPRs: 12 [-Rpass-analysis=kernel-resource-usage]",
    ])
    u = build.kernel_resources(text)
    k = "_ZN4mpcg12k_solve_wideILi0ELb1EdLi1ELb1EEEvNS_8WideArgsE"
    assert u[k] == {"VGPRs": 256, "ScratchSize [bytes/lane]": 128, "Occupancy [waves/SIMD]": 2,
                    "SGPRs Spill": 341, "LDS Size [bytes/block]": 4096}
    assert u["_ZN4mpcg11k_sched_keyElPKdPfPi"] == {"VGPRs": 12}


def test_parallel_build_units_cover_every_instance_group():
    """The parallel build compiles mpcg_wide_inst.hip once per group: the groups it names are
    exactly the groups of the instance lists in mpcg_wide_kern.h (a group without a unit would
    leave its kernels undefined at link time; a unit without instances is wasted), and every
    solve instance's (model, split, blocks) has an fp64 resume instance (its parked problems, and
    the fp32 solver's escalations)."""
    import re

    from mpc_ros_amd import build

    text = open(os.path.join(build.CSRC, "mpcg_wide_kern.h")).read()
    solve = re.findall(r"X\((\d+), (\d), (true|false), (double|float), (\d), (true|false), (\d)\)", text)
    resume = re.findall(r"X\((\d+), (\d), (true|false), (double|float), (\d)\)", text)
    assert solve and resume
    groups = {int(g[0]) for g in solve} | {int(g[0]) for g in resume}
    units = [u for u in build.compile_units() if u[0] == build.INST]
    assert sorted(int(u[1][0].split("=")[1]) for u in units) == sorted(groups) == list(range(build.N_INST))
    res = {tuple(r[1:]) for r in resume}
    for _g, m, sp, ty, nb, _d, _w in solve:
        # (the fp32 solver's problems that need the restoration phase are solved again by the
        # fp64 resume instance of the same horizon)
        assert (m, sp, "double", nb) in res
    # every source of the library is compiled exactly once besides the instance groups
    others = [u[0] for u in build.compile_units() if u[0] != build.INST]
    assert sorted(others) == sorted(s for s in build.SOURCES if s != build.INST)
