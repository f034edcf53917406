"""The C-ABI library: loads, exports every symbol include/*.h declares, parameter
handling -- all without a GPU (no compute calls here)."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def declared_functions(header: str) -> list[str]:
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mpcg_[a-z_0-9]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(libmpcg):
    from mpc_ros_amd import _lib

    names = declared_functions("mpcg.h")
    assert len(names) >= 15
    for n in names:
        assert hasattr(libmpcg, n), n
        assert n in _lib.SIGNATURES, f"{n} missing from the ctypes signature table"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    # class MPC (include/mpc_planner.h): ctor, LoadParams, SolveRaw behind the Solve template, SolveBatch
    for mangled in ("_ZN3MPCC1Ev", "_ZN3MPC10LoadParams", "_ZN3MPC8SolveRawEPKdS1_", "_ZN3MPC10SolveBatch",
                    "_ZN3MPCD1Ev"):
        assert mangled in out, mangled


def test_abi_version_and_struct_size(libmpcg):
    from mpc_ros_amd import _lib

    assert libmpcg.mpcg_abi_version() == _lib.ABI_VERSION == 2
    # C struct layout: compile a tiny probe against the header and compare sizeof/offsets
    src = ("#include <stdio.h>\n#include <stddef.h>\n#include \"mpcg.h\"\nint main(){printf(\"%zu %zu %zu %zu %zu %zu\","
           "sizeof(mpcg_params),offsetof(mpcg_params,tol),offsetof(mpcg_params,filter_cap),"
           "offsetof(mpcg_params,wheelbase),offsetof(mpcg_params,max_cpu_time),"
           "offsetof(mpcg_params,filter_reset_trigger));}\n")
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "p.c"), "w").write(src)
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", os.path.join(d, "p"),
                               os.path.join(d, "p.c")])
        got = [int(v) for v in subprocess.check_output([os.path.join(d, "p")]).split()]
    P = _lib.MpcgParams
    assert got == [C.sizeof(P), P.tol.offset, P.filter_cap.offset, P.wheelbase.offset, P.max_cpu_time.offset,
                   P.filter_reset_trigger.offset]


def test_build_id_is_the_source_hash(libmpcg):
    """The library carries the hash of the sources it was built from; the loader refuses
    a library whose id differs from the tree's sources (no stale binary on a GPU box)."""
    from mpc_ros_amd import build

    assert libmpcg.mpcg_build_id().decode() == build.source_hash() == build.built_id()


def test_param_defaults_and_keys(libmpcg):
    from mpc_ros_amd import _lib

    p = _lib.MpcgParams()
    assert libmpcg.mpcg_params_default(C.byref(p)) == 0
    assert (p.steps, p.max_angvel, p.max_throttle, p.bound) == (20, 3.0, 1.0, 1000.0)
    assert (p.dt, p.ref_v, p.w_cte, p.w_etheta, p.w_v, p.w_angvel, p.w_accel) == (0.1, 0.5, 100, 100, 1, 100, 50)
    assert (p.tol, p.max_iter, p.bound_relax_factor, p.mu_init) == (1e-8, 3000, 1e-8, 0.1)
    # the reference's max_cpu_time and Ipopt 3.12's defaults for the line-search mechanisms
    assert (p.max_cpu_time, p.acceptable_tol, p.acceptable_iter, p.max_soc, p.kappa_soc) == (0.5, 1e-6, 15, 4, 0.99)
    assert (p.watchdog_shortened_iter_trigger, p.watchdog_trial_iter_max, p.max_soft_resto_iters) == (10, 3, 10)
    assert (p.soft_resto_pderror_reduction_factor, p.obj_max_inc, p.max_filter_resets) == (0.9999, 5.0, 5)
    assert libmpcg.mpcg_params_plugin_default(C.byref(p)) == 0
    assert (p.ref_v, p.w_cte, p.w_accel_d, p.max_angvel) == (1.0, 1000, 10, 1.0)
    assert libmpcg.mpcg_params_set(C.byref(p), b"STEPS", 33.7) == 0 and p.steps == 33
    assert libmpcg.mpcg_params_set(C.byref(p), b"W_EPSI", 12.0) == 0 and p.w_etheta == 12.0
    assert libmpcg.mpcg_params_set(C.byref(p), b"NOT_A_KEY", 1.0) == 1
    assert libmpcg.mpcg_params_check(C.byref(p)) == 0
    p.steps = 1
    assert libmpcg.mpcg_params_check(C.byref(p)) < 0
    assert b"STEPS" in libmpcg.mpcg_last_error()
    p.steps = 20
    p.w_v = -1
    assert libmpcg.mpcg_params_check(C.byref(p)) < 0


def test_workspace_bytes(libmpcg):
    """Workspace slots per resident wavefront (not per problem), in 8 equal per-XCD
    partitions of at least min(B, 32), and a park area for the problems that enter the
    restoration phase, plus the solve-order buffers beyond 2048.  Four 256-byte blocks of
    flags and counters (slot flags, park count/taken/done, park indices, park ready flags)
    precede them.  N = 20: a slot is 114N + 2*448 = 3176 doubles (rare-path copies and the
    filter entries beyond the 64 held in LDS) rounded to whole 128-byte lines, 3184; a park
    entry 32 + 2372 (LDS image) + 11684 (a slot, 2372 for the original problem's image, 262N
    of restoration records -- 190N of them per stage, iterative-refinement residuals and saved
    steps included -- and the restoration filter's overflow) = 14088, 14096 in whole lines;
    without a GPU the slot count falls back to 4096."""
    from mpc_ros_amd import _lib

    p = _lib.MpcgParams()
    libmpcg.mpcg_params_plugin_default(C.byref(p))
    b1 = libmpcg.mpcg_workspace_bytes(C.byref(p), 1)
    assert b1 == 4 * 256 + (8 * 3184 + 14096) * 8
    b2 = libmpcg.mpcg_workspace_bytes(C.byref(p), 2)
    assert b2 == 4 * 256 + (16 * 3184 + 2 * 14096) * 8
    big = libmpcg.mpcg_workspace_bytes(C.byref(p), 65536)
    assert big < 65536 * 3184 * 8 // 4  # (bounded by residency, not by B)
    assert libmpcg.mpcg_workspace_bytes(C.byref(p), 0) == 0
    assert libmpcg.mpcg_handle_workspace_bytes(None, 1) == 0  # (no handle: nothing)
    # the fp32 configuration: + the hand-over (4 + 30N floats per problem in whole 128-byte
    # lines: 608 at N = 20), the fp64 phase's order and, beyond 2048 problems, the head's own
    # workspace (B / 1024 problems of the fp64 solver, a park entry each)
    p.precision = 1
    w2048 = libmpcg.mpcg_workspace_bytes(C.byref(p), 2048)
    w2049 = libmpcg.mpcg_workspace_bytes(C.byref(p), 2049)
    assert w2048 >= 2048 * 608 * 4
    assert w2049 - w2048 >= 608 * 4 + 2 * 14096 * 8  # (one more hand-over row, the head's park entries)
    assert libmpcg.mpcg_last_solve_order(None) == 0


def test_create_without_gpu_fails_loudly(libmpcg):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    rc = libmpcg.mpcg_create(0, C.byref(h))
    assert rc < 0 and not h.value
    assert libmpcg.mpcg_last_error()


def test_product_refuses_to_run_without_gpu():
    """No CPU fallback anywhere in the product: solver construction raises."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mpc_ros_amd import _lib
    from mpc_ros_amd.solver import BatchSolver

    with pytest.raises(_lib.MpcgError):
        BatchSolver(0)


def test_product_package_never_imports_oracle():
    """The product (mpc_ros_amd/) never imports, includes or links the oracle."""
    pkg = os.path.join(ROOT, "mpc_ros_amd")
    bad = re.compile(r"(^\s*(import|from)\s+oracle\b|pyoracle|liboracle|#\s*include\s*[\"<][^\">]*ora\.h)", re.M)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not bad.search(txt), f


def test_multi_gpu_shard_and_gather_plan(libmpcg):
    """mpcg_solve_multi's arithmetic through the C-ABI (no GPU): shards contiguous and
    balanced (B % G != 0, empty shards for B < G); for each of the five output arrays the
    messages of all GPUs tile the root's gathered buffer exactly once; rank 0's slot is in
    place; the bytes per GPU are count x (32 + 24 N)."""
    from mpc_ros_amd import _lib

    for B, G, N in ((7, 3, 20), (2, 4, 20), (524288, 8, 20), (65537, 8, 40), (1, 1, 3), (0, 2, 20)):
        total = libmpcg.mpcg_multi_out_bytes(B, N)
        assert total == B * (32 + 24 * N)
        cover = np.zeros(total, dtype=np.int32)
        start, count = C.c_int64(), C.c_int64()
        nxt = 0
        for r in range(G):
            assert libmpcg.mpcg_shard_range(B, G, r, C.byref(start), C.byref(count)) == 0
            assert start.value == nxt and count.value == B // G + (1 if r < B % G else 0)
            nxt += count.value
            x = (_lib.MpcgXfer * _lib.GATHER_ARRAYS)()
            assert libmpcg.mpcg_multi_gather_plan(B, N, G, r, x) == 0
            assert sum(m.bytes for m in x) == count.value * (32 + 24 * N)
            for m in x:
                if r == 0:
                    assert m.src_offset == m.dst_offset
                cover[m.dst_offset:m.dst_offset + m.bytes] += 1
        assert nxt == B
        assert (cover == 1).all()
    assert libmpcg.mpcg_shard_range(10, 2, 2, C.byref(start), C.byref(count)) < 0
    assert libmpcg.mpcg_last_error()


def test_multi_context_buffers_and_no_gpu(libmpcg):
    """The persistent multi-GPU context's per-GPU device buffers (mpcg_multi_buffer_bytes): every
    GPU holds the inputs of the largest shard (80 B per problem); the root the gathered outputs
    of B_max problems, the others their shard's outputs (32 + 24 N B per problem) -- summed
    over the GPUs, the outputs are B_max + (G - 1) largest shards.  Creating a context without a
    GPU fails with an error, never a CPU fallback."""
    import torch

    for B, G, N in ((524288, 8, 20), (65537, 8, 40), (7, 3, 20), (2, 4, 20), (1, 1, 3)):
        cmax = -(-B // G)
        per_out = 32 + 24 * N
        for r in range(G):
            got = libmpcg.mpcg_multi_buffer_bytes(B, N, G, r)
            out = (B if r == 0 else cmax) * per_out
            assert got == 80 * max(cmax, 1) + max(out, 1)
    assert libmpcg.mpcg_multi_buffer_bytes(10, 20, 2, 2) == 0 and libmpcg.mpcg_multi_buffer_bytes(10, 0, 2, 0) == 0
    if torch.cuda.is_available():
        return
    from mpc_ros_amd import _lib

    p = _lib.MpcgParams()
    libmpcg.mpcg_params_plugin_default(C.byref(p))
    dev = (C.c_int * 2)(0, 1)
    h = C.c_void_p()
    assert libmpcg.mpcg_multi_create(2, dev, C.byref(p), 1024, C.byref(h)) < 0 and not h.value
    assert libmpcg.mpcg_last_error()
    libmpcg.mpcg_multi_destroy(None)
