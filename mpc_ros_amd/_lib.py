"""ctypes binding of libmpcg.so (include/mpcg.h).

The HIP library is built in-tree (``python -m mpc_ros_amd.build`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no CPU
fallback: if the library or a GPU is missing, the calls raise.

torch is imported before the library is loaded so that both share the one HIP
runtime of the process (libamdhip64.so.7 is resolved by soname); device tensors
and torch streams can then be handed to ``mpcg_solve_device`` directly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmpcg.so")


class MpcgParams(C.Structure):
    """Mirror of ``struct mpcg_params`` (include/mpcg.h)."""

    _fields_ = [
        ("steps", C.c_int32), ("model", C.c_int32),
        ("dt", C.c_double), ("ref_cte", C.c_double), ("ref_etheta", C.c_double), ("ref_v", C.c_double),
        ("w_cte", C.c_double), ("w_etheta", C.c_double), ("w_v", C.c_double), ("w_angvel", C.c_double),
        ("w_accel", C.c_double), ("w_angvel_d", C.c_double), ("w_accel_d", C.c_double),
        ("max_angvel", C.c_double), ("max_throttle", C.c_double), ("bound", C.c_double),
        ("tol", C.c_double), ("max_iter", C.c_int32), ("filter_cap", C.c_int32),
        ("bound_relax_factor", C.c_double), ("mu_init", C.c_double), ("wheelbase", C.c_double),
        ("max_cpu_time", C.c_double),
        ("acceptable_tol", C.c_double), ("acceptable_dual_inf_tol", C.c_double),
        ("acceptable_constr_viol_tol", C.c_double), ("acceptable_compl_inf_tol", C.c_double),
        ("acceptable_obj_change_tol", C.c_double), ("kappa_soc", C.c_double),
        ("soft_resto_pderror_reduction_factor", C.c_double), ("obj_max_inc", C.c_double),
        ("tiny_step_tol", C.c_double), ("tiny_step_y_tol", C.c_double), ("dual_inf_tol", C.c_double),
        ("constr_viol_tol", C.c_double), ("compl_inf_tol", C.c_double),
        ("acceptable_iter", C.c_int32), ("max_soc", C.c_int32), ("watchdog_shortened_iter_trigger", C.c_int32),
        ("watchdog_trial_iter_max", C.c_int32), ("max_soft_resto_iters", C.c_int32),
        ("max_filter_resets", C.c_int32), ("filter_reset_trigger", C.c_int32), ("precision", C.c_int32),
        ("no_restoration", C.c_int32),
    ]


# Every symbol include/mpcg.h declares, with its ctypes signature.
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_PP = C.POINTER(MpcgParams)


class MpcgXfer(C.Structure):
    """mpcg_xfer (include/mpcg.h): one gather message of mpcg_solve_multi."""
    _fields_ = [("src_offset", C.c_size_t), ("dst_offset", C.c_size_t), ("bytes", C.c_size_t)]


GATHER_ARRAYS = 5  # MPCG_GATHER_ARRAYS
SIGNATURES = {
    "mpcg_abi_version": ([], C.c_int),
    "mpcg_build_id": ([], C.c_char_p),
    "mpcg_last_error": ([], C.c_char_p),
    "mpcg_params_default": ([_PP], C.c_int),
    "mpcg_params_plugin_default": ([_PP], C.c_int),
    "mpcg_params_set": ([_PP, C.c_char_p, C.c_double], C.c_int),
    "mpcg_params_check": ([_PP], C.c_int),
    "mpcg_create": ([C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "mpcg_destroy": ([C.c_void_p], None),
    "mpcg_set_params": ([C.c_void_p, _PP], C.c_int),
    "mpcg_get_params": ([C.c_void_p, _PP], C.c_int),
    "mpcg_workspace_bytes": ([_PP, C.c_int64], C.c_size_t),
    "mpcg_handle_workspace_bytes": ([C.c_void_p, C.c_int64], C.c_size_t),
    "mpcg_reserve": ([C.c_void_p, C.c_int64], C.c_int),
    "mpcg_solve": ([C.c_void_p, C.c_int64, _dp, _dp, _dp, _dp, _ip, _dp, _ip], C.c_int),
    "mpcg_solve_device": ([C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                           C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mpcg_solve_ex": ([C.c_void_p, C.c_int64, _dp, _dp, _dp, _dp, _ip, _dp, _ip, _ip], C.c_int),
    "mpcg_solve_device_ex": ([C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mpcg_preprocess_device": ([C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mpcg_track_device": ([C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    "mpcg_synchronize": ([C.c_void_p], C.c_int),
    "mpcg_solve_multi": ([C.c_int, C.POINTER(C.c_int), _PP, C.c_int64, _dp, _dp, _dp, _dp, _ip, _dp, _ip], C.c_int),
    "mpcg_shard_range": ([C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)], C.c_int),
    "mpcg_multi_gather_plan": ([C.c_int64, C.c_int32, C.c_int, C.c_int, C.c_void_p], C.c_int),
    "mpcg_multi_out_bytes": ([C.c_int64, C.c_int32], C.c_size_t),
    "mpcg_multi_buffer_bytes": ([C.c_int64, C.c_int32, C.c_int, C.c_int], C.c_size_t),
    "mpcg_multi_create": ([C.c_int, C.POINTER(C.c_int), _PP, C.c_int64, C.POINTER(C.c_void_p)], C.c_int),
    "mpcg_multi_solve": ([C.c_void_p, C.c_int64, _dp, _dp, _dp, _dp, _ip, _dp, _ip], C.c_int),
    "mpcg_multi_destroy": ([C.c_void_p], None),
    "mpcg_set_strategy": ([C.c_void_p, C.c_int32], C.c_int),
    "mpcg_get_strategy": ([C.c_void_p], C.c_int),
    "mpcg_set_park_capacity": ([C.c_void_p, C.c_int64], C.c_int),
    "mpcg_last_kernel": ([C.c_void_p], C.c_char_p),
    "mpcg_last_solve_order": ([C.c_void_p], C.c_int),
    "mpcg_synth_infinity_device": ([C.c_void_p, C.c_uint64, C.c_int64, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p], C.c_int),
}

STRATEGY = {"auto": 0, "lane": 1, "wave": 2}  # (LANE was removed in ABI 2: selecting it raises)
ABI_VERSION = 2

_lib = None


class MpcgError(RuntimeError):
    pass


def lib():
    """Load libmpcg.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MpcgError(f"{LIB_PATH} not found: build it with `python -m mpc_ros_amd.build`")
        import torch  # noqa: F401  -- share torch's HIP runtime (see module docstring)
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.mpcg_abi_version() != ABI_VERSION:
            raise MpcgError("libmpcg ABI version mismatch")
        from . import build

        want, got = build.build_id(), L.mpcg_build_id().decode()
        if got != want:
            raise MpcgError(f"{LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                            "rebuild with `python -m mpc_ros_amd.build`")
        _lib = L
    return _lib


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise MpcgError(f"{what} failed ({rc}): {lib().mpcg_last_error().decode()}")
    return rc


def params_from_map(m: dict, base: str = "plugin") -> MpcgParams:
    """mpcg_params from a reference-style parameter map (the 15 LoadParams keys)."""
    p = MpcgParams()
    L = lib()
    check((L.mpcg_params_plugin_default if base == "plugin" else L.mpcg_params_default)(C.byref(p)), "defaults")
    for k, v in m.items():
        L.mpcg_params_set(C.byref(p), k.encode(), float(v))
    return p
