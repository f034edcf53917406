"""Build libmpcg.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m mpc_ros_amd.build [--force] [--verbose]
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmpcg.so")
SOURCES = [os.path.join(CSRC, f) for f in ("mpcg_kernels.hip", "mpcg_wide.hip", "mpcg_track.hip", "mpcg_api.cpp", "mpc_planner.cpp")]
HEADERS = [os.path.join(CSRC, f) for f in ("ipm_core.h", "wide_core.h", "wave_dev.h", "mpcg_internal.h")] + [
    os.path.join(ROOT, "include", f) for f in ("mpcg.h", "mpc_planner.h")]
ARCH = os.environ.get("MPCG_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    return "hipcc"


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-unused-value",
           f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]
    if verbose:
        cmd.append("-Rpass-analysis=kernel-resource-usage")
    cmd += SOURCES + ["-o", LIB + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        sys.stderr.write(r.stderr)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="--verbose" in sys.argv))
