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
SOURCES = [os.path.join(CSRC, f) for f in ("mpcg_wide.hip", "mpcg_wide_inst.hip", "mpcg_track.hip", "mpcg_synth.hip",
                                           "mpcg_api.cpp", "mpcg_multi.cpp", "mpc_planner.cpp")]
INST = os.path.join(CSRC, "mpcg_wide_inst.hip")
N_INST = 12  # MPCG_INST groups of mpcg_wide_inst.hip (mpcg_wide_kern.h)
HEADERS = [os.path.join(CSRC, f) for f in ("ipm_core.h", "wide_core.h", "wave_dev.h", "mpcg_internal.h",
                                           "mpcg_wide_kern.h")] + [
    os.path.join(ROOT, "include", f) for f in ("mpcg.h", "mpc_planner.h")]
ARCH = os.environ.get("MPCG_OFFLOAD_ARCH", "gfx950")


def source_hash() -> str:
    """Hash of every source and header the library is built from (baked into the library
    as mpcg_build_id(); the loader refuses a library built from other sources)."""
    import hashlib

    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    return "hipcc"


def built_id(lib: str = LIB) -> str | None:
    """mpcg_build_id() of a built library, read from its file (no GPU runtime needed)."""
    if not os.path.exists(lib):
        return None
    with open(lib, "rb") as fh:
        data = fh.read()
    i = data.find(b"MPCG-BUILD-ID:")
    return data[i + 14:data.find(b"\0", i)].decode() if i >= 0 else None


def extra_cflags() -> list:
    """MPCG_EXTRA_CFLAGS (diagnostic builds only, e.g. -DMPCG_DEBUG_GUARD)."""
    return os.environ.get("MPCG_EXTRA_CFLAGS", "").split()


def build_id() -> str:
    """The sources' hash, + the extra flags of a diagnostic build: such a library never passes
    for the product (the loader compares against the id of the environment it runs in)."""
    x = extra_cflags()
    return source_hash() + ("+" + "".join(c for c in "_".join(x) if c.isalnum() or c == "_") if x else "")


def stale() -> bool:
    return built_id() != build_id()


def compile_units() -> list:
    """(source, extra flags, object name) of every translation unit: the kernel instance
    groups of mpcg_wide_inst.hip (the bulk of the compile time) and the other sources."""
    units = [(INST, [f"-DMPCG_INST={g}"], f"inst{g}.o") for g in range(N_INST)]
    units += [(s, [], os.path.basename(s) + ".o") for s in SOURCES if s != INST]
    return units


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    if not force and not stale():
        return LIB
    # (-disable-promote-alloca-to-lds: the solver owns the whole dynamic LDS from address 0;
    # the backend would otherwise move a private array into static LDS, which the launch
    # refuses -- mpcg_wide.hip checks sharedSizeBytes == 0)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-mllvm", "-disable-promote-alloca-to-lds", "-mllvm", "-disable-machine-licm",
             "-Wno-unused-result", "-Wno-unused-value",
             f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}", "-Rpass-analysis=kernel-resource-usage"]
    # (diagnostic builds only: extra compiler flags, part of the build id)
    flags += [f'-DMPCG_BUILD_ID="MPCG-BUILD-ID:{build_id()}"'] + extra_cflags()
    tmp = tempfile.mkdtemp(prefix="mpcg_build_")
    try:
        def cc(unit):
            src, extra, obj = unit
            cmd = [hipcc(), "-c"] + flags + extra + [src, "-o", os.path.join(tmp, obj)]
            return cmd, subprocess.run(cmd, capture_output=True, text=True)

        units = compile_units()
        jobs = jobs or min(len(units), max(1, min(os.cpu_count() or 1, 16)))
        with ThreadPoolExecutor(jobs) as ex:
            results = list(ex.map(cc, units))
        remarks = ""
        for cmd, r in results:
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            remarks += r.stderr
        link = [hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared"] + [os.path.join(tmp, u[2]) for u in units] + [
            "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-o", LIB + ".tmp"]
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if verbose:
        sys.stderr.write(remarks)
    usage = kernel_resources(remarks)
    bad = [k for k, u in usage.items() if ("k_solve_wide" in k or "k_resume_wide" in k) and u.get("LDS Size [bytes/block]", 0) != 0]
    if bad:
        os.remove(LIB + ".tmp")
        raise RuntimeError(f"static LDS in {bad}: the solver addresses its dynamic LDS from 0")
    os.replace(LIB + ".tmp", LIB)
    save_resources(usage)
    return LIB


RESOURCES = os.path.join(ROOT, "profiles", "r6", "resources.json")


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return dict(zip(names, out))
    except OSError:
        return {n: n for n in names}


def save_resources(usage: dict, path: str = RESOURCES) -> None:
    """Register / spill / scratch / occupancy figures of every solver kernel instance and of the
    restoration phase's out-of-line function, from the build's kernel-resource-usage remarks."""
    import json

    keep = {k: v for k, v in usage.items() if "k_solve_wide" in k or "k_resume_wide" in k or "resto_phase" in k}
    names = demangle(sorted(keep))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"build_id": source_hash(), "arch": ARCH,
                   "functions": {names[k]: keep[k] for k in sorted(keep)}}, f, indent=1)


def kernel_resources(remarks: str) -> dict:
    """Per-kernel resource usage from hipcc's kernel-resource-usage remarks
    ({mangled name: {"VGPRs": .., "SGPRs Spill": .., "Occupancy [waves/SIMD]": .., ...}})."""
    import re

    out, cur = {}, None
    for line in remarks.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z][^:]*?):\s+(-?\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="--verbose" in sys.argv))
