"""DIAGNOSTIC: build tools/diag_stamps.hip, run it on the benchmark batch, print per-pass shares."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_ros_amd import infinity
out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
exe = os.path.join(out, "diag_stamps")
extra = os.environ.get("DIAG_FLAGS", "").split()
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-w", "-I", os.path.join(ROOT, "mpc_ros_amd", "csrc"),
                       os.path.join(ROOT, "tools", "diag_stamps.hip"), "-o", exe] + extra)
st, cf = infinity.make_problems(np.arange(B))
with open(os.path.join(out, "inputs.bin"), "wb") as f:
    np.array([B], dtype=np.int64).tofile(f)
    np.concatenate([st, cf], 1).astype(np.float64).tofile(f)
print(subprocess.check_output(["timeout", "-k", "10", "300", exe, os.path.join(out, "inputs.bin"), os.path.join(out, "diag.bin")]).decode())
d = np.fromfile(os.path.join(out, "diag.bin"), dtype=np.uint64).reshape(B, 8).astype(np.float64)
it = d[:, 6]
names = ["stats", "riccati", "forward", "linesearch", "accept"]
tot = d[:, 5]
print("iters mean %.2f max %d" % (it.mean(), it.max()))
sl = np.argmax(it)
print("slowest problem: iters %d total %.3e cycles -> %.1f us/iter" % (it[sl], tot[sl], tot[sl] / it[sl] / 100.0))
for j, n in enumerate(names):
    print("%-10s share %.3f   cycles/iter (mean over problems) %.0f" % (n, d[:, j].sum() / d[:, :5].sum(), (d[:, j] / np.maximum(it, 1)).mean()))
print("cycles/iter overall mean %.0f" % ((tot / np.maximum(it, 1)).mean()))
print("slowest problem per pass cycles/iter:", " ".join("%s=%.0f" % (n, d[sl, j] / it[sl]) for j, n in enumerate(names)))
waves = it[: (B // 64) * 64].reshape(-1, 64).max(1)
print("per-wave max iters: mean %.1f p50 %d p90 %d p99 %d max %d" % (waves.mean(), np.percentile(waves, 50), np.percentile(waves, 90), np.percentile(waves, 99), waves.max()))
