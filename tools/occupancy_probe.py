"""Diagnostic (a build with MPCG_EXTRA_CFLAGS=-DMPCG_LDS_PAD_ENV): batch time against problems
per CU, by padding each workgroup's LDS (MPCG_LDS_PAD bytes) -- how far the batch is bound by
the wavefronts' own latency rather than by the SIMDs' issue rate.

    python tools/occupancy_probe.py N pad [pad ...]"""
import os
import subprocess
import sys

N = int(sys.argv[1])
for pad in sys.argv[2:]:
    env = dict(os.environ, MPCG_LDS_PAD=pad)
    out = subprocess.run([sys.executable, "bench.py", "--horizon", str(N), "--steps", "10", "--warmup", "2",
                          "--cpu-seconds", "0"], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if out.returncode or not line:
        print("pad", pad, "failed", out.returncode, out.stderr[-500:], flush=True)
        sys.exit(1)
    import json
    d = json.loads(line[-1])
    print(f"N {N} pad {pad}: {d['ms_per_step']:.3f} ms/step", flush=True)
