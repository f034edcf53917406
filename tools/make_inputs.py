"""Write the benchmark batch as <outdir>/inputs_<B>.bin (default tools/, the tools use exp/) ([int64 B][B x 6 state][B x 4 coeffs]),
the input format of the diagnostic tools (wide_time.hip, wide_prof.hip).

    python tools/make_inputs.py [B] [outdir]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import infinity  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
st, cf = infinity.make_problems(np.arange(B))
outdir = sys.argv[2] if len(sys.argv) > 2 else os.path.dirname(os.path.abspath(__file__))
os.makedirs(outdir, exist_ok=True)
out = os.path.join(outdir, f"inputs_{B}.bin")
with open(out, "wb") as f:
    f.write(np.int64(B).tobytes())
    f.write(np.ascontiguousarray(st, dtype=np.float64).tobytes())
    f.write(np.ascontiguousarray(cf, dtype=np.float64).tobytes())
print(out)
