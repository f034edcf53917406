"""configs[2] rows whose fp32 phase ends in another local minimum (diagnostic, GPU).

    python tools/fp32_minima_probe.py OUT.npz [B] [N]

Solves the bench's infinity set (B problems, horizon N, generated on the device) three ways --
the fp64 solver, the fp32 phase alone (no_restoration = 1: its own ending), the two-phase fp32
configuration -- and saves per row: inputs, u0, objective, iterations, status, diag."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mpc_ros_amd import params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402


def main():
    out = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    dev = torch.device("cuda:0")
    P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
    res = {}
    for name, s in (("f64", BatchSolver(0, P)), ("f32only", BatchSolver(0, P, dtype="fp32", no_restoration=1)),
                    ("f32", BatchSolver(0, P, dtype="fp32"))):
        pose, vel, plan = s.synth_infinity_device(0, B)
        st = torch.empty((B, 6), dtype=torch.float64, device=dev)
        cf = torch.empty((B, 4), dtype=torch.float64, device=dev)
        s.preprocess_device(pose, vel, plan, st, cf)
        u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        obj = torch.empty(B, dtype=torch.float64, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        diag = torch.empty((B, 4), dtype=torch.int32, device=dev)
        s.solve_device(st, cf, u0, status=status, obj=obj, iters=iters, diag=diag)
        torch.cuda.synchronize()
        for k, v in dict(u0=u0, status=status, obj=obj, iters=iters, diag=diag).items():
            res[f"{name}_{k}"] = v.cpu().numpy()
        res["state"], res["coeffs"] = st.cpu().numpy(), cf.cpu().numpy()
        print(name, "done", flush=True)
    np.savez_compressed(out, **res)
    om = np.abs(res["f32_obj"] - res["f64_obj"]) > 1e-6 * np.abs(res["f64_obj"])
    print("other minima:", np.flatnonzero(om).tolist())


if __name__ == "__main__":
    main()
