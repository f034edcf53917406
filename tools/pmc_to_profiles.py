"""Copy the PMC summaries of a tools/gpu_r5.sh run (gpurun_out/<tag>/pmc_<cfg>/summary.json) to
the names bench.py reads its roofline traffic from (profiles/<round>/pmc_<model>_<mode>_<dtype>_B<B>_N<N>.json,
round = $MPCG_PROFILE_ROUND, default r6).

    python tools/pmc_to_profiles.py gpurun_out/r6f"""
import json
import os
import shutil
import sys

NAMES = {"n20": "diffdrive_solve_fp64_B65536_N20", "n40": "diffdrive_solve_fp64_B65536_N40",
         "bic25": "bicycle_solve_fp64_B65536_N25", "n40f32": "diffdrive_solve_fp32_B65536_N40",
         "b4096": "diffdrive_solve_fp64_B4096_N20"}
src = sys.argv[1]
root = os.path.join(os.path.dirname(__file__), "..", "profiles", os.environ.get("MPCG_PROFILE_ROUND", "r6"))
os.makedirs(root, exist_ok=True)
for cfg, name in NAMES.items():
    f = os.path.join(src, f"pmc_{cfg}", "summary.json")
    if os.path.exists(f):
        d = json.load(open(f))
        shutil.copy(f, os.path.join(root, f"pmc_{name}.json"))
        print(cfg, "->", name, "hbm MB", round(d.get("hbm_bytes_per_launch", 0) / 1e6, 1),
              "valu/solve", round(d.get("sq_insts_valu_per_solve", 0)))
