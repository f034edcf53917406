"""Benchmark: NMPC solves/s of the MPC::Solve hot path on MI355X.

    python bench.py [--gpus N --steps K --warmup W --batch B --horizon N]

With --gpus N > 1 and no torch.distributed environment (RANK/WORLD_SIZE unset), the
process launches N ranks itself -- `python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 ... bench.py <same args>` as a child -- before anything touches
the GPU, and exits with the child's code.  Under an outside launcher WORLD_SIZE must
equal --gpus (a mismatch is an error, never a silently smaller run).

A step = one pass of the hot path over one batch: every rank solves its shard of
B problems (BASELINE.json configs[3]: 524288 problems over 8 GPUs = 65536 per GPU,
N = 20, fp64, differential drive) with the HIP kernel, then the controls and
statuses are gathered to rank 0 (torch.distributed.gather: RCCL point-to-point over
xGMI, each rank sends its slice only) -- the only exchange.  Each rank generates its shard of
the synthetic robots on its own GPU from (seed, global index) (mpcg_synth_infinity_device) and
preprocesses them there (findBestPath, mpcg_preprocess_device); the inputs are resident in HBM
before the timed region (weak scaling: the per-GPU batch is fixed).  Rank 0 prints one JSON line.

roofline: the dominant kernel, mpcg::k_solve_wide (one problem per wavefront, whole
problem state in LDS; the restoration phase's k_resume_wide runs beside it on a second
stream and both are inside the timed events).  The path is not HBM-bound (SURVEY.md
§8d): it is FP64 vector-ALU issue/latency bound, so bound = "valu_fp64" and achieved =
the useful flops of SURVEY.md §8d's formula (iterations x Riccati and forward-pass flops
per stage, per solve) x the solves of one launch / the launch's average duration
(HIP events on the stream it runs on), against the FP64 vector peak.  traffic =
memory-side bytes per launch (FETCH_SIZE + WRITE_SIZE) from the committed rocprofv3 PMC
summary of this exact configuration (profiles/r6/pmc_<model>_<mode>_<dtype>_B<B>_N<N>.json),
or null.  The line also carries hbm = algorithmic bytes per launch (B x 8 x (6 + 4 + 2 +
3N) = B x 576 B at N = 20) / kernel time against 8 TB/s, and valu_fp64 = PMC-counted
FP64 lane-FLOPs (redundant lanes included) / kernel time.
cpu_baseline: the oracle (the Ipopt restatement, "port") on a bounded sample of the
same problems, rank 0, N = 1 only: its KKT systems in stage order factored within their
band (the structured linear algebra, as Ipopt's sparse solver would) as the value, the
checker's dense factorisation as a second figure.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_VALU_PEAK_TFLOPS = 78.6
FP32_VALU_PEAK_TFLOPS = 157.3


def algorithmic_flops_per_solve(N: int, iters_mean: float) -> float:
    """iters x [(N - 1) F_stage + 60 N], F_stage = 4n^3 + 6n^2 m + 4 n m^2 + 2n^2
    + 4nm of the dense Riccati stage and forward pass at n = 8 (state + previous control),
    m = 2: 3136 flop."""
    n, m = 8, 2
    f_stage = 4 * n ** 3 + 6 * n * n * m + 4 * n * m * m + 2 * n * n + 4 * n * m
    return iters_mean * ((N - 1) * f_stage + 60 * N)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=80, help="timed steps (default: a timed region of ~1.3 s)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="problems per GPU")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--gather-traj", action="store_true", help="also gather the 3N trajectories")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget (0 = skip)")
    ap.add_argument("--profile-name", default=None, help="PMC summary to read traffic from")
    ap.add_argument("--strategy", default="auto", choices=["auto", "wave"],
                    help="kernel strategy: one problem per wavefront (the only one)")
    ap.add_argument("--model", default="diffdrive", choices=["diffdrive", "bicycle"],
                    help="dynamics: FG_eval's differential drive, or the kinematic bicycle (BASELINE configs[4]: "
                         "run with --horizon 25)")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"],
                    help="solver arithmetic: fp64 (the reference's) or the fp32 solver (BASELINE configs[2]: "
                         "run with --horizon 40)")
    ap.add_argument("--selftest", action="store_true",
                    help="launch/shard/gather plumbing only: gloo on CPU, a stub solver that writes each "
                         "problem's global index (tests/test_bench_launch.py); no GPU, no timing claim")
    ap.add_argument("--restoration", default="auto", choices=["auto", "on", "off"],
                    help="Ipopt's feasibility-restoration phase: auto = the dtype's default (fp64: on; fp32: the "
                         "two phases, fp32 then fp64), on / off = mpcg_params.no_restoration 0 / 1 (fp32 off: the "
                         "fp32 phase alone)")
    ap.add_argument("--inputs", default="device", choices=["device", "host"],
                    help="where each rank generates its shard of the synthetic robots from (seed, global index): "
                         "device = mpcg_synth_infinity_device + the device preprocessing (findBestPath); host = "
                         "infinity.py (numpy) and a copy in")
    ap.add_argument("--mode", default="solve", choices=["solve", "track"],
                    help="solve: MPC::Solve on preprocessed inputs (the metric); track: the whole control "
                         "tick from raw poses and waypoint plans (findBestPath + solve + post-processing)")
    return ap.parse_args()


def host_cpu():
    """(threads available to this process, CPU model name)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)  # the box's CPU share when set
    threads = max(1, min(n, env) if env > 0 else n)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, model


def _time_oracle(O, P, st, cf, opts, threads, budget_s):
    """Solves/s of the oracle on the first problems of the batch within about budget_s."""
    n = threads * 8  # (pilot: long enough that thread start-up does not inflate the estimate)
    t0 = time.perf_counter()
    O.mpc_solve_batch(P, st[:n], cf[:n], opts=opts, nthreads=threads)
    per = (time.perf_counter() - t0) / n
    m = int(max(n, min(len(st), budget_s / max(per, 1e-6))))
    t0 = time.perf_counter()
    r = O.mpc_solve_batch(P, st[:m], cf[:m], opts=opts, nthreads=threads)
    dt = time.perf_counter() - t0
    return m / dt, m, dt, float(np.mean(r["iters"]))


def cpu_baseline(P, st, cf, budget_s):
    """The Ipopt restatement (oracle/ipm.c) timed on the host cores this process may use:
    value = its KKT systems in stage order factored within their band (kkt_structured: the
    cost of Ipopt's sparse LDL^T on this block-tridiagonal system, the same algorithm the
    GPU runs); dense_value = the checker's dense Bunch-Kaufman, as a second figure."""
    from oracle import pyoracle as O

    O.build()
    threads, model = host_cpu()
    opts = O.ref_opts(int(P["STEPS"]))
    sopts = O.ref_opts(int(P["STEPS"]))
    sopts.kkt_structured = 1
    v, m, dt, it = _time_oracle(O, P, st, cf, sopts, threads, budget_s)
    dv, dm, ddt, _ = _time_oracle(O, P, st, cf, opts, threads, budget_s / 3)
    return dict(value=v, unit="solves/s", cores=threads, kind="port", cpu_model=model,
                sample=f"first {m} problems of the benchmark batch, oracle/ipm.c (Ipopt 3.12 algorithm with SOC, "
                       f"watchdog, restoration) with the KKT matrix in stage order and an envelope Bunch-Kaufman "
                       f"LDL^T (kkt_structured), {threads} OpenMP threads, one problem per thread "
                       f"(sched_getaffinity, capped by OMP_NUM_THREADS: the box's CPU share), {dt:.1f} s",
                iters_mean=it, dense_value=dv,
                dense_sample=f"first {dm} problems, the checker's dense Bunch-Kaufman KKT, {ddt:.1f} s")


def latency_b1(P, st, cf, solver, dev, reps=50):
    """One robot per call (the reference's use: one MPC::Solve per control tick):
    device-resident launch-to-completion, the host-buffer path (copies included),
    and the oracle on one host thread; medians over repetitions of problem 0."""
    import torch

    from oracle import pyoracle as O

    s1, c1 = st[:1], cf[:1]
    ts, tc = torch.from_numpy(s1).to(dev), torch.from_numpy(c1).to(dev)
    u = torch.empty((1, 2), dtype=torch.float64, device=dev)
    dev_ms, host_ms, cpu_ms = [], [], []
    for r in range(reps + 5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        solver.solve_device(ts, tc, u)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        solver.solve(s1, c1)
        t2 = time.perf_counter()
        if r >= 5:
            dev_ms.append((t1 - t0) * 1e3)
            host_ms.append((t2 - t1) * 1e3)
    opts = O.ref_opts(int(P["STEPS"]))
    for r in range(min(reps, 20)):
        t0 = time.perf_counter()
        O.mpc_solve_batch(P, s1, c1, opts=opts, nthreads=1)
        cpu_ms.append((time.perf_counter() - t0) * 1e3)
    return {"gpu_device_ms": float(np.median(dev_ms)), "gpu_host_buffers_ms": float(np.median(host_ms)),
            "cpu_oracle_ms": float(np.median(cpu_ms)),
            "sample": f"problem 0 of the batch, B = 1, median of {reps} (GPU) / {min(reps, 20)} (CPU, 1 thread)"}


def pmc_name(a) -> str:
    """The PMC summary of exactly this configuration (model, mode, dtype, batch, horizon)."""
    off = "_norestoration" if getattr(a, "restoration", "on") == "off" else ""
    return a.profile_name or f"r6/pmc_{a.model}_{a.mode}_{a.dtype}_B{a.batch}_N{a.horizon}{off}"


def pmc_profile(name):
    path = os.path.join(ROOT, "profiles", f"{name}.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start n ranks (one process per GPU) under torch.distributed.run and wait for them.
    Runs in a parent that has not imported torch: the GPU is touched only by the children."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def selftest_main(a):
    """--selftest: the multi-rank plumbing of main() (shard, gather to rank 0, barrier,
    max over ranks) on gloo/CPU with a stub solver; rank 0 checks the gathered order."""
    import torch
    import torch.distributed as dist

    from mpc_ros_amd import dist as D

    rank, world, _ = D.env_rank_world()
    if world > 1:
        dist.init_process_group("gloo")
    total = a.batch * world
    start, count = D.shard(total, rank, world)
    u0 = torch.empty((count, 2), dtype=torch.float64)
    status = torch.empty(count, dtype=torch.int32)

    def step():
        idx = torch.arange(start, start + count, dtype=torch.float64)
        u0[:, 0] = idx
        u0[:, 1] = -idx
        status.fill_(1)
        if world > 1:
            return D.gather_rows(u0, total), D.gather_rows(status, total)
        return u0, status

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g_u0, g_st = step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    if rank == 0:
        ok = bool(torch.equal(g_u0[:, 0], torch.arange(total, dtype=torch.float64))) and bool((g_st == 1).all())
        print(json.dumps({"selftest": True, "n_gpus": world, "steps": a.steps, "total_batch": total,
                          "gather_ok": ok, "ms_per_step": elapsed / a.steps * 1e3}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "RANK" not in os.environ and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world_env}: launch with matching counts")
    if a.selftest:
        return selftest_main(a)
    import torch
    import torch.distributed as dist

    from mpc_ros_amd import dist as D
    from mpc_ros_amd import infinity, params
    from mpc_ros_amd.solver import BatchSolver

    rank, world, local = D.env_rank_world()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    N = a.horizon
    B = a.batch
    total = B * world
    P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
    if a.model == "bicycle":  # steering bound 0.5 rad, wheelbase 0.5 m (tests/golden/bicycle_N25.npz)
        P.update(MODEL=1, LF=0.5, ANGVEL=0.5)
    start, count = D.shard(total, rank, world)
    extra = {} if a.restoration == "auto" else {"no_restoration": int(a.restoration == "off")}
    solver = BatchSolver(dev.index, P, strategy=a.strategy, dtype=a.dtype, **extra)
    if a.inputs == "device":
        # this rank's robots from (seed, global index) on its GPU, preprocessed there
        tpose, tvel, tplan = solver.synth_infinity_device(start, count)
        tst = torch.empty((count, 6), dtype=torch.float64, device=dev)
        tcf = torch.empty((count, 4), dtype=torch.float64, device=dev)
        solver.preprocess_device(tpose, tvel, tplan, tst, tcf)
        torch.cuda.synchronize()
        st, cf = (tst.cpu().numpy(), tcf.cpu().numpy()) if rank == 0 else (None, None)
    else:
        st, cf = infinity.make_problems(np.arange(start, start + count))
        tst = torch.from_numpy(st).to(dev)
        tcf = torch.from_numpy(cf).to(dev)
        if a.mode == "track":
            sc = infinity.draw_scenarios(np.arange(start, start + count))
            px, py, yaw, plan = infinity.scenario_poses(sc)
            tpose = torch.from_numpy(np.ascontiguousarray(np.stack([px, py, yaw], 1))).to(dev)
            tvel = torch.from_numpy(np.ascontiguousarray(np.stack([sc["v"], sc["w_prev"], sc["a_prev"]], 1))).to(dev)
            tplan = torch.from_numpy(np.ascontiguousarray(plan)).to(dev)
    if a.mode == "track":
        cmd = torch.empty((count, 3), dtype=torch.float64, device=dev)
    solver.reserve(count)
    u0 = torch.empty((count, 2), dtype=torch.float64, device=dev)
    traj = torch.empty((count, 3, N), dtype=torch.float64, device=dev)
    status = torch.empty(count, dtype=torch.int32, device=dev)
    iters = torch.empty(count, dtype=torch.int32, device=dev)
    diag = torch.zeros((count, 4), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    k_ms = []

    g_ms = []

    def step(timed):
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        if a.mode == "track":
            solver.track_device(tpose, tvel, tplan, cmd, traj, status, stream=stream)
        else:
            solver.solve_device(tst, tcf, u0, traj, status, None, iters, stream=stream, diag=diag)
        if timed:
            e1.record(stream)
            k_ms.append((e0, e1))
        if world > 1:
            g_u0 = D.gather_rows(cmd if a.mode == "track" else u0, total)
            g_st = D.gather_rows(status, total)
            if a.gather_traj:
                D.gather_rows(traj.view(count, -1), total)
            if timed:  # (the collectives are stream-ordered before this event)
                e2 = torch.cuda.Event(enable_timing=True)
                e2.record(stream)
                g_ms.append((e1, e2))
            return g_u0, g_st
        return u0, status

    for _ in range(a.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern = float(np.mean([e0.elapsed_time(e1) for e0, e1 in k_ms])) if k_ms else float("nan")
    gath = float(np.mean([e1.elapsed_time(e2) for e1, e2 in g_ms])) if g_ms else 0.0
    per_rank = None
    if world > 1:
        # per-rank kernel and gather times, then the max over ranks
        mine = torch.tensor([elapsed, kern, gath], dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        allr = torch.stack(allr).cpu().numpy()
        per_rank = {"kernel_ms": allr[:, 1].tolist(), "gather_ms": allr[:, 2].tolist()}
        elapsed, kern, gath = float(allr[:, 0].max()), float(allr[:, 1].max()), float(allr[:, 2].max())
    if a.mode == "track":  # iteration counts of the same problems
        solver.solve_device(tst, tcf, u0, None, status, None, iters, stream=stream, diag=diag)
        torch.cuda.synchronize()
    it = iters.cpu().numpy()
    sts = status.cpu().numpy()
    dg = diag.cpu().numpy()
    # (per-rank status and diagnostic counts, summed over ranks)
    codes = list(range(16))
    mine = torch.tensor([int(np.sum(sts == c)) for c in codes] +
                        [int(np.sum(dg[:, 0] > 0)), int(dg[:, 0].sum()), int(np.sum(dg[:, 2] == 1)),
                         int(np.sum(dg[:, 2] == 3)), int(np.sum(dg[:, 2] == 4)), int(np.sum(dg[:, 1] > 0)),
                         int(dg[:, 3].max(initial=0))], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(mine[:-1])
        peak = mine[-1:].clone()
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)
        mine[-1:] = peak
    cnt = mine.cpu().numpy()
    if rank == 0:
        value = total * a.steps / elapsed
        bytes_per_solve = 8 * (6 + 4 + 2 + 3 * N)
        achieved = count * bytes_per_solve / (kern * 1e-3) / 1e9
        prof = pmc_name(a)
        pmc = pmc_profile(prof)
        traffic = pmc.get("hbm_bytes_per_launch")
        fl = pmc.get("fp64_flops_per_solve")
        valu = None
        if fl:
            got = fl * count / (kern * 1e-3) / 1e12
            valu = {"achieved": got, "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": got / FP64_VALU_PEAK_TFLOPS, "flops_per_solve": fl,
                    "source": f"profiles/{prof}.json (SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes: physical FP64 "
                              f"lane-FLOPs, replicated and idle lanes included)"}
        af = algorithmic_flops_per_solve(N, float(it.mean()))
        got_a = af * count / (kern * 1e-3) / 1e12
        peak_a = FP64_VALU_PEAK_TFLOPS if a.dtype == "fp64" else FP32_VALU_PEAK_TFLOPS
        valu_alg = {"achieved": got_a, "peak": peak_a, "unit": "TFLOP/s", "frac": got_a / peak_a,
                    "flops_per_solve": af,
                    "source": "SURVEY.md §8d: iters_mean x [(N-1) x 3136 + 60 N] (useful Riccati + forward-pass "
                              "flops) / kernel time"}
        line = {
            "metric": "NMPC solves/sec (whole node), N=20 diff-drive, at 1/2/4/8 MI355X",
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # (the fp32 configuration's default runs an fp32 phase, then an fp64 phase on the same batch)
            "dtype": "f64" if a.dtype == "fp64" else ("f32" if a.restoration == "off" else "f32+f64"),
            "data": "synthetic (infinity set: lemniscate course, findBestPath preprocessing; seeded per problem, "
                    + ("generated per rank on its GPU)" if a.inputs == "device" else "generated on the host)"),
            "config": {"workload": f"{'diff-drive' if a.model == 'diffdrive' else 'kinematic-bicycle'} NMPC "
                                   f"(MPC::Solve NLP, Ipopt algorithm), N={N}, {a.dtype}, "
                                   f"{B} problems per GPU (BASELINE configs[3] shard), gather to rank 0",
                       "batch_per_gpu": B, "total_batch": total, "horizon": N, "parallelism": f"dp{world}",
                       "mode": a.mode, "model": a.model, "dtype": a.dtype, "restoration": a.restoration},
            "roofline": {"bound": "valu_fp64" if a.dtype == "fp64" else "valu_fp32", "achieved": got_a,
                         "peak": peak_a, "unit": "TFLOP/s", "frac": got_a / peak_a, "traffic": traffic,
                         "kernel": solver.last_kernel, "kernel_ms": kern,
                         "algorithmic_flops_per_solve": af, "solves_per_launch": count,
                         "traffic_source": f"profiles/{prof}.json" if traffic else None,
                         "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes_per_solve": bytes_per_solve},
                         "valu_fp64": valu, "valu_algorithmic": valu_alg},
            "solver": {"iters_mean": float(it.mean()), "iters_max": int(it.max()),
                       "success_frac": float(cnt[1] / total),
                       "status_counts": {str(c): int(cnt[c]) for c in codes if cnt[c]},
                       "restoration": {"problems": int(cnt[16]), "phases": int(cnt[17]), "parked": int(cnt[18])},
                       # (the fp32 configuration's fp64 phase: problems solved again from the start
                       # where the fp32 solve did not converge, and continued from its iterate)
                       "fp64_phase": {"from_start": int(cnt[19]), "continued": int(cnt[20])},
                       "filter": {"problems_dropping_entries": int(cnt[21]), "peak_entries": int(cnt[22])},
                       "sample": "all problems of the last timed step, all ranks"},
            "timing": {"kernel_ms": kern, "gather_ms": gath, "per_rank": per_rank},
        }
        if world == 1 and a.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(P, st, cf, a.cpu_seconds)
            line["latency_b1"] = latency_b1(P, st, cf, solver, dev)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
