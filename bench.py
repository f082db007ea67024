"""bench.py — trajectories/sec of the batched minimum-snap solve on MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1
launched under torch.distributed.run, one rank per GPU.  Rank 0 prints ONE
JSON line.

Workload (BASELINE.json configs[1]): a batch of 1024 random 10-segment, N=10,
3-D minimum-snap problems per GPU (createRandomVertices seeds 105 + global
index, estimateSegmentTimes(v_max=3, a_max=5)); inputs resident in HBM.  One
step = one batched solve (mtg_linear_solve: R assembly, block-tridiagonal
Cholesky of R_pp, coefficient recovery, computeCost) over the rank's batch;
with N > 1 the ranks also all-gather the per-trajectory costs over RCCL and
select the global argmin (config 4's selection step).  Weak scaling: each rank
owns a contiguous shard of trajectories.

`--workload time` runs config 5 instead (time-allocation optimisation, 50
objective evaluations per trajectory, B=4096); `--workload tube` config 3
(tube QCQP, B=4096).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (AMD spec; 1/2 of the 157.3 TF FP32 vector peak)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=None, help="trajectories per GPU")
    p.add_argument("--segments", type=int, default=10)
    p.add_argument("--workload", choices=["linear", "time", "tube", "time-qcqp", "sample",
                                          "extrema"], default="linear")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="eager launches (no HIP graph)")
    p.add_argument("--soft", action="store_true",
                   help="time workload: soft constraints max|v| <= 3, max|a| <= 5 in the objective")
    return p.parse_args()


def _oracle_problems(N, D, S, seeds, tube=False):
    """Dense vertex form of the bench problems (same generator and seeds as
    the GPU batch).  tube=True: the tube pattern (positions at every vertex,
    start/end derivatives fixed to the vertex values, qcqp_impl:48-65)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    K = N // 2
    B = len(seeds)
    masks = np.zeros((B, S + 1, K), np.uint8)
    vals = np.zeros((B, S + 1, K, D))
    times = np.zeros((B, S))
    for i, sd in enumerate(seeds):
        v = pyoracle.random_vertices(N // 2 - 1, S, D, -10.0, 10.0, int(sd), K=K)
        masks[i], vals[i] = v.mask, v.vals
        times[i] = pyoracle.estimate_segment_times(v, 3.0, 5.0)
    if tube:
        masks[:] = 0
        masks[:, :, 0] = 1
        masks[:, 0, :] = 1
        masks[:, S, :] = 1
        pos = vals[:, :, 0, :].copy()
        vals[:] = 0.0
        vals[:, :, 0, :] = pos
    return pyoracle, masks, vals, times


def cpu_baseline(wl, N, D, r, S, seconds, sample_args=None):
    """Oracle (reference-faithful C++ port, 1 thread) on a bounded sample of
    the same workload.  Returns (rate, units, description)."""
    import ctypes
    seeds = range(105, 105 + (256 if wl in ("linear", "sample", "extrema") else
                              16 if wl == "time-qcqp" else 64))
    pyoracle, masks, vals, times = _oracle_problems(N, D, S, seeds,
                                                    tube=wl in ("tube", "time-qcqp"))
    K = N // 2
    B = len(seeds)
    if wl == "linear":
        L = pyoracle.lib()
        dp = ctypes.POINTER(ctypes.c_double)
        L.orc_bench_linear.argtypes = [ctypes.c_int] * 6 + [
            ctypes.POINTER(ctypes.c_uint8), dp, dp, ctypes.c_int, ctypes.c_double,
            ctypes.POINTER(ctypes.c_int64), dp]
        n, sec = ctypes.c_int64(), ctypes.c_double()
        rc = L.orc_bench_linear(N, D, r, S, K, B,
                                masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                vals.ctypes.data_as(dp), times.ctypes.data_as(dp), 1, seconds,
                                ctypes.byref(n), ctypes.byref(sec))
        if rc != 0:
            raise RuntimeError(f"oracle baseline failed ({rc})")
        units, sec = n.value, sec.value
        what = "solves (setupFromVertices + solveLinear + computeCost)"
    elif wl == "time":
        units, sec = pyoracle.bench_workload(1, N, D, r, S, K, masks, vals, times,
                                             param_i=50, seconds=seconds)
        what = "50-evaluation time optimisations (orc_time_optimize)"
    elif wl == "tube":
        radii = np.full((B, S, 2), 0.15)
        units, sec = pyoracle.bench_workload(2, N, D, r, S, K, masks, vals, times, radii=radii,
                                             seconds=seconds)
        what = "tube QCQP solves (oracle primal-dual IPM, tol 1e-10)"
    elif wl == "time-qcqp":
        radii = np.full((B, S, 2), 0.15)
        units, sec = pyoracle.bench_workload(5, N, D, r, S, K, masks, vals, times, radii=radii,
                                             seconds=seconds)
        what = ("time-objective evaluations with the QCQP inner solve and the central-"
                "difference gradient (2S+1 oracle IPM solves each)")
    elif wl == "extrema":
        units, sec = pyoracle.bench_workload(4, N, D, r, S, K, masks, vals, times,
                                             seconds=seconds)
        what = ("soft-constraint evaluations (two computeMaximumOfMagnitude searches, "
                "companion-matrix roots)")
    else:
        dt, kmax = sample_args
        units, sec = pyoracle.bench_workload(3, N, D, r, S, K, masks, vals, times, param_i=kmax,
                                             param_d=dt, seconds=seconds)
        what = f"samples (evaluateRange, derivatives 0..{kmax}, dt={dt})"
    desc = (f"{units} {what} cycling over {B} of the same {S}-seg problems "
            f"(seeds 105..{104 + B}), oracle C++ port, 1 thread, ~{seconds:.0f} s")
    return units / sec, units, desc


def load_pmc_traffic(workload, config_key):
    """HBM bytes per launch from the committed rocprofv3 PMC pass, if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            data = json.load(f)
        entry = data.get(workload, {})
        if entry.get("config") == config_key:
            return entry.get("bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import mav_tube_trajectory_generation_amd as mtg

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    N, D, r, S = 10, 3, 4, args.segments
    wl = args.workload
    B = args.batch or {"linear": 1024, "time": 4096, "tube": 4096, "time-qcqp": 1024,
                       "sample": 1024, "extrema": 1024}[wl]
    from mav_tube_trajectory_generation_amd.shard import select_best, shard_range
    global_batch = B * world
    seed0 = 105 + shard_range(global_batch, world, rank)[0]  # contiguous shard
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=seed0)
    ctx = mtg.Context(local_rank)
    plan = mtg.LinearPlan(ctx, N, D, r, S, mask)
    fixed_d = torch.from_numpy(fixed).to(dev)
    times_d = torch.from_numpy(times).to(dev)
    nf = plan.n_fixed
    stream = torch.cuda.current_stream(dev)

    if wl == "linear":
        out = plan.solve(fixed_d, times_d, free=False)

        def step():
            plan.solve(fixed_d, times_d, free=False, out=out)
            if world > 1:  # RCCL all-gather of costs + global argmin
                return select_best(out["cost"], global_batch)
            return None

        bytes_per_traj = (D * nf + S) * 8 + (S * D * N + 1) * 8 + 4  # + status
        metric = "trajectories/sec (10-seg, N=10, 3D minimum-snap) at 1/2/4/8 MI355X"
        unit = "trajectories/s"
        units_per_step = B
    elif wl == "time":
        max_evals = 50

        soft = [(1, 3.0), (2, 5.0)] if args.soft else None

        def step():
            return plan.time_optimize(fixed_d, times_d, max_evals=max_evals, soft=soft)

        bytes_per_traj = (D * nf + S) * 8 + (S + 2) * 8
        metric = "time-allocation optimisations/sec (4096 traj x 50 evals, 10-seg, N=10, 3D)"
        if args.soft:
            metric += " + soft max|v|<=3, max|a|<=5"
        unit = "trajectories/s"
        units_per_step = B
    elif wl == "sample":
        # Sampling of solved trajectories (evaluateRange for derivatives 0..4,
        # the [t, p, v, a, j, s] rows of printMatlabSampledTrajectory) at
        # dt = 0.01 (nonlinear_impl:2915); coefficients resident in HBM.
        sol = plan.solve(fixed_d, times_d, free=False)
        dt, K = 0.01, 4
        n_max = (int(float(times_d.sum(dim=1).max().item()) / dt) + 2 + 63) // 64 * 64
        smp, stm, cnt = mtg.sample_trajectories(sol["coeffs"], times_d, dt, max_derivative=K,
                                                n_max=n_max)
        torch.cuda.synchronize(dev)
        n_total = int(cnt.sum().item())

        def step():
            return mtg.sample_trajectories(sol["coeffs"], times_d, dt, max_derivative=K,
                                           n_max=n_max)

        # written: every sample's (K+1) D channels + its time; read: coeffs, times
        bytes_per_traj = (n_total / B) * ((K + 1) * D + 1) * 8 + (S * D * N + S) * 8
        metric = "trajectory samples/sec (evaluateRange, dt=0.01, derivatives 0..4, 3D)"
        unit = "samples/s"
        units_per_step = n_total
    elif wl == "extrema":
        # Soft-constraint cost of max |v| <= 3, max |a| <= 5 (v_max, a_max of
        # estimateSegmentTimes) on solved trajectories: two batched
        # computeMaximumOfMagnitude searches + the exp cost
        # (evaluateMaximumMagnitudeAsSoftConstraint, nonlinear_impl:2735-2766).
        sol = plan.solve(fixed_d, times_d, free=False)
        ext_out = mtg.soft_constraint_cost(sol["coeffs"], times_d, [1, 2], [3.0, 5.0])

        def step():
            return mtg.soft_constraint_cost(sol["coeffs"], times_d, [1, 2], [3.0, 5.0],
                                            out=ext_out)

        # per search: read coeffs + times, write one maximum; + cost pass
        bytes_per_traj = 2 * ((S * D * N + S) * 8 + 8) + (2 * 8 + 8)
        metric = "soft-constraint evaluations/sec (max |v|, |a| extremum search, 10-seg, N=10, 3D)"
        unit = "trajectories/s"
        units_per_step = B
    else:  # tube, time-qcqp
        radii = torch.full((B, S, 2), 0.15, dtype=torch.float64, device=dev)
        pos_d = torch.from_numpy(pos).to(dev)
        # Tube fixed values: start derivs 0..M-1 then end derivs, per dim.
        M = N // 2
        tf = np.zeros((B, 3, N))
        tf[:, :, 0] = pos[:, 0, :]
        tf[:, :, M] = pos[:, S, :]
        tfix = torch.from_numpy(tf).to(dev)

        if wl == "tube":
            def step():
                return mtg.tube_solve(ctx, N, r, pos_d, tfix, times_d, times_d, radii)

            bytes_per_traj = ((S + 1) * 3 + 3 * N + 2 * S + 2 * S) * 8 + (S * 3 * N + 1) * 8
            metric = "tube QCQP solves/sec (4096 x 10-seg, N=10, 3D)"
        else:
            # config 5's callback in the fork's form (solveQCQP inside
            # objectiveFunctionTime, nonlinear_impl:892) with the central-
            # difference gradient the optimiser uses: 2S+1 QCQPs per unit.
            def step():
                return mtg.tube_time_cost(ctx, N, r, pos_d, tfix, times_d, times_d, radii,
                                          grad=True)

            # inputs once + cost and gradient out (scratch traffic not counted)
            bytes_per_traj = ((S + 1) * 3 + 3 * N + 2 * S + 2 * S) * 8 + (S + 1) * 8 + 4
            metric = ("time-objective evaluations/sec with the QCQP inner solve + FD gradient "
                      "(1024 x 10-seg, N=10, 3D)")
        unit = "trajectories/s"
        units_per_step = B

    # World 1: the K timed steps are captured into one HIP graph and
    # replayed, so launches are back to back (no host launch gaps) and the
    # per-launch duration is (end - start) / K from two HIP events on the
    # launch stream.  Otherwise (collective per step, or millisecond kernels)
    # eager launches with one event pair per launch.
    # (time-qcqp takes stream-ordered scratch inside the call: eager.)
    use_graph = world == 1 and not args.no_graph and wl != "time-qcqp"
    if use_graph:
        graphs = {}
        for name, n in (("warmup", args.warmup), ("timed", args.steps)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    step()
            graphs[name] = g
        graphs["warmup"].replay()
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    if use_graph:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        graphs["timed"].replay()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        kernel_ms = ev0.elapsed_time(ev1) / args.steps
    else:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
        t0 = time.perf_counter()
        for i in range(args.steps):
            ev[i][0].record(stream)
            step()
            ev[i][1].record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    fp64 = None
    if wl == "linear":
        # SURVEY.md 8(d) dense FLOP count per trajectory (81 032 at S=10);
        # the kernel's banded / time-scaled route does fewer operations.
        nf_, np_ = plan.n_fixed, plan.n_free
        flops = (4 * N ** 3 * S + N ** 2 * S + np_ ** 3 / 3 + 2 * np_ * nf_ * D
                 + 2 * np_ ** 2 * D + 2 * N ** 2 * D * S + D * S * (2 * N ** 2 + 2 * N))
        tf = flops * B / (kernel_ms * 1e-3) / 1e12
        fp64 = {"algorithmic_flops_per_traj": flops, "achieved_tflops": tf,
                "peak_tflops": FP64_PEAK_TFLOPS, "frac": tf / FP64_PEAK_TFLOPS}
    total_units = units_per_step * args.steps * world
    value = total_units / elapsed
    alg_bytes = bytes_per_traj * B
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    config_key = f"{wl}:B{B}:S{S}"
    traffic = load_pmc_traffic(wl, config_key)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            rate, _, desc = cpu_baseline(wl, N, D, r, S, args.cpu_seconds,
                                         sample_args=(0.01, 4) if wl == "sample" else None)
            cpu = {"value": rate, "unit": unit, "cores": 1, "kind": "port", "sample": desc}
        line = {
            "metric": metric,
            "value": value,
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (createRandomVertices seeds 105+i, estimateSegmentTimes v=3 a=5)",
            "config": {"workload": f"{wl}: {B} x {S}-segment N={N} D={D} r={r} per GPU",
                       "batch_per_gpu": B, "segments": S, "N": N, "D": D,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel_ms": kernel_ms, "alg_bytes_per_launch": alg_bytes,
                         "kernel_timing": ("HIP events around one graph replay of the K "
                                           "launches, / K" if use_graph else
                                           "HIP event pair per launch, mean"),
                         "fp64_vector": fp64},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
