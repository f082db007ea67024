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
                                          "extrema", "collision"], default="linear")
    p.add_argument("--cpu-seconds", type=float, default=20.0,
                   help="total CPU-baseline budget (all reps, both modes)")
    p.add_argument("--cpu-reps", type=int, default=5)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="eager launches (no HIP graph)")
    p.add_argument("--select", action="store_true",
                   help="linear: include the device selection step (RCCL all-gather + argmin, "
                        "always on at --gpus > 1) also on one GPU")
    p.add_argument("--kernel", default="auto",
                   choices=["auto", "generic", "standard", "lane", "lane_pair"],
                   help="linear-solve kernel (mtg_plan_set_kernel); auto picks by batch size")
    p.add_argument("--optimizer", choices=["fd", "sbplx"], default="fd",
                   help="time workload: the device optimiser (fd: projected central-difference "
                        "descent; sbplx: LN_SBPLX, the reference's default algorithm)")
    p.add_argument("--soft", action="store_true",
                   help="time workload: soft constraints max|v| <= 3, max|a| <= 5 in the objective")
    p.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--graph-head", type=int, default=0,
                   help="steps in the first captured graph of the timed region (0: no head)")
    p.add_argument("--graph-chunk", type=int, default=0,
                   help="steps per captured graph after the head (0: all in one graph)")
    p.add_argument("--sync", choices=["spin", "auto"], default=None,
                   help="host wait mode of the HIP runtime (hipSetDeviceFlags): spin polls for "
                        "completion (the default, MTG_BENCH_SYNC overrides it), auto is the "
                        "runtime's own default")
    p.add_argument("--events", choices=["device", "system"],
                   default=os.environ.get("MTG_BENCH_EVENTS", "system"),
                   help="release scope of the two timing events around the timed replay: "
                        "device (hipEventDisableSystemFence, HIP's flag for events used only "
                        "to time) or system (hipEventRecord's default, with a system-scope "
                        "cache writeback and invalidation at each event)")
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


def _cpu_threads():
    """All-core mode: the CPUs this process may run on, capped by
    OMP_NUM_THREADS when set (the GPU box's CPU share is 16)."""
    n = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _median_rate(run, reps, seconds):
    """run(seconds) -> (units, wall seconds); one short warm-up, then the
    median over `reps` repetitions of the rate."""
    run(min(0.3, seconds))
    rates = sorted(u / s for u, s in (run(seconds) for _ in range(reps)))
    return rates[len(rates) // 2], rates


def cpu_baseline_collision(N, r, coll, seconds, reps):
    """Oracle port of the device optimiser (orc_coll_optimize: the same
    projected L-BFGS on objectiveFunctionFreeConstraintsAndCollision) over 8
    of the bench's starts, 1 thread and all cores (orc_bench_coll)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    mask, df = coll["mask"], coll["df"]
    S = mask.shape[0] - 1
    K = mask.shape[1]
    D = df.shape[0]
    vals = np.zeros((S + 1, K, D))
    vals[0, :, :] = df[:, :K].T
    vals[S, :, :] = df[:, K:].T
    v = pyoracle.Vertices(mask, vals)
    X0 = coll["X0"][:8]

    def run(threads, sec):
        return pyoracle.bench_coll(N, r, v, coll["times"], coll["occ"], coll["params"], X0,
                                   coll["max_evals"], threads=threads, seconds=sec)
    threads = _cpu_threads()
    per_rep = seconds / (2 * reps)
    one, one_all = _median_rate(lambda s_: run(1, s_), reps, per_rep)
    allc, allc_all = _median_rate(lambda s_: run(threads, s_), reps, per_rep)
    return {
        "value": allc, "cores": threads, "kind": "port",
        "single_core": {"value": one, "cores": 1, "reps": [round(x, 3) for x in one_all]},
        "all_core_reps": [round(x, 3) for x in allc_all],
        "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
        "method": (f"median of {reps} repetitions of ~{per_rep:.1f} s after a warm-up, "
                   "std::chrono::steady_clock"),
        "sample": (f"{coll['max_evals']}-evaluation collision optimisations (orc_coll_optimize) "
                   f"cycling over 8 of the bench's starts of main.cpp's problem, oracle C++ port "
                   f"(-O3 -march=x86-64-v3); value = all {threads} threads"),
    }


def cpu_baseline(wl, N, D, r, S, seconds, reps, sample_args=None, optimizer="fd"):
    """Oracle (reference-faithful C++ port, oracle/mtg_oracle.cpp, built
    -O3 -march=x86-64-v3) on a bounded sample of the same workload, on the GPU
    host: 1 thread and all cores (std::thread pool over independent
    trajectories), median of `reps` repetitions after a warm-up
    (the harness shape of polynomial_timing_evaluation.cpp:
    93-127).  The reference's unconditional stdout prints (linear_impl:
    287-292, 370) are not part of the port, so they are excluded.  For the
    linear workload also C1 (one 3-segment problem, 1 thread)."""
    import ctypes
    seeds = range(105, 105 + (256 if wl in ("linear", "sample", "extrema") else
                              16 if wl == "time-qcqp" else 64))
    pyoracle, masks, vals, times = _oracle_problems(N, D, S, seeds,
                                                    tube=wl in ("tube", "time-qcqp"))
    K = N // 2
    B = len(seeds)
    dp = ctypes.POINTER(ctypes.c_double)

    def linear_runner(m, v, t, nb, s_):
        L = pyoracle.lib()
        L.orc_bench_linear.argtypes = [ctypes.c_int] * 6 + [
            ctypes.POINTER(ctypes.c_uint8), dp, dp, ctypes.c_int, ctypes.c_double,
            ctypes.POINTER(ctypes.c_int64), dp]

        def run(threads, sec):
            n, el = ctypes.c_int64(), ctypes.c_double()
            rc = L.orc_bench_linear(N, D, r, s_, K, nb,
                                    m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                    v.ctypes.data_as(dp), t.ctypes.data_as(dp), threads, sec,
                                    ctypes.byref(n), ctypes.byref(el))
            if rc != 0:
                raise RuntimeError(f"oracle baseline failed ({rc})")
            return n.value, el.value
        return run

    radii = np.full((B, S, 2), 0.15)
    if wl == "linear":
        run = linear_runner(masks, vals, times, B, S)
        what = "solves (setupFromVertices + solveLinear + computeCost)"
    else:
        kind, pi, pd, rad, what = {
            "time": ((6, 50, 0.0, None, "50-evaluation LN_SBPLX time optimisations "
                      "(orc_time_optimize_sbplx)") if optimizer == "sbplx" else
                     (1, 50, 0.0, None, "50-evaluation time optimisations (orc_time_optimize)")),
            "tube": (2, 0, 0.0, radii, "tube QCQP solves (oracle primal-dual IPM, tol 1e-10)"),
            "time-qcqp": ((7, 50, 0.0, radii, "50-evaluation LN_SBPLX time optimisations "
                           "with the QCQP inner solve (orc_tube_time_optimize_sbplx)")
                          if optimizer == "sbplx" else
                          (5, 0, 0.0, radii,
                           "time-objective evaluations with the QCQP inner solve and the "
                           "central-difference gradient (2S+1 oracle IPM solves each)")),
            "extrema": (4, 0, 0.0, None, "soft-constraint evaluations (two "
                        "computeMaximumOfMagnitude searches, companion-matrix roots)"),
        }.get(wl, (3, None, None, None, None))
        if kind == 3:
            dt, kmax = sample_args
            pi, pd = kmax, dt
            what = f"samples (evaluateRange, derivatives 0..{kmax}, dt={dt})"

        def run(threads, sec):
            return pyoracle.bench_workload(kind, N, D, r, S, K, masks, vals, times, radii=rad,
                                           param_i=pi, param_d=pd, threads=threads,
                                           seconds=sec)
    threads = _cpu_threads()
    per_rep = seconds / (2 * reps + (1 if wl == "linear" else 0))
    one, one_all = _median_rate(lambda s_: run(1, s_), reps, per_rep)
    allc, allc_all = _median_rate(lambda s_: run(threads, s_), reps, per_rep)
    out = {
        "value": allc, "cores": threads, "kind": "port",
        "single_core": {"value": one, "cores": 1, "reps": [round(x, 3) for x in one_all]},
        "all_core_reps": [round(x, 3) for x in allc_all],
        "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
        "method": (f"median of {reps} repetitions of ~{per_rep:.1f} s after a warm-up, "
                   "std::chrono::steady_clock; the reference's stdout prints excluded"),
        "sample": (f"{what} cycling over {B} of the same {S}-seg problems (seeds 105..{104 + B}),"
                   f" oracle C++ port (-O3 -march=x86-64-v3); value = all {threads} threads"),
    }
    if wl == "linear":
        # C1: a single 3-segment problem (BASELINE.json configs[0]), 1 thread.
        _, m1, v1, t1 = _oracle_problems(N, D, 3, [105])
        c1, _ = _median_rate(lambda s_: linear_runner(m1, v1, t1, 1, 3)(1, s_), reps,
                             per_rep / reps)
        out["c1_3seg_single"] = {"value": c1, "unit": "trajectories/s", "cores": 1,
                                 "latency_us": 1e6 / c1}
    return out


def device_kernel(wl, plan, B, N, D, r, S):
    """rocprofv3 name (substring) of the launch's dominant kernel: the key,
    with the workload / batch / segments, of its committed counter passes."""
    # the library's A/B switches (mtg_linear_std.hip, mtg_time_std.hip,
    # mtg_tube.hip) force the runtime-S kernels
    std_rt = os.environ.get("MTG_STD_RUNTIME_S", "").startswith("1")
    tube_rt = os.environ.get("MTG_TUBE_RUNTIME_S", "").startswith("1")
    wave_ok = (N, r, D) == (10, 4, 3) and 2 <= S <= 16 and not std_rt
    if wl == "linear":
        k = plan.kernel_for_batch(B)
        if k == "standard":
            return "linear_wave_kernel" if wave_ok else "linear_std_kernel"
        return {"lane": "linear_lane_kernel", "lane_pair": "linear_lane2_kernel",
                "generic": "linear_solve_kernel"}[k]
    if wl == "extrema":
        return "soft_cost_kernel" if B < 4096 else "max_magnitude_kernel"
    if wl == "time":
        return "time_optimize_wave_kernel" if wave_ok else "time_optimize_std_kernel"
    if wl in ("tube", "time-qcqp"):
        return ("tube_solve_s_kernel" if N == 10 and 2 <= S <= 16 and not tube_rt else
                "tube_solve_kernel")
    return {"sample": "sample_kernel", "collision": "coll_walk_kernel"}[wl]


# rocprofv3's kernel trace adds a per-dispatch cost of its own: the C2
# kernel (4.6 us unprofiled) averages 5.2-5.7 us in the trace passes and its
# event-timed launches 5.2-7.6 us in the same runs (round 5), so a profiled
# average may exceed this run's time by that much on the same build.
PROFILER_SLACK_MS = 0.0012


class TimingEvents:
    """The two events around the timed replay, recorded on the launch stream
    through the HIP runtime torch loaded.  scope "device" creates them with
    hipEventDisableSystemFence: HIP documents it for events used only to
    time, "avoiding the cost of cache writeback and invalidation" that a
    default event's system-scope fence adds when it is recorded (a fixed
    cost per replay that the K launches would otherwise share).  The host
    still waits for the work with torch.cuda.synchronize, so the wall-clock
    ms_per_step is unaffected.  scope "system": torch's default events."""

    def __init__(self, scope):
        import ctypes
        import torch
        self.scope = scope
        if scope == "system":
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            return
        path = None
        with open("/proc/self/maps") as f:  # the runtime torch has mapped
            for line in f:
                if "libamdhip64.so" in line:
                    path = line.split()[-1]
                    break
        self.hip = hip = ctypes.CDLL(path or "libamdhip64.so")
        hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                            ctypes.c_void_p]
        hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = (ctypes.c_void_p(), ctypes.c_void_p())
        for e in self.ev:
            rc = hip.hipEventCreateWithFlags(ctypes.byref(e), 0x20000000)  # DisableSystemFence
            if rc != 0:
                raise RuntimeError(f"hipEventCreateWithFlags failed ({rc})")

    def record(self, i, stream):
        if self.scope == "system":
            self.ev[i].record(stream)
            return
        rc = self.hip.hipEventRecord(self.ev[i], ctypes_stream(stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed ({rc})")

    def elapsed_ms(self):
        if self.scope == "system":
            return self.ev[0].elapsed_time(self.ev[1])
        import ctypes
        ms = ctypes.c_float()
        rc = self.hip.hipEventSynchronize(self.ev[1])
        rc = rc or self.hip.hipEventElapsedTime(ctypes.byref(ms), self.ev[0], self.ev[1])
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed ({rc})")
        for e in self.ev:
            self.hip.hipEventDestroy(e)
        return float(ms.value)


def ctypes_stream(stream):
    import ctypes
    return ctypes.c_void_p(stream.cuda_stream)


def same_build_time(profiled_ms, kernel_ms):
    """A profiled kernel time (avg_ns of a committed rocprofv3 pass) that can
    come from this build: within 15 % of this run's kernel time, plus the
    profiler's per-dispatch cost above it."""
    return 0.85 * kernel_ms <= profiled_ms <= 1.15 * kernel_ms + PROFILER_SLACK_MS


def load_pmc_traffic(key, kernel_ms):
    """HBM bytes per launch of this workload's kernel from the committed
    rocprofv3 PMC passes (profiles/pmc_traffic.json, keyed
    workload:batch:segments:kernel), or None.  An entry whose kernel time
    differs from this run's by more than 15 % (plus, above, the profiler's own
    per-dispatch cost, PROFILER_SLACK_MS) was measured on another build and
    is not used."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(key)
        if entry and entry.get("avg_ns"):
            if same_build_time(entry["avg_ns"] * 1e-6, kernel_ms):
                return entry.get("bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def load_sq_executed(config_key, kernel_ms):
    """Executed FP64 FLOP per trajectory (SQ instruction counts x active
    lanes, tools/sq_summary.py) from the committed profiles/sq_executed.json,
    for the workload/batch/kernel key, if measured on this build: like the
    traffic entries, only when the pass's kernel time (avg_ns, from the same
    build's kernel-trace pass) is within 15 % of this run's."""
    path = os.path.join(REPO, "profiles", "sq_executed.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(config_key)
        if entry and entry.get("avg_ns"):
            if same_build_time(entry["avg_ns"] * 1e-6, kernel_ms):
                return entry["executed_f64_flop_per_trajectory"], entry["source"]
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def tube_flops_per_iter(N, S):
    """FLOP per interior-point iteration of one tube QCQP:
    m (2 v^2 + 2 v) constraint evaluation + m v^2 Hessian accumulation +
    (S-1) (b^3/3 + b^3 + 2 b^3) block-tridiagonal KKT factorisation, with
    m = (S-1) + 3 S (N-2) constraints, v = 3 N variables per constraint
    stencil, b = 3 N/2 per block (0.79 MFLOP at S = 10, N = 10)."""
    m = (S - 1) + 3 * S * (N - 2)
    v = 3 * N
    b = 3 * (N // 2)
    return m * (2 * v * v + 2 * v) + m * v * v + (S - 1) * (b ** 3 / 3 + b ** 3 + 2 * b ** 3)


def linear_flops_alg(N, D, S, r):
    """FP64 operations of the algorithm the linear kernels run, per solve
    ("FLOP counts"): 11 036 at S = 10, N = 10, D = 3, r = 4.
    Symbols as SURVEY.md 8(d); M = N/2, MF = M - 1 free derivatives per
    intermediate vertex (the standard pattern), TRI = MF (MF + 1) / 2.
      powers     S (2N + M - 4): T^e chains + one reciprocal per segment
      assembly   (S-1) (3 TRI + MF^2 + 5 MF + 5 D MF): A_v = H11(v-1) + H00(v)
                 (two table x power products per entry), C_v = H01(v), the
                 row coefficients and b_v (time-scaled H, no 4N^3 S GEMMs)
                 + 2 (MF^2 + 2 D MF^2): the fixed end vertices' share of b
      LDL^T      (S-2) [MF^3/3 + 2 MF^2 (MF + D) + 2 MF TRI + 2 MF^2 D]:
                 factor, solve for the coupling and right-hand-side columns,
                 symmetric Schur and right-hand-side updates, per block step;
                 + the middle block MF^3/3 + 2 MF^2 D + TRI + D MF
                 + (S-2) 2 MF^2 D back substitution
      recovery   S D (N-2 + M + 2 nnz - M + N-1): f = e T^(j mod M), h =
                 A(1)^-1 f over its nnz = M N structural non-zeros of the
                 lower half, c = T^-i h
      cost       S D ((N-r)(N-r+1) + 2 (N-r) + 2): 0.5 c^T Q c as the
                 quadratic form of h with the constant weights"""
    M = N // 2
    MF = M - 1
    TRI = MF * (MF + 1) // 2
    powers = S * (2 * N + M - 4)
    assembly = (S - 1) * (3 * TRI + MF * MF + 5 * MF + 5 * D * MF) + 2 * (MF * MF + 2 * D * MF * MF)
    ldlt = 0.0
    if S >= 2:
        step = MF ** 3 / 3 + 2 * MF * MF * (MF + D) + 2 * MF * TRI + 2 * MF * MF * D
        ldlt = ((S - 2) * (step + 2 * MF * MF * D)
                + MF ** 3 / 3 + 2 * MF * MF * D + TRI + D * MF)
    recovery = S * D * ((N - 2) + M + (2 * M * N - M) + (N - 1))
    cost = S * D * ((N - r) * (N - r + 1) + 2 * (N - r) + 2)
    return powers + assembly + ldlt + recovery + cost


def linear_flops(N, D, S, nf, np_):
    """SURVEY.md 8(d) dense algorithmic FLOP count of one linear solve (81 032
    at S = 10): every entry of the dense blocks.  Kept beside the count above
    as roofline.dense_equiv_frac; the kernels' time-scaled, banded route does
    about 7x fewer operations, so this one is not a bound."""
    return (4 * N ** 3 * S + N ** 2 * S + np_ ** 3 / 3 + 2 * np_ * nf * D
            + 2 * np_ ** 2 * D + 2 * N ** 2 * D * S + D * S * (2 * N ** 2 + 2 * N))


def config_name(wl, B, world, S, global_batch=None):
    global_batch = B * world if global_batch is None else global_batch
    if wl == "linear" and S == 10:
        if global_batch == 65536:
            return f"C4: 65536 x 10-segment sharded {world} way(s)"
        if world == 1 and B == 1024:
            return "C2: 1024 x 10-segment linear solve"
    if wl == "tube" and S == 10 and B == 4096 and world == 1:
        return "C3: 4096 x 10-segment tube QCQP"
    if wl == "time" and S == 10 and B == 4096 and world == 1:
        return "C5: 4096 x 50-evaluation time allocation"
    if wl == "time-qcqp" and S == 10 and B == 4096 and world == 1:
        return "C5 (QCQP inner solve): 4096 x 50-evaluation time allocation"
    if wl == "collision":
        return f"demo: {B} x main.cpp's 4-segment collision objective per GPU"
    return f"{wl}: {B} x {S}-segment per GPU"


def graph_chunks(k, head, chunk):
    """Sizes of the graphs the K timed steps are captured into, in replay
    order: `head` steps first (0: none), then graphs of `chunk` steps (0: the
    rest in one graph).  Smaller first graphs let the device start while the
    host still submits the later ones."""
    sizes = []
    if 0 < head < k:
        sizes.append(head)
    rest = k - sum(sizes)
    c = chunk if chunk > 0 else rest
    while rest > 0:
        sizes.append(min(c, rest))
        rest -= sizes[-1]
    return sizes


def launch_ranks(n, argv, port=None):
    """`--gpus N` without a launcher: run N ranks of this script under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a
    child process, before this process touches the GPU, and return its exit
    code.  Rank 0 prints the JSON line on the inherited stdout."""
    import socket
    import subprocess
    if port is None:
        with socket.socket() as sk:  # a free port on the loopback interface
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def launch_check():
    """`--launch-check` (tests): each rank joins a gloo group over the
    launcher's rendezvous, all-reduces its rank and rank 0 prints one JSON line
    {world, rank_sum}; no GPU is touched."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank())])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "rank_sum": t.item()}))
    dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if int(env_world or "1") != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU "
              f"(torch.distributed.run --nproc-per-node {args.gpus}) or pass --gpus "
              f"{env_world}", file=sys.stderr)
        sys.exit(2)
    if args.launch_check:
        launch_check()
        return
    import torch
    import torch.distributed as dist

    # Host wait: spin by default (the host polls for the replay's completion
    # instead of sleeping on an interrupt: 0.05-0.16 us less per C2 step at
    # K = 20).  Fatal only when asked for explicitly.
    sync_explicit = args.sync is not None or "MTG_BENCH_SYNC" in os.environ
    if args.sync is None:
        args.sync = os.environ.get("MTG_BENCH_SYNC", "spin")
    host_sync = args.sync
    if args.sync == "spin":
        # Before the first HIP call of the process: the host polls for
        # completion instead of sleeping on an interrupt.  The flag must go
        # to the runtime torch uses, so it is resolved from torch's own
        # library directory (importing torch does not initialise HIP).
        import ctypes
        import glob
        import torch
        cands = sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib",
                                              "libamdhip64.so*")))
        hip = ctypes.CDLL(cands[0] if cands else "libamdhip64.so")
        rc = hip.hipSetDevice(ctypes.c_int(int(os.environ.get("LOCAL_RANK", "0"))))
        rc = rc or hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
        if rc != 0:
            print(f"bench: setting spin-wait failed (HIP {rc})", file=sys.stderr)
            if sync_explicit:
                sys.exit(2)
            host_sync = f"auto (spin-wait not set: HIP {rc})"

    import mav_tube_trajectory_generation_amd as mtg

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    select = world > 1 or args.select
    # RCCL prints its version banner on stdout at communicator set-up; keep
    # stdout for the one JSON line (the banner goes to stderr).
    import contextlib

    @contextlib.contextmanager
    def stdout_to_stderr():
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            yield
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    if select:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local_rank)
        with stdout_to_stderr():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    N, D, r, S = 10, 3, 4, args.segments
    wl = args.workload
    from mav_tube_trajectory_generation_amd.shard import SelectionPipeline, shard_range
    # --gpus N > 1 without --batch: BASELINE config 4, a 65 536-trajectory
    # global batch in contiguous shards (8 192 per GPU at N = 8): total work
    # fixed as N grows ("strong").  N = 1 stays config 2 (1024), the
    # configuration the metric is quoted on.  --batch B: B per GPU ("weak").
    c4_default = wl == "linear" and world > 1 and args.batch is None and S == 10
    if c4_default:
        global_batch = 65536
        B = shard_range(global_batch, world, rank)[1]
    else:
        B = args.batch or {"linear": 1024, "time": 4096, "tube": 4096,
                           "time-qcqp": 4096 if args.optimizer == "sbplx" else 1024,
                           "sample": 1024, "extrema": 1024, "collision": 4096}[wl]
        global_batch = B * world
    seed0 = 105 + shard_range(global_batch, world, rank)[0]  # contiguous shard
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=seed0)
    ctx = mtg.Context(local_rank)
    plan = mtg.LinearPlan(ctx, N, D, r, S, mask).set_kernel(args.kernel)
    fixed_d = torch.from_numpy(fixed).to(dev)
    times_d = torch.from_numpy(times).to(dev)
    nf = plan.n_fixed
    stream = torch.cuda.current_stream(dev)
    bound = "fp64_vector"
    flops_per_step = None   # algorithmic FP64 work of one step (None: not FP64-bound)
    dense_per_step = None   # SURVEY 8(d)'s dense-equivalent count, where it differs
    flop_note = None
    useful_per_step = None  # units that count towards `value` (converged solves)
    metric_base = "trajectories/sec (10-seg, N=10, 3D minimum-snap) at 1/2/4/8 MI355X"
    coll = None  # collision workload inputs (also the CPU baseline's)
    extra_cfg = {}
    pipe = None  # linear: the selection pipeline (its open bucket closes in end_steps)

    def end_steps():
        if pipe is not None:
            pipe.drain()

    if wl == "linear":
        out = plan.solve(fixed_d, times_d, free=False)
        shard_start = shard_range(global_batch, world, rank)[0]
        # The selection step (shard argmin, RCCL all-gather of the triples,
        # global argmin) is pipelined (shard.SelectionPipeline): step k's
        # launch also reduces step k - 1's costs in one extra workgroup, and
        # the triples of a bucket of steps (here: all K steps of the timed
        # graph) are all-gathered in one collective with every step's winner
        # taken at once.  On one GPU without a process group the all-gather
        # and the global argmin are the identity.
        pipe = SelectionPipeline(plan, fixed_d, times_d,
                                 [out, plan.solve(fixed_d, times_d, free=False)], global_batch,
                                 shard_start, rank, dev, use_dist=select,
                                 bucket=max(args.steps, args.warmup, 1))

        def step_selected():
            return pipe.step()

        def step():
            if select:
                return step_selected()
            plan.solve(fixed_d, times_d, free=False, out=out)
            return None

        bytes_per_traj = (D * nf + S) * 8 + (S * D * N + 1) * 8 + 4  # + status
        metric = metric_base
        unit = "trajectories/s"
        units_per_step = B
        flops_per_step = linear_flops_alg(N, D, S, r) * B
        dense_per_step = linear_flops(N, D, S, nf, plan.n_free) * B
        flop_note = (f"the kernels' algorithm, {linear_flops_alg(N, D, S, r):.0f} FLOP per solve "
                     "(bench.linear_flops_alg, DESIGN 6) x B")
    elif wl == "time":
        max_evals = 50

        soft = [(1, 3.0), (2, 5.0)] if args.soft else None

        def step():
            return plan.time_optimize(fixed_d, times_d, max_evals=max_evals, soft=soft,
                                      optimizer=args.optimizer)

        probe = step()
        torch.cuda.synchronize(dev)
        solves = int(probe["solves"].sum().item())
        evals_mean = float(probe["evals"].float().mean().item())
        bytes_per_traj = (D * nf + S) * 8 + (S + 2) * 8
        metric = "time-allocation optimisations/sec (4096 traj x 50 evals, 10-seg, N=10, 3D)"
        if args.optimizer == "sbplx":
            metric += ", LN_SBPLX"
            res_np = probe["result"].cpu().numpy()
            extra_cfg = {"optimizer": "LN_SBPLX (device restatement)",
                         "results": {int(k): int(v) for k, v in
                                     zip(*np.unique(res_np, return_counts=True))}}
        if args.soft:
            metric += " + soft max|v|<=3, max|a|<=5"
            bound = "fp64_vector (soft: extremum search not counted)"
        unit = "trajectories/s"
        units_per_step = B
        flops_per_step = linear_flops_alg(N, D, S, r) * solves
        dense_per_step = linear_flops(N, D, S, nf, plan.n_free) * solves
        flop_note = (f"the solve's algorithm count x {solves} inner solves per launch (measured, gradient "
                     f"points included; {solves / B:.1f} per trajectory, {evals_mean:.1f} "
                     "counted evaluations)")
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
        bound = "hbm"
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
        bound = "hbm"
    elif wl == "collision":
        # The reference demo's objective (main.cpp:77, 104-105:
        # kOptimizeFreeConstraintsAndCollision with LD_LBFGS, max_iterations
        # 25, main.cpp's weights): mtg_coll_optimize's projected L-BFGS on B
        # starts around the demo's tube-QCQP solution (main.cpp:69-73, solved
        # here on the device), over a synthetic forest map standing in for the
        # demo's private supereight map (mav_tube_trajectory_generation_amd/
        # demo.py).  One unit = one 25-evaluation optimisation.
        from mav_tube_trajectory_generation_amd import demo
        pos_m = demo.MAIN_POSITIONS
        Sd = pos_m.shape[0] - 1
        t_m = demo.estimate_segment_times(pos_m, 2.0, 2.0)  # main.cpp:51-53
        cmask, cdf = demo.tube_pattern(pos_m)
        cplan = mtg.LinearPlan(ctx, N, D, r, Sd, cmask)
        T1 = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        tf1 = np.zeros((1, 3, N))
        tf1[0] = cdf
        q = mtg.tube_solve(ctx, N, r, T1(pos_m[None]), T1(tf1), T1(t_m[None]), T1(t_m[None]),
                           T1(demo.MAIN_RADII[None]))
        x0 = q["x"][0].cpu().numpy()
        X0 = np.array([x0] + demo.perturbed_starts(x0, B - 1, 0.005, seed=23))
        occ_np = demo.forest_map()
        cparams = demo.coll_params()
        prm = mtg.make_coll_params(**cparams)
        c_df, c_x0, c_t = T1(np.repeat(cdf[None], B, 0)), T1(X0), T1(np.repeat(t_m[None], B, 0))
        c_occ = T1(occ_np)
        c_max_evals = int(demo.MAIN_PARAMS["max_iterations"])
        c_ws = torch.empty(cplan.coll_workspace_bytes(B, prm, 0, True), dtype=torch.uint8,
                           device=dev)
        # the map's near field (mtg_coll_field), once per map, outside the
        # timed steps: the walk then reads one voxel record per sample
        c_field = mtg.coll_field(c_occ, prm)
        coll = {"mask": cmask, "df": cdf, "times": t_m, "occ": occ_np, "params": cparams,
                "X0": X0, "max_evals": c_max_evals}

        def step():
            return cplan.coll_optimize(c_df, c_x0, c_t, c_occ, prm, max_evals=c_max_evals,
                                       workspace=c_ws, near_field=c_field)

        probe = step()
        torch.cuda.synchronize(dev)
        ev = probe["evals"].cpu().numpy()
        res_hist = {int(k): int(v) for k, v in zip(*np.unique(probe["result"].cpu().numpy(),
                                                               return_counts=True))}
        nvar = X0.shape[1]
        # inputs (x0, d_f, times) + outputs (x, cost, evals, result, status,
        # terms); the map (1.3 MB, L2-resident) read per launch
        bytes_per_traj = (nvar + D * 2 * (N // 2) + Sd) * 8 + (nvar + 1 + 4) * 8 + 12
        bytes_per_traj += occ_np.nbytes / B
        metric = ("collision optimisations/sec (main.cpp's kOptimizeFreeConstraintsAndCollision "
                  "objective, 25 evaluations, 4-seg, N=10, 3D, synthetic forest map)")
        unit = "optimisations/s"
        units_per_step = B
        bound = "hbm"
        extra_cfg = {"segments": Sd, "max_evals": c_max_evals, "mean_evals": float(ev.mean()),
                     "results": res_hist, "map_voxels": list(occ_np.shape)}
    else:  # tube, time-qcqp
        radii = torch.full((B, S, 2), 0.15, dtype=torch.float64, device=dev)
        pos_d = torch.from_numpy(pos).to(dev)
        # Tube fixed values: start derivs 0..M-1 then end derivs, per dim.
        M = N // 2
        tf = np.zeros((B, 3, N))
        tf[:, :, 0] = pos[:, 0, :]
        tf[:, :, M] = pos[:, S, :]
        tfix = torch.from_numpy(tf).to(dev)
        # The same inputs every step, so the per-step status and iteration
        # counts are those of this probe (read once, outside the timed loop).
        probe = mtg.tube_solve(ctx, N, r, pos_d, tfix, times_d, times_d, radii)
        torch.cuda.synchronize(dev)
        conv = int((probe["status"] == 0).sum().item())
        iters = int(probe["iters"].sum().item())
        hist = {int(k): int(v) for k, v in zip(*np.unique(probe["status"].cpu().numpy(),
                                                           return_counts=True))}
        f_iter = tube_flops_per_iter(N, S)

        if wl == "tube":
            def step():
                return mtg.tube_solve(ctx, N, r, pos_d, tfix, times_d, times_d, radii)

            # inputs (positions, fixed values, two time vectors, radii) + outputs
            # (x: 3 (S-1) N/2 free control-point values, coefficients, cost,
            # iteration count, status)
            bytes_per_traj = (((S + 1) * 3 + 3 * N + 2 * S + 2 * S) * 8
                              + (3 * (S - 1) * (N // 2) + S * 3 * N + 1) * 8 + 4 + 4)
            metric = "converged tube QCQP solves/sec (4096 x 10-seg, N=10, 3D)"
            useful_per_step = conv
            flops_per_step = f_iter * iters
            flop_note = (f"SURVEY 8(d) C3: {f_iter:.0f} FLOP/iteration x {iters} IPM iterations "
                         f"per launch (measured, {iters / B:.1f} per problem); status "
                         f"histogram {hist}")
        elif args.optimizer == "sbplx":
            # Config 5 in the reference's own kOptimizeTime path: LN_SBPLX
            # (the default algorithm) over objectiveFunctionTime with
            # solveQCQP() at every evaluation (nonlinear_impl:332-397,
            # 877-945), 50 evaluations per trajectory.  One step = the whole
            # optimisation: 50 rounds of one batched tube launch each plus the
            # machine step (mtg_tube_time_optimize_ex, optimizer 1).
            from mav_tube_trajectory_generation_amd._abi import make_time_params
            E = 50
            tparams = make_time_params(500.0, 0.1, 0.1, 1.0, 2, None, 100.0, optimizer="sbplx")
            ws = torch.empty(mtg.tube_time_workspace_bytes(N, S, B, tparams, True),
                             dtype=torch.uint8, device=dev)

            def step():
                return mtg.tube_time_optimize(ctx, N, r, pos_d, tfix, radii, times_d,
                                              max_evals=E, optimizer="sbplx", workspace=ws)

            res = step()
            torch.cuda.synchronize(dev)
            ev = res["evals"].cpu().numpy()
            rh = {int(k): int(v) for k, v in zip(*np.unique(res["result"].cpu().numpy(),
                                                             return_counts=True))}
            # inputs once + times, cost, evals, result, status out
            bytes_per_traj = (((S + 1) * 3 + 3 * N + 2 * S + S) * 8 + (S + 1) * 8 + 3 * 4)
            metric = ("LN_SBPLX time optimisations/sec with the QCQP inner solve "
                      f"({B} x 10-seg, N=10, 3D, {E} evaluations)")
            flops_per_step = f_iter * (iters / B) * float(ev.sum())
            flop_note = (f"approximate: {f_iter:.0f} FLOP/iteration x {iters / B:.1f} IPM "
                         f"iterations per solve (the T0 probe) x {int(ev.sum())} evaluations "
                         "per step (one QCQP each); kernel_ms is the whole step (50 tube "
                         "launches + the machine steps)")
            extra_cfg = {"optimizer": "sbplx", "max_evals": E, "mean_evals": float(ev.mean()),
                         "results": rh}
        else:
            # config 5's callback in the fork's form (solveQCQP inside
            # objectiveFunctionTime, nonlinear_impl:892) with the central-
            # difference gradient the optimiser uses: 2S+1 QCQPs per unit.
            from mav_tube_trajectory_generation_amd._abi import make_time_params
            tparams = make_time_params(500.0, 0.1, 0.1, 1.0, 2, None, 100.0)
            ws = torch.empty(mtg.tube_time_workspace_bytes(N, S, B, tparams, False),
                             dtype=torch.uint8, device=dev)

            def step():
                return mtg.tube_time_cost(ctx, N, r, pos_d, tfix, times_d, times_d, radii,
                                          grad=True, workspace=ws)

            # inputs once + cost and gradient out (scratch traffic not counted)
            bytes_per_traj = ((S + 1) * 3 + 3 * N + 2 * S + 2 * S) * 8 + (S + 1) * 8 + 4
            metric = ("time-objective evaluations/sec with the QCQP inner solve + FD gradient "
                      "(1024 x 10-seg, N=10, 3D)")
            flops_per_step = f_iter * iters * (2 * S + 1)
            flop_note = (f"approximate: {f_iter:.0f} FLOP/iteration x the IPM iterations of the "
                         f"base solves ({iters / B:.1f} per problem) x (2S+1) problems")
        unit = "trajectories/s"
        units_per_step = B

    # The K timed steps are captured into one HIP graph and replayed, so
    # launches are back to back (no host launch gaps) and the per-step device
    # time is (end - start) / K from two HIP events on the launch stream.
    # World > 1 (linear): the step, RCCL all-gather included, is captured the
    # same way after eager warm-up steps (the communicator is initialised
    # outside the capture).  A failed capture is fatal (exit 3) on every
    # rank: the line never carries eager timings unless --no-graph asks for
    # them.
    use_graph = not args.no_graph
    graphs = {}
    if select:  # communicator set up and first collectives outside any capture
        with stdout_to_stderr():
            for _ in range(max(args.warmup, 2)):
                step()
            end_steps()
            torch.cuda.synchronize(dev)
            dist.barrier()
    if use_graph:
        capture_error = None
        try:  # capture only: nothing executes (no collective runs) here
            for name, sizes in (("warmup", [args.warmup]),
                                ("timed", graph_chunks(args.steps, args.graph_head,
                                                       args.graph_chunk))):
                gl = []
                for n in sizes:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for _ in range(n):
                            step()
                        end_steps()
                    gl.append(g)
                graphs[name] = gl
        except Exception as exc:
            capture_error = f"{type(exc).__name__}: {exc}"
        if world > 1:
            # Every rank takes the same path (a replayed all-gather on one
            # rank would wait for a collective that never comes).
            ok = torch.tensor([0.0 if capture_error else 1.0], dtype=torch.float64, device=dev)
            try:
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if ok.item() < 0.5 and capture_error is None:
                    capture_error = "graph capture failed on another rank"
            except Exception as exc:
                capture_error = capture_error or f"capture agreement failed: {exc}"
        if capture_error is not None:
            print(f"bench: graph capture failed ({capture_error}); not publishing eager "
                  "timings (pass --no-graph to time eager launches)", file=sys.stderr)
            sys.exit(3)
        for g in graphs["warmup"]:
            g.replay()
    else:
        for _ in range(args.warmup):
            step()
        end_steps()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    if use_graph:
        tev = TimingEvents(args.events)
        t0 = time.perf_counter()
        tev.record(0, stream)
        for g in graphs["timed"]:
            g.replay()
        tev.record(1, stream)
        torch.cuda.synchronize(dev)
        if world > 1:  # one rank: the synchronize above already closes the region
            dist.barrier()
            torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        kernel_ms = tev.elapsed_ms() / args.steps
    else:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
        t0 = time.perf_counter()
        for i in range(args.steps):
            ev[i][0].record(stream)
            step()
            ev[i][1].record(stream)
        end_steps()
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

    # One GPU: also time the selection-inclusive step (the step every rank runs
    # at --gpus > 1, minus the all-gather), so the scaling curve's N = 1 and
    # N > 1 points can be compared step for step.
    selection_ms = None
    if wl == "linear" and not select:
        for _ in range(3):
            step_selected()
        end_steps()
        torch.cuda.synchronize(dev)
        sev = TimingEvents(args.events)
        if use_graph:
            try:
                gs = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gs):
                    for _ in range(args.steps):
                        step_selected()
                    end_steps()
            except Exception as exc:
                print(f"bench: graph capture of the selection step failed ({exc})",
                      file=sys.stderr)
                sys.exit(3)
            gs.replay()  # warm replay, then the timed one
            torch.cuda.synchronize(dev)
            sev.record(0, stream)
            gs.replay()
            sev.record(1, stream)
        else:
            sev.record(0, stream)
            for _ in range(args.steps):
                step_selected()
            end_steps()
            sev.record(1, stream)
        torch.cuda.synchronize(dev)
        selection_ms = sev.elapsed_ms() / args.steps

    if useful_per_step is not None:
        total_units = useful_per_step * args.steps * world
    else:  # every rank's shard (shards differ by one when world does not divide)
        total_units = units_per_step * global_batch // B * args.steps
    value = total_units / elapsed
    alg_bytes = bytes_per_traj * B
    gbs = alg_bytes / (kernel_ms * 1e-3) / 1e9
    config_key = (f"{wl}:B{B}:S{S}" + (":soft" if getattr(args, "soft", False) else "")
                  + (":sbplx" if wl in ("time", "time-qcqp") and args.optimizer == "sbplx"
                     else ""))
    dev_kernel = device_kernel(wl, plan, B, N, D, r, S)
    traffic = load_pmc_traffic(f"{config_key}:{dev_kernel}", kernel_ms)
    timing = (f"HIP events ({args.events}-scope release) around one graph replay of the K "
              "steps, / K" if use_graph else
              "HIP event pair per step, mean (--no-graph)")
    hbm = {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
           "alg_bytes_per_launch": alg_bytes, "traffic": traffic}
    if flops_per_step is not None:
        tfl = flops_per_step / (kernel_ms * 1e-3) / 1e12
        roof = {"bound": bound, "achieved": tfl, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tfl / FP64_PEAK_TFLOPS, "traffic": traffic,
                "alg_flops_per_launch": flops_per_step, "flop_count": flop_note,
                "hbm": hbm}
        if dense_per_step is not None:
            # SURVEY 8(d)'s dense count over the same time (not a bound: the
            # kernels skip the structural zeros and the H-block GEMMs)
            roof["dense_equiv_frac"] = (dense_per_step / (kernel_ms * 1e-3) / 1e12
                                        / FP64_PEAK_TFLOPS)
            roof["dense_flops_per_launch"] = dense_per_step
    else:
        roof = {"bound": "hbm", **{k: hbm[k] for k in ("achieved", "peak", "unit", "frac")},
                "traffic": traffic, "alg_bytes_per_launch": alg_bytes}
    roof["kernel_ms"] = kernel_ms
    roof["kernel"] = dev_kernel
    roof["kernel_timing"] = timing
    # Executed FP64 work beside the dense-equivalent count: the kernel's SQ
    # FP64 instruction counts x active lanes (a committed rocprofv3 pass at
    # this workload, batch and kernel) over this run's kernel time.
    ex_flop, ex_src = load_sq_executed(f"{config_key}:{dev_kernel}", kernel_ms)
    if ex_flop is not None:
        ex_tf = ex_flop * B / (kernel_ms * 1e-3) / 1e12
        roof["executed"] = {"achieved": ex_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": ex_tf / FP64_PEAK_TFLOPS,
                            "flop_per_trajectory": ex_flop, "source": ex_src}
    if select and wl == "linear":
        roof["kernel_timing"] += ("; per-step device time includes the selection: each "
                                  "launch reduces the previous step's costs in one extra "
                                  "workgroup, and the K steps' triples are all-gathered "
                                  "(RCCL) in one collective with every step's winner taken at "
                                  "once")

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            if wl == "collision":
                cpu = cpu_baseline_collision(N, r, coll, args.cpu_seconds, args.cpu_reps)
            else:
                cpu = cpu_baseline(wl, N, D, r, S, args.cpu_seconds, args.cpu_reps,
                                   sample_args=(0.01, 4) if wl == "sample" else None,
                                   optimizer=args.optimizer)
            cpu["unit"] = unit
        cfg = {"workload": config_name(wl, B, world, S, global_batch),
               "global_batch": global_batch,
               "kernel": plan.kernel_for_batch(B) if wl == "linear" else None,
               "batch_per_gpu": B, "segments": S, "N": N, "D": D, "r": r,
               "parallelism": f"shard{world}",
               "selection": bool(select and wl == "linear"), "host_sync": host_sync}
        if wl == "linear":
            cfg["selection_bucket"] = pipe.bucket
        cfg.update(extra_cfg)
        if useful_per_step is not None:
            cfg["converged_per_step"] = useful_per_step
        if selection_ms is not None:
            # device ms per step of solve + fused shard argmin + global argmin
            cfg["selection_step_ms"] = selection_ms
            cfg["selection_overhead_ms"] = selection_ms - kernel_ms
        line = {
            "metric": metric,
            "value": value,
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if c4_default else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (main.cpp's vertices, starts perturbed around the device tube "
                     "QCQP solution, synthetic forest occupancy map)" if wl == "collision" else
                     "synthetic (createRandomVertices seeds 105+i, estimateSegmentTimes v=3 a=5)"),
            "config": cfg,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if select:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
