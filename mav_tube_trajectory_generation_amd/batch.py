"""Batched Python front end of libmtg_hip.so.

Device buffers are torch CUDA (HIP) tensors: PyTorch supplies HBM
allocations and the current stream only; every computation is a gfx950 kernel
of libmtg_hip.so.  Host-array entry points (numpy) copy through the library's
own host ABI.
"""
import ctypes

import numpy as np

from . import _abi
from ._abi import (MTGError, check, lib, make_coll_params, make_collision_params,  # noqa: F401
                   make_time_params)


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require(t, shape, name):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise MTGError(f"{name} must be a CUDA tensor")
    if t.dtype != torch.float64:
        raise MTGError(f"{name} must be float64 (the path computes in FP64)")
    if tuple(t.shape) != tuple(shape):
        raise MTGError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    if not t.is_contiguous():
        raise MTGError(f"{name} must be contiguous")


class Context:
    """One HIP device (mtg_ctx_create)."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        check(lib().mtg_ctx_create(device, ctypes.byref(self._h)), "mtg_ctx_create")
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().mtg_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LinearPlan:
    """(N, D, r, S, constraint pattern) -> batched solves (mtg_plan_create)."""

    def __init__(self, ctx, N, D, r, S, fixed_mask):
        mask = np.ascontiguousarray(np.asarray(fixed_mask, dtype=np.uint8).reshape(-1))
        if mask.size != (S + 1) * (N // 2):
            raise MTGError(f"fixed_mask must have (S+1)*N/2 = {(S + 1) * (N // 2)} entries")
        self.ctx, self.N, self.D, self.r, self.S = ctx, N, D, r, S
        self.mask = mask.reshape(S + 1, N // 2).copy()
        self._h = ctypes.c_void_p()
        check(lib().mtg_plan_create(ctx.handle, N, D, r, S,
                                    mask.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                    ctypes.byref(self._h)), "mtg_plan_create")
        nf, np_ = ctypes.c_int(), ctypes.c_int()
        check(lib().mtg_plan_counts(self._h, ctypes.byref(nf), ctypes.byref(np_)), "counts")
        self.n_fixed, self.n_free = nf.value, np_.value

    KERNELS = {"auto": 0, "generic": 1, "standard": 2, "lane": 3, "lane_pair": 4}
    _NAMES = {v: k for k, v in KERNELS.items()}

    def set_kernel(self, which):
        """Select the linear-solve kernel: "auto" (default), "generic",
        "standard" (one wavefront per trajectory) or "lane" (one
        (trajectory, dimension) per lane); MTGError where the pattern or
        sizes do not allow it."""
        check(lib().mtg_plan_set_kernel(self._h, self.KERNELS[which]), "mtg_plan_set_kernel")
        return self

    @property
    def kernel(self):
        """The forced kernel, or for "auto" the wavefront kernel ("generic" or
        "standard"); see kernel_for_batch."""
        k = lib().mtg_plan_kernel(self._h)
        check(min(k, 0), "mtg_plan_kernel")
        return self._NAMES[k]

    def kernel_for_batch(self, B):
        """Kernel a solve of B trajectories runs."""
        k = lib().mtg_plan_kernel_for_batch(self._h, B)
        check(min(k, 0), "mtg_plan_kernel_for_batch")
        return self._NAMES[k]

    def close(self):
        if self._h:
            lib().mtg_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- device (torch) API -------------------------------------------------
    def solve(self, fixed_vals, times, cost=True, free=False, status=True, out=None):
        """Batched solveLinear + computeCost on device tensors.

        fixed_vals [B, D, n_fixed], times [B, S] (float64, CUDA).  Returns a
        dict with coeffs [B, S, D, N] and optionally cost [B], free [B, D,
        n_free], status [B] (int32).
        """
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        dev = times.device
        o = out or {}
        if "coeffs" not in o:
            o["coeffs"] = torch.empty((B, self.S, self.D, self.N), dtype=torch.float64, device=dev)
        if cost and "cost" not in o:
            o["cost"] = torch.empty(B, dtype=torch.float64, device=dev)
        if free and "free" not in o:
            o["free"] = torch.empty((B, self.D, self.n_free), dtype=torch.float64, device=dev)
        if status and "status" not in o:
            o["status"] = torch.empty(B, dtype=torch.int32, device=dev)
        check(lib().mtg_linear_solve(self._h, B, _ptr(fixed_vals), _ptr(times), _ptr(o["coeffs"]),
                                     _ptr(o.get("cost")), _ptr(o.get("free")),
                                     _ptr(o.get("status")), _stream(dev)), "mtg_linear_solve")
        return o

    def select_workspace(self, B, device):
        """Workspace of solve_select for B trajectories (per-workgroup
        partials of the lane kernels; empty for the wavefront kernels)."""
        import torch
        n = lib().mtg_select_workspace_bytes(self._h, B)
        if n < 0:
            check(int(n), "mtg_select_workspace_bytes")
        return torch.empty(int(n), dtype=torch.uint8, device=device)

    def solve_select(self, fixed_vals, times, start, rank, workspace, out=None, free=False,
                     status=True):
        """solve() followed by the shard's selection (mtg_linear_solve_select:
        lane kernels reduce per-workgroup partials written by the solve's
        epilogue): adds "triple" = (cost, start + index, rank), the
        select_local rule, as a float64 device tensor [3].
        workspace from select_workspace(B)."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        dev = times.device
        o = out or {}
        if "coeffs" not in o:
            o["coeffs"] = torch.empty((B, self.S, self.D, self.N), dtype=torch.float64, device=dev)
        if "cost" not in o:
            o["cost"] = torch.empty(B, dtype=torch.float64, device=dev)
        if free and "free" not in o:
            o["free"] = torch.empty((B, self.D, self.n_free), dtype=torch.float64, device=dev)
        if status and "status" not in o:
            o["status"] = torch.empty(B, dtype=torch.int32, device=dev)
        if "triple" not in o:
            o["triple"] = torch.empty(3, dtype=torch.float64, device=dev)
        check(lib().mtg_linear_solve_select(
            self._h, B, _ptr(fixed_vals), _ptr(times), _ptr(o["coeffs"]), _ptr(o["cost"]),
            _ptr(o.get("free")), _ptr(o.get("status")), int(start), int(rank), _ptr(o["triple"]),
            _ptr(workspace), workspace.numel(), _stream(dev)), "mtg_linear_solve_select")
        return o

    def solve_select_prev(self, fixed_vals, times, out, prev_cost=None, prev_start=0, rank=0,
                          prev_triple=None):
        """solve() into the output set `out` (coeffs, cost, status) with the
        previous step's shard selection in the same launch
        (mtg_linear_solve_select_prev): prev_cost [n] (another output set's
        costs) reduced to prev_triple [3] = (cost, prev_start + index, rank).
        prev_cost None: the plain solve."""
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        n = 0 if prev_cost is None else prev_cost.numel()
        check(lib().mtg_linear_solve_select_prev(
            self._h, B, _ptr(fixed_vals), _ptr(times), _ptr(out["coeffs"]), _ptr(out.get("cost")),
            _ptr(out.get("free")), _ptr(out.get("status")), _ptr(prev_cost), n, int(prev_start),
            int(rank), _ptr(prev_triple), _stream(times.device)), "mtg_linear_solve_select_prev")
        return out

    def coefficients(self, fixed_vals, free_vals, times):
        """Coefficients and cost from given d_f and d_p, no solve
        (setFreeConstraints, linear_impl:497-506).  Returns (coeffs, cost,
        status)."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        _require(free_vals, (B, self.D, self.n_free), "free_vals")
        dev = times.device
        coeffs = torch.empty((B, self.S, self.D, self.N), dtype=torch.float64, device=dev)
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        check(lib().mtg_coeffs_from_constraints(self._h, B, _ptr(fixed_vals), _ptr(free_vals),
                                                _ptr(times), _ptr(coeffs), _ptr(cost),
                                                _ptr(status), _stream(dev)),
              "mtg_coeffs_from_constraints")
        return coeffs, cost, status

    def time_cost(self, fixed_vals, times, time_penalty=500.0, grad_mode=0, increment=0.1,
                  w_d=0.1, w_t=1.0, soft=None, soft_weight=100.0, hard=False,
                  hard_tolerance=0.1):
        """objectiveFunctionTime per trajectory (mtg_time_cost); soft: list of
        (derivative, maximum_value) soft magnitude constraints."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        dev = times.device
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        grad = torch.empty((B, self.S), dtype=torch.float64, device=dev) if grad_mode else None
        status = torch.empty(B, dtype=torch.int32, device=dev)
        p = make_time_params(time_penalty, increment, w_d, w_t, grad_mode, soft, soft_weight,
                             hard=hard, hard_tolerance=hard_tolerance)
        check(lib().mtg_time_cost(self._h, B, _ptr(fixed_vals), _ptr(times), ctypes.byref(p),
                                  _ptr(cost), _ptr(grad), _ptr(status), _stream(dev)),
              "mtg_time_cost")
        return dict(cost=cost, grad=grad, status=status)

    def time_optimize(self, fixed_vals, times, max_evals=50, time_penalty=500.0, increment=0.1,
                      w_d=0.1, w_t=1.0, soft=None, soft_weight=100.0, hard=False,
                      hard_tolerance=0.1, optimizer="fd", f_rel=0.05, f_abs=-1.0,
                      initial_stepsize_rel=0.1):
        """Optimise segment times in place on a copy; returns dict(times, cost,
        evals, solves, result, status); solves = inner solves run (gradient
        points included), result = the nlopt_result stopping code
        (mtg_time_optimize_ex).  optimizer "fd" (projected central-difference
        descent) or "sbplx" (LN_SBPLX, the reference's default algorithm,
        with f_rel / f_abs / initial_stepsize_rel as
        NonlinearOptimizationParameters)."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        dev = times.device
        t = times.clone()
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        evals = torch.empty(B, dtype=torch.int32, device=dev)
        solves = torch.empty(B, dtype=torch.int32, device=dev)
        result = torch.empty(B, dtype=torch.int32, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        p = make_time_params(time_penalty, increment, w_d, w_t, 2, soft, soft_weight,
                             hard=hard, hard_tolerance=hard_tolerance, optimizer=optimizer,
                             f_rel=f_rel, f_abs=f_abs, initial_stepsize_rel=initial_stepsize_rel)
        check(lib().mtg_time_optimize_ex(self._h, B, _ptr(fixed_vals), _ptr(t), ctypes.byref(p),
                                         max_evals, _ptr(cost), _ptr(evals), _ptr(solves),
                                         _ptr(result), _ptr(status), _stream(dev)),
              "mtg_time_optimize_ex")
        return dict(times=t, cost=cost, evals=evals, solves=solves, result=result,
                    status=status)

    def free_cost(self, fixed_vals, free_vals, times, mode=0, time_penalty=500.0, soft=None,
                  soft_weight=100.0, grad=True):
        """Free-derivative objectives (mtg_free_cost): mode 0
        objectiveFunctionFreeConstraints (J_d [+ soft], gradient of J_d
        [B, D, n_free]); mode 1 objectiveFunctionTimeAndConstraints."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        _require(free_vals, (B, self.D, self.n_free), "free_vals")
        dev = times.device
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        g = (torch.empty((B, self.D, self.n_free), dtype=torch.float64, device=dev)
             if (grad and mode == 0) else None)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        p = make_time_params(time_penalty, 0.1, 0.1, 1.0, 0, soft, soft_weight)
        check(lib().mtg_free_cost(self._h, B, _ptr(fixed_vals), _ptr(free_vals), _ptr(times),
                                  ctypes.byref(p), mode, _ptr(cost), _ptr(g), _ptr(status),
                                  _stream(dev)), "mtg_free_cost")
        return dict(cost=cost, grad=g, status=status)

    def free_optimize(self, fixed_vals, free_vals, times, max_evals=50, lower=None, upper=None,
                      soft=None, soft_weight=100.0):
        """Optimise the free derivatives (mtg_free_optimize) on a copy of
        free_vals; returns dict(free, cost, evals, status)."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        _require(free_vals, (B, self.D, self.n_free), "free_vals")
        for name, a in (("lower", lower), ("upper", upper)):
            if a is not None:
                _require(a, (B, self.D, self.n_free), name)
        dev = times.device
        d = free_vals.clone()
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        evals = torch.empty(B, dtype=torch.int32, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        p = make_time_params(500.0, 0.1, 0.1, 1.0, 0, soft, soft_weight)
        check(lib().mtg_free_optimize(self._h, B, _ptr(fixed_vals), _ptr(d), _ptr(times),
                                      _ptr(lower), _ptr(upper), ctypes.byref(p), max_evals,
                                      _ptr(cost), _ptr(evals), _ptr(status), _stream(dev)),
              "mtg_free_optimize")
        return dict(free=d, cost=cost, evals=evals, status=status)

    def time_free_optimize(self, fixed_vals, free_vals, times, max_evals=50, time_penalty=500.0,
                           increment=0.1, soft=None, soft_weight=100.0, optimizer="fd",
                           f_rel=0.05, f_abs=-1.0, initial_stepsize_rel=0.1):
        """Optimise segment times and free derivatives together
        (mtg_time_free_optimize_ex, optimizeTimeAndFreeConstraints) on copies;
        optimizer "sbplx" runs LN_SBPLX over [T; d_p] (the reference's
        algorithm), "fd" the block-alternating descent.  Returns dict(times,
        free, cost, evals, result, status)."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        _require(free_vals, (B, self.D, self.n_free), "free_vals")
        dev = times.device
        t = times.clone()
        d = free_vals.clone()
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        evals = torch.empty(B, dtype=torch.int32, device=dev)
        result = torch.full((B,), 0, dtype=torch.int32, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        p = make_time_params(time_penalty, increment, 0.1, 1.0, 0, soft, soft_weight,
                             optimizer=optimizer, f_rel=f_rel, f_abs=f_abs,
                             initial_stepsize_rel=initial_stepsize_rel)
        check(lib().mtg_time_free_optimize_ex(self._h, B, _ptr(fixed_vals), _ptr(d), _ptr(t),
                                              ctypes.byref(p), max_evals, _ptr(cost),
                                              _ptr(evals), _ptr(result), _ptr(status),
                                              _stream(dev)), "mtg_time_free_optimize_ex")
        return dict(times=t, free=d, cost=cost, evals=evals, result=result, status=status)

    def collision_cost(self, coeffs, times, occupancy, params, grad=True):
        """Collision cost over a dense occupancy grid (mtg_collision_cost,
        getCostAndGradientCollision): coeffs [B, S, 3, N], times [B, S],
        occupancy float32 CUDA tensor [nz, ny, nx] (occupied iff >= 0),
        params from make_collision_params.  Returns dict(cost, collision,
        grad_coeffs, grad_free)."""
        import torch
        B = times.shape[0]
        _require(times, (B, self.S), "times")
        _require(coeffs, (B, self.S, self.D, self.N), "coeffs")
        if not (isinstance(occupancy, torch.Tensor) and occupancy.is_cuda and
                occupancy.dtype == torch.float32 and occupancy.dim() == 3 and
                occupancy.is_contiguous()):
            raise MTGError("occupancy must be a contiguous float32 CUDA tensor [nz, ny, nx]")
        nz, ny, nx = occupancy.shape
        dev = times.device
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        coll = torch.empty(B, dtype=torch.int32, device=dev)
        gc = torch.empty((B, self.S, self.D, self.N), dtype=torch.float64, device=dev) \
            if grad else None
        gf = torch.empty((B, self.D, self.n_free), dtype=torch.float64, device=dev) \
            if grad else None
        check(lib().mtg_collision_cost(self._h, B, _ptr(coeffs), _ptr(times), _ptr(occupancy),
                                       nx, ny, nz, ctypes.byref(params), _ptr(cost), _ptr(coll),
                                       _ptr(gc), _ptr(gf), _stream(dev)), "mtg_collision_cost")
        return dict(cost=cost, collision=coll, grad_coeffs=gc, grad_free=gf)

    # -- collision-driven objectives (mtg_coll_cost / mtg_coll_optimize) -----
    def _n_vars(self, mode):
        return (self.S if mode else 0) + self.D * self.n_free

    def coll_workspace_bytes(self, B, params, mode=0, optimize=False):
        n = lib().mtg_coll_workspace_bytes(self._h, B, mode, ctypes.byref(params),
                                           1 if optimize else 0)
        if n < 0:
            check(int(n), "mtg_coll_workspace_bytes")
        return int(n)

    def _coll_inputs(self, fixed_vals, x, times, occupancy, mode):
        import torch
        B = x.shape[0]
        _require(fixed_vals, (B, self.D, self.n_fixed), "fixed_vals")
        _require(x, (B, self._n_vars(mode)), "x")
        if mode == 0:
            _require(times, (B, self.S), "times")
        if not (isinstance(occupancy, torch.Tensor) and occupancy.is_cuda and
                occupancy.dtype == torch.float32 and occupancy.dim() == 3 and
                occupancy.is_contiguous()):
            raise MTGError("occupancy must be a contiguous float32 CUDA tensor [nz, ny, nx]")
        return B

    def coll_cost(self, fixed_vals, x, times, occupancy, params, mode=0, raise_ref=None,
                  grad=True, workspace=None, near_field=None):
        """objectiveFunctionFreeConstraintsAndCollision (mode 0, x = d_p
        [B, D*n_free]) or ...AndCollisionAndTime (mode 1, x = [T; d_p]
        [B, S + D*n_free]) on the device (mtg_coll_cost).  params from
        make_coll_params; raise_ref [B] the collision raise reference (None:
        0); near_field from coll_field(occupancy, params) (None: every
        sample's box is scanned).  Returns dict(cost, grad, terms [B, 4],
        collision, status)."""
        import torch
        B = self._coll_inputs(fixed_vals, x, times, occupancy, mode)
        _check_field(near_field, occupancy)
        dev = x.device
        nz, ny, nx = occupancy.shape
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        g = torch.empty((B, self._n_vars(mode)), dtype=torch.float64, device=dev) if grad else None
        terms = torch.empty((B, 4), dtype=torch.float64, device=dev)
        coll = torch.empty(B, dtype=torch.int32, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        nb = self.coll_workspace_bytes(B, params, mode, False)
        ws = _workspace(workspace, nb, dev)
        check(lib().mtg_coll_cost(self._h, B, mode, _ptr(fixed_vals), _ptr(x),
                                  _ptr(times) if mode == 0 else None, _ptr(occupancy), nx, ny,
                                  nz, _ptr(near_field), ctypes.byref(params), _ptr(raise_ref),
                                  _ptr(cost), _ptr(g),
                                  _ptr(terms), _ptr(coll), _ptr(st), _ptr(ws), nb,
                                  _stream(dev)), "mtg_coll_cost")
        return dict(cost=cost, grad=g, terms=terms, collision=coll, status=st)

    def coll_optimize(self, fixed_vals, x0, times, occupancy, params, mode=0, max_evals=25,
                      lower=None, upper=None, initial_step=None, workspace=None,
                      near_field=None, history=False):
        """Device L-BFGS over the collision objective (mtg_coll_optimize;
        optimizeFreeConstraintsAndCollision / ...AndTime with NLopt
        replaced); near_field as coll_cost.  Returns dict(x, cost, evals,
        result, status, terms); with history=True also x_history
        (B x max_evals x nv, nv = the number of optimisation variables,
        _n_vars(mode): D * n_free in mode 0, S + D * n_free in mode 1; the
        evaluated points in order, rows past evals unset:
        mtg_coll_optimize_trace)."""
        import torch
        B = self._coll_inputs(fixed_vals, x0, times, occupancy, mode)
        _check_field(near_field, occupancy)
        dev = x0.device
        nv = self._n_vars(mode)
        for a, name in ((lower, "lower"), (upper, "upper"), (initial_step, "initial_step")):
            if a is not None:
                _require(a, (B, nv), name)
        nz, ny, nx = occupancy.shape
        x = x0.clone()
        cost = torch.empty(B, dtype=torch.float64, device=dev)
        ev = torch.empty(B, dtype=torch.int32, device=dev)
        res = torch.empty(B, dtype=torch.int32, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        terms = torch.empty((B, 4), dtype=torch.float64, device=dev)
        nb = self.coll_workspace_bytes(B, params, mode, True)
        ws = _workspace(workspace, nb, dev)
        hist = (torch.full((B, max_evals, nv), float("nan"), dtype=torch.float64, device=dev)
                if history else None)
        check(lib().mtg_coll_optimize_trace(self._h, B, mode, _ptr(fixed_vals), _ptr(x),
                                            _ptr(times) if mode == 0 else None, _ptr(lower),
                                            _ptr(upper), _ptr(initial_step), _ptr(occupancy), nx,
                                            ny, nz, _ptr(near_field), ctypes.byref(params),
                                            max_evals, _ptr(cost), _ptr(ev), _ptr(res), _ptr(st),
                                            _ptr(terms), _ptr(hist), _ptr(ws), nb, _stream(dev)),
              "mtg_coll_optimize_trace")
        out = dict(x=x, cost=cost, evals=ev, result=res, status=st, terms=terms)
        if history:
            out["x_history"] = hist
        return out

    # -- host (numpy) API ---------------------------------------------------
    def solve_host(self, fixed_vals, times):
        fixed_vals = np.ascontiguousarray(fixed_vals, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        B = times.shape[0]
        coeffs = np.zeros((B, self.S, self.D, self.N))
        cost = np.zeros(B)
        free = np.zeros((B, self.D, self.n_free))
        status = np.zeros(B, dtype=np.int32)
        dp = ctypes.POINTER(ctypes.c_double)
        rc = lib().mtg_linear_solve_host(
            self._h, B, fixed_vals.ctypes.data_as(dp), times.ctypes.data_as(dp),
            coeffs.ctypes.data_as(dp), cost.ctypes.data_as(dp), free.ctypes.data_as(dp),
            status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if rc not in (0, _abi_numeric()):
            check(rc, "mtg_linear_solve_host")
        return dict(coeffs=coeffs, cost=cost, free=free, status=status)


def _abi_numeric():
    return -5  # MTG_ERR_NUMERIC: per-trajectory status carries the detail


def segment_matrices(ctx, N, r, times):
    """Q, A, A^-1, H for each time in a CUDA float64 tensor [n] -> 4 x [n, N, N]."""
    import torch
    n = times.shape[0]
    _require(times, (n,), "times")
    outs = [torch.empty((n, N, N), dtype=torch.float64, device=times.device) for _ in range(4)]
    check(lib().mtg_segment_matrices(ctx.handle, N, r, n, _ptr(times), *[_ptr(o) for o in outs],
                                     _stream(times.device)), "mtg_segment_matrices")
    return outs


def generate_random_problems(N, D, S, B, seed0=105, pos_bound=10.0, v_max=3.0, a_max=5.0):
    """Standard-pattern batch (host): mask [(S+1), N/2], fixed_vals [B, D, n_f],
    times [B, S], positions [B, S+1, D] — createRandomVertices(seed0 + b) +
    estimateSegmentTimes, bit-identical to the reference generator."""
    M = N // 2
    nf = 2 * M + (S - 1)
    mask = np.zeros((S + 1, M), np.uint8)
    fixed = np.zeros((B, D, nf))
    times = np.zeros((B, S))
    pos = np.zeros((B, S + 1, D))
    dp = ctypes.POINTER(ctypes.c_double)
    check(lib().mtg_generate_random_problems(
        N, D, S, B, seed0, pos_bound, v_max, a_max,
        mask.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), fixed.ctypes.data_as(dp),
        times.ctypes.data_as(dp), pos.ctypes.data_as(dp)), "mtg_generate_random_problems")
    return mask, fixed, times, pos


def tube_num_constraints(N, S):
    return lib().mtg_tube_num_constraints(N, S)


def tube_residuals(ctx, N, r, positions, fixed_vals, times_cp, times, radii, x):
    import torch
    B, S = times.shape
    m = tube_num_constraints(N, S)
    resid = torch.empty((B, m), dtype=torch.float64, device=times.device)
    check(lib().mtg_tube_residuals(ctx.handle, N, r, S, B, _ptr(positions), _ptr(fixed_vals),
                                   _ptr(times_cp), _ptr(times), _ptr(radii), _ptr(x),
                                   _ptr(resid), _stream(times.device)), "mtg_tube_residuals")
    return resid


def tube_solve(ctx, N, r, positions, fixed_vals, times_cp, times, radii, tol=1e-10,
               max_iter=100):
    import torch
    B, S = times.shape
    dev = times.device
    for name, t, shp in (("positions", positions, (B, S + 1, 3)),
                         ("fixed_vals", fixed_vals, (B, 3, N)),
                         ("times_cp", times_cp, (B, S)), ("radii", radii, (B, S, 2))):
        _require(t, shp, name)
    n = 3 * (S - 1) * (N // 2)
    x = torch.empty((B, n), dtype=torch.float64, device=dev)
    coeffs = torch.empty((B, S, 3, N), dtype=torch.float64, device=dev)
    cost = torch.empty(B, dtype=torch.float64, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    check(lib().mtg_tube_solve(ctx.handle, N, r, S, B, _ptr(positions), _ptr(fixed_vals),
                               _ptr(times_cp), _ptr(times), _ptr(radii), tol, max_iter, _ptr(x),
                               _ptr(coeffs), _ptr(cost), _ptr(iters), _ptr(status),
                               _stream(dev)), "mtg_tube_solve")
    return dict(x=x, coeffs=coeffs, cost=cost, iters=iters, status=status)


def _tube_geometry(N, positions, fixed_vals, radii, B, S):
    for name, t, shp in (("positions", positions, (B, S + 1, 3)),
                         ("fixed_vals", fixed_vals, (B, 3, N)), ("radii", radii, (B, S, 2))):
        _require(t, shp, name)


def tube_time_workspace_bytes(N, S, B, params, optimize):
    """Device scratch the QCQP time objective / optimiser needs
    (mtg_tube_time_workspace_bytes)."""
    n = lib().mtg_tube_time_workspace_bytes(N, S, B, ctypes.byref(params), 1 if optimize else 0)
    if n < 0:
        check(int(n), "mtg_tube_time_workspace_bytes")
    return int(n)


def _workspace(workspace, nbytes, dev):
    import torch
    if workspace is None:
        return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    if not isinstance(workspace, torch.Tensor) or not workspace.is_cuda or \
            not workspace.is_contiguous() or workspace.numel() * workspace.element_size() < nbytes:
        raise MTGError(f"workspace must be a contiguous CUDA tensor of >= {nbytes} bytes")
    return workspace


def tube_time_cost(ctx, N, r, positions, fixed_vals, times_cp, times, radii, time_penalty=500.0,
                   grad=False, increment=0.1, soft=None, soft_weight=100.0, tol=1e-10,
                   max_iter=100, workspace=None):
    """objectiveFunctionTime with the QCQP inner solve (mtg_tube_time_cost):
    J = computeCost() of the tube QCQP at `times` + time_penalty (sum T)^2
    [+ soft]; grad=True adds the central-difference gradient (grad_mode 2).
    workspace: optional device tensor of >= tube_time_workspace_bytes bytes
    (allocated from torch's caching allocator when None).
    Returns dict(cost [B], grad [B, S] or None, status [B])."""
    import torch
    B, S = times.shape
    dev = times.device
    _tube_geometry(N, positions, fixed_vals, radii, B, S)
    _require(times_cp, (B, S), "times_cp")
    _require(times, (B, S), "times")
    p = make_time_params(time_penalty, increment, 0.1, 1.0, 2 if grad else 0, soft, soft_weight)
    cost = torch.empty(B, dtype=torch.float64, device=dev)
    g = torch.empty((B, S), dtype=torch.float64, device=dev) if grad else None
    status = torch.empty(B, dtype=torch.int32, device=dev)
    nbytes = tube_time_workspace_bytes(N, S, B, p, False)
    ws = _workspace(workspace, nbytes, dev)
    check(lib().mtg_tube_time_cost(ctx.handle, N, r, S, B, _ptr(positions), _ptr(fixed_vals),
                                   _ptr(times_cp), _ptr(times), _ptr(radii), tol, max_iter,
                                   ctypes.byref(p), _ptr(cost), _ptr(g), _ptr(status), _ptr(ws),
                                   ws.numel() * ws.element_size(), _stream(dev)),
          "mtg_tube_time_cost")
    return dict(cost=cost, grad=g, status=status)


def tube_time_optimize(ctx, N, r, positions, fixed_vals, radii, times, max_evals,
                       time_penalty=500.0, increment=0.1, soft=None, soft_weight=100.0,
                       tol=1e-10, max_iter=100, workspace=None, optimizer="fd", f_rel=0.05,
                       f_abs=-1.0, initial_stepsize_rel=0.1):
    """optimizeTime in the fork's QCQP form (mtg_tube_time_optimize_ex).  times
    [B, S] are the initial times (and the control-point times).  optimizer
    "sbplx" runs LN_SBPLX, the reference's default (one QCQP per evaluation,
    f_rel / f_abs / initial_stepsize_rel as NonlinearOptimizationParameters);
    "fd" the projected central-difference descent.  Returns dict(times, cost,
    evals, result, status) with new tensors; result is the nlopt_result code."""
    import torch
    B, S = times.shape
    dev = times.device
    _tube_geometry(N, positions, fixed_vals, radii, B, S)
    _require(times, (B, S), "times")
    p = make_time_params(time_penalty, increment, 0.1, 1.0, 2, soft, soft_weight,
                         optimizer=optimizer, f_rel=f_rel, f_abs=f_abs,
                         initial_stepsize_rel=initial_stepsize_rel)
    t = times.clone()
    cost = torch.empty(B, dtype=torch.float64, device=dev)
    evals = torch.empty(B, dtype=torch.int32, device=dev)
    result = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    nbytes = tube_time_workspace_bytes(N, S, B, p, True)
    ws = _workspace(workspace, nbytes, dev)
    check(lib().mtg_tube_time_optimize_ex(ctx.handle, N, r, S, B, _ptr(positions),
                                          _ptr(fixed_vals), _ptr(radii), _ptr(t), tol, max_iter,
                                          ctypes.byref(p), max_evals, _ptr(cost), _ptr(evals),
                                          _ptr(result), _ptr(status), _ptr(ws),
                                          ws.numel() * ws.element_size(), _stream(dev)),
          "mtg_tube_time_optimize_ex")
    return dict(times=t, cost=cost, evals=evals, result=result, status=status)


def sample_trajectories(coeffs, times, dt, t_start=0.0, t_end=-1.0, max_derivative=0,
                        n_max=None, with_times=True):
    """Batched Trajectory::evaluateRange (trajectory.cpp:74-134) for derivatives
    0..max_derivative (mtg_sample_trajectories).

    coeffs [B, S, D, N], times [B, S] (float64, CUDA).  Returns (samples
    [B, (max_derivative+1)*D, n_max] channel-major, sample_times [B, n_max]
    or None, n_samples [B] int32).  n_max defaults to the longest trajectory's
    sample count.
    """
    import torch
    B, S, D, N = coeffs.shape
    _require(coeffs, (B, S, D, N), "coeffs")
    _require(times, (B, S), "times")
    dev = times.device
    if not dt > 0:
        raise MTGError("dt must be > 0")
    if n_max is None:
        span = float(times.sum(dim=1).max().item()) if t_end < 0 else t_end
        n_max = int(span / dt) + 2
        n_max = (n_max + 63) // 64 * 64  # 512-byte aligned channel rows
    nch = (max_derivative + 1) * D
    samples = torch.empty((B, nch, n_max), dtype=torch.float64, device=dev)
    stimes = torch.empty((B, n_max), dtype=torch.float64, device=dev) if with_times else None
    count = torch.empty(B, dtype=torch.int32, device=dev)
    check(lib().mtg_sample_trajectories(N, D, S, B, _ptr(coeffs), _ptr(times), t_start, t_end,
                                        dt, n_max, max_derivative, _ptr(samples), _ptr(stimes),
                                        _ptr(count), _stream(dev)), "mtg_sample_trajectories")
    return samples, stimes, count


def max_magnitude(coeffs, times, derivative, out=None):
    """Batched PolynomialOptimization::computeMaximumOfMagnitude
    (linear_impl:455-487; mtg_max_magnitude).

    coeffs [B, S, D, N], times [B, S] (float64, CUDA).  Returns a dict of
    time [B] (relative to the segment start), value [B], segment [B] int32:
    the Extremum of |p^(derivative)| over the trajectory.
    """
    import torch
    B, S, D, N = coeffs.shape
    _require(coeffs, (B, S, D, N), "coeffs")
    _require(times, (B, S), "times")
    dev = times.device
    if out is None:
        out = {"time": torch.empty(B, dtype=torch.float64, device=dev),
               "value": torch.empty(B, dtype=torch.float64, device=dev),
               "segment": torch.empty(B, dtype=torch.int32, device=dev)}
    check(lib().mtg_max_magnitude(N, D, S, B, _ptr(coeffs), _ptr(times), derivative,
                                  _ptr(out["time"]), _ptr(out["value"]), _ptr(out["segment"]),
                                  _stream(dev)), "mtg_max_magnitude")
    return out


def _check_field(field, occupancy):
    if field is None:
        return
    import torch
    nz, ny, nx = occupancy.shape
    if not (isinstance(field, torch.Tensor) and field.is_cuda and field.dtype == torch.int16 and
            field.is_contiguous() and field.numel() == nz * ny * nx * 8):
        raise MTGError("near_field must be coll_field()'s int16 CUDA tensor [nz, ny, nx, 8]")


def coll_field(occupancy, params):
    """Near field of an occupancy map for the collision walk (mtg_coll_field):
    per voxel the seven box minima the walk would scan for (uint16 bits in an
    int16 tensor [nz, ny, nx, 8]).  params: make_coll_params(...) or
    make_collision_params(...) (only box_side is read).  Compute once per map
    and pass as near_field to LinearPlan.coll_cost / coll_optimize."""
    import torch
    nz, ny, nx = occupancy.shape
    cp = getattr(params, "coll", params)
    field = torch.empty((nz, ny, nx, 8), dtype=torch.int16, device=occupancy.device)
    check(lib().mtg_coll_field(_ptr(occupancy), nx, ny, nz, ctypes.byref(cp), _ptr(field),
                               _stream(occupancy.device)), "mtg_coll_field")
    return field


def magnitude_candidates(coeffs, times, derivative, max_candidates=None):
    """Batched candidate lists of the magnitude extrema
    (Segment::computeMinMaxMagnitudeCandidates, segment.cpp:82-161, per
    segment over all D dimensions; mtg_magnitude_candidates).

    coeffs [B, S, D, N], times [B, S] (float64, CUDA).  Returns a dict of
    time / value [B, S, C] and count [B, S] int32: per segment t = 0, T and
    the real roots of d/dt |p^(derivative)|^2 in [0, T] ascending, with
    |p^(derivative)| at each.  C defaults to 2 (N - derivative) - 1, which
    always suffices.  count is the number of candidates the search found, as
    the C ABI returns it (a count above C means a smaller max_candidates
    truncated the list); stored [B, S] = min(count, C) is the number of
    valid entries, and entries past it are unset.  (Round 4 had briefly
    clamped count and moved the found number to a "found" key; that
    alias is kept for callers written against it.)
    """
    import torch
    B, S, D, N = coeffs.shape
    _require(coeffs, (B, S, D, N), "coeffs")
    _require(times, (B, S), "times")
    dev = times.device
    C = int(max_candidates or 2 * (N - derivative) - 1)
    out = {"time": torch.empty((B, S, C), dtype=torch.float64, device=dev),
           "value": torch.empty((B, S, C), dtype=torch.float64, device=dev),
           "count": torch.empty((B, S), dtype=torch.int32, device=dev)}
    check(lib().mtg_magnitude_candidates(N, D, S, B, _ptr(coeffs), _ptr(times), derivative, C,
                                         _ptr(out["time"]), _ptr(out["value"]),
                                         _ptr(out["count"]), _stream(dev)),
          "mtg_magnitude_candidates")
    out["stored"] = torch.clamp(out["count"], max=C)
    out["found"] = out["count"]
    return out


def min_max_magnitude(coeffs, times, derivative):
    """Batched Trajectory::computeMinMaxMagnitude (trajectory.cpp:184-220;
    mtg_min_max_magnitude) over all D dimensions of coeffs [B, S, D, N].
    Returns a dict of min_time, min_value, min_segment, max_time, max_value,
    max_segment [B]."""
    import torch
    B, S, D, N = coeffs.shape
    _require(coeffs, (B, S, D, N), "coeffs")
    _require(times, (B, S), "times")
    dev = times.device
    out = {k: torch.empty(B, dtype=torch.float64, device=dev)
           for k in ("min_time", "min_value", "max_time", "max_value")}
    out["min_segment"] = torch.empty(B, dtype=torch.int32, device=dev)
    out["max_segment"] = torch.empty(B, dtype=torch.int32, device=dev)
    check(lib().mtg_min_max_magnitude(N, D, S, B, _ptr(coeffs), _ptr(times), derivative,
                                      _ptr(out["min_time"]), _ptr(out["min_value"]),
                                      _ptr(out["min_segment"]), _ptr(out["max_time"]),
                                      _ptr(out["max_value"]), _ptr(out["max_segment"]),
                                      _stream(dev)), "mtg_min_max_magnitude")
    return out


def soft_constraint_cost(coeffs, times, derivatives, limits, weight=100.0, maximum_cost=1.0e12,
                         out=None):
    """Batched evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:
    2735-2766; mtg_soft_constraint_cost) for the constraints
    (derivatives[c], limits[c]) of addMaximumMagnitudeConstraint.

    Returns a dict of cost [B] and maxima [B, n_constraints].
    """
    import ctypes

    import torch
    B, S, D, N = coeffs.shape
    _require(coeffs, (B, S, D, N), "coeffs")
    _require(times, (B, S), "times")
    nc = len(derivatives)
    if len(limits) != nc:
        raise MTGError("derivatives and limits differ in length")
    dev = times.device
    if out is None:
        out = {"cost": torch.empty(B, dtype=torch.float64, device=dev),
               "maxima": torch.empty((B, nc), dtype=torch.float64, device=dev)}
    der = (ctypes.c_int * max(nc, 1))(*[int(d) for d in derivatives])
    lim = (ctypes.c_double * max(nc, 1))(*[float(v) for v in limits])
    check(lib().mtg_soft_constraint_cost(N, D, S, B, _ptr(coeffs), _ptr(times), nc, der, lim,
                                         float(weight), float(maximum_cost), _ptr(out["maxima"]),
                                         _ptr(out["cost"]), _stream(dev)),
          "mtg_soft_constraint_cost")
    return out
