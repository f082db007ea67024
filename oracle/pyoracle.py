"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes view of oracle/liboracle.so, the FP64 CPU restatement of the
reference's hot path (see oracle/mtg_oracle.h for the per-function reference
citations).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg import this module; the product package never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_ip = ctypes.POINTER(ctypes.c_int)


def build():
    """Compile liboracle.so from oracle/mtg_oracle.cpp (g++ only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        L = _lib
        L.orc_base_coefficients.argtypes = [ctypes.c_int, _dp]
        L.orc_base_coeffs_with_time.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp]
        L.orc_segment_matrices.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp]
        L.orc_random_vertices.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                          ctypes.c_uint64, ctypes.c_int, _u8p, _dp]
        L.orc_estimate_segment_times.argtypes = [ctypes.c_int, ctypes.c_int, _dp, ctypes.c_double,
                                                 ctypes.c_double, ctypes.c_int, ctypes.c_double, _dp]
        L.orc_linear_solve.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, _dp, _dp, _dp, _dp, _ip, _ip]
        L.orc_linear_matrices.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.orc_time_cost.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, ctypes.c_double, ctypes.c_int,
                                                         ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                                         _dp, _dp]
        L.orc_control_point_map.argtypes = [ctypes.c_int, ctypes.c_double, _dp]
        L.orc_tube_num_constraints.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_tube_qcqp_assemble.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, _dp, _dp, _dp, _dp, _dp,
                                                                  _dp, _dp, _ip]
        L.orc_tube_residuals.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, _dp, _dp, _dp, _dp]
        L.orc_tube_qcqp_solve.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, _dp, _dp, ctypes.c_double,
                                                               ctypes.c_int, _dp, _dp, _dp, _ip]
    return _lib


def _d(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"oracle {what} failed with status {rc}")
    return rc


def base_coefficients(n=22):
    out = np.zeros((n, n))
    _check(lib().orc_base_coefficients(n, _d(out)), "base_coefficients")
    return out


def base_coeffs_with_time(N, deriv, t):
    out = np.zeros(N)
    _check(lib().orc_base_coeffs_with_time(N, deriv, t, _d(out)), "base_coeffs_with_time")
    return out


def segment_matrices(N, r, T):
    Q, A, Ai, H = (np.zeros((N, N)) for _ in range(4))
    _check(lib().orc_segment_matrices(N, r, T, _d(Q), _d(A), _d(Ai), _d(H)), "segment_matrices")
    return Q, A, Ai, H


class Vertices:
    """Dense vertex constraints: mask[(S+1), K], vals[(S+1), K, D]."""

    def __init__(self, mask, vals):
        self.mask = np.ascontiguousarray(mask, dtype=np.uint8)
        self.vals = np.ascontiguousarray(vals, dtype=np.float64)

    @property
    def S(self):
        return self.mask.shape[0] - 1

    @property
    def K(self):
        return self.mask.shape[1]

    @property
    def D(self):
        return self.vals.shape[2]

    def positions(self):
        return np.ascontiguousarray(self.vals[:, 0, :])


def random_vertices(max_deriv, S, D, pos_min, pos_max, seed, K=None):
    K = K or (max_deriv + 1)
    mask = np.zeros((S + 1, K), np.uint8)
    vals = np.zeros((S + 1, K, D))
    pmin = np.ascontiguousarray(np.broadcast_to(np.asarray(pos_min, float), (D,)))
    pmax = np.ascontiguousarray(np.broadcast_to(np.asarray(pos_max, float), (D,)))
    _check(lib().orc_random_vertices(max_deriv, S, D, _d(pmin), _d(pmax), seed, K,
                                     mask.ctypes.data_as(_u8p), _d(vals)), "random_vertices")
    return Vertices(mask, vals)


def estimate_segment_times(vertices, v_max, a_max, method=0, magic=6.5):
    pos = vertices.positions()
    t = np.zeros(vertices.S)
    _check(lib().orc_estimate_segment_times(vertices.S, vertices.D, _d(pos), v_max, a_max,
                                            method, magic, _d(t)), "estimate_segment_times")
    return t


def linear_solve(N, r, vertices, times):
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    coeffs = np.zeros((S, D, N))
    cost = np.zeros(1)
    nf, np_ = ctypes.c_int(), ctypes.c_int()
    n_all = (S + 1) * (N // 2)
    df = np.zeros(D * n_all)
    dp = np.zeros(D * n_all)
    rc = lib().orc_linear_solve(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p), _d(vertices.vals),
                                _d(times), _d(coeffs), _d(cost), _d(df), _d(dp),
                                ctypes.byref(nf), ctypes.byref(np_))
    _check(rc, "linear_solve")
    nf, np_ = nf.value, np_.value
    return dict(coeffs=coeffs, cost=float(cost[0]), df=df[:D * nf].reshape(D, nf),
                dp=dp[:D * np_].reshape(D, np_), nf=nf, np=np_, status=rc)


def linear_matrices(N, r, vertices, times):
    S, D, K = vertices.S, vertices.D, vertices.K
    sol = linear_solve(N, r, vertices, times)
    nc = sol["nf"] + sol["np"]
    NS = N * S
    R = np.zeros((nc, nc))
    M = np.zeros((NS, nc))
    A = np.zeros((NS, NS))
    Ai = np.zeros((NS, NS))
    Mp = np.zeros((nc, NS))
    times = np.ascontiguousarray(times, dtype=np.float64)
    _check(lib().orc_linear_matrices(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                     _d(vertices.vals), _d(times), _d(R), _d(M), _d(A), _d(Ai),
                                     _d(Mp)), "linear_matrices")
    return dict(R=R, M=M, A=A, Ainv=Ai, Mpinv=Mp, **sol)


def time_cost(N, r, vertices, times, time_penalty=500.0, grad_mode=0, increment=0.1,
              w_d=0.1, w_t=1.0, soft=None, soft_weight=100.0, soft_maximum_cost=1.0e12):
    """objectiveFunctionTime (orc_time_cost / orc_time_cost_soft); soft: list
    of (derivative, maximum_value) soft magnitude constraints."""
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    cost = np.zeros(1)
    grad = np.zeros(S)
    L = lib()
    if soft:
        der = np.ascontiguousarray([d for d, _ in soft], dtype=np.int32)
        lim = np.ascontiguousarray([v for _, v in soft], dtype=np.float64)
        L.orc_time_cost_soft.argtypes = [ctypes.c_int] * 5 + [
            _u8p, _dp, _dp, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double,
            ctypes.c_double, ctypes.c_int, _ip, _dp, ctypes.c_double, ctypes.c_double, _dp, _dp]
        _check(L.orc_time_cost_soft(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                    _d(vertices.vals), _d(times), time_penalty, grad_mode,
                                    increment, w_d, w_t, len(der), der.ctypes.data_as(_ip),
                                    _d(lim), soft_weight, soft_maximum_cost, _d(cost), _d(grad)),
               "time_cost_soft")
    else:
        _check(L.orc_time_cost(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                               _d(vertices.vals), _d(times), time_penalty, grad_mode, increment,
                               w_d, w_t, _d(cost), _d(grad)), "time_cost")
    return float(cost[0]), (grad if grad_mode else None)


def time_optimize(N, r, vertices, times, max_evals, time_penalty=500.0, increment=0.1,
                  soft=None, soft_weight=100.0, soft_maximum_cost=1.0e12, hard=False,
                  hard_tolerance=0.1):
    """orc_time_optimize(_soft / _hard): the mtg_time_optimize algorithm on
    the oracle objective.  Returns (times, cost, evals)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    t = np.array(times, dtype=np.float64)
    cost = np.zeros(1)
    evals = ctypes.c_int()
    L = lib()
    if soft and hard:
        der = np.ascontiguousarray([d for d, _ in soft], dtype=np.int32)
        lim = np.ascontiguousarray([v for _, v in soft], dtype=np.float64)
        L.orc_time_optimize_hard.argtypes = [ctypes.c_int] * 5 + [
            _u8p, _dp, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int, _ip,
            _dp, ctypes.c_double, _dp, _ip]
        _check(L.orc_time_optimize_hard(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                        _d(vertices.vals), _d(t), time_penalty, increment,
                                        max_evals, len(der), der.ctypes.data_as(_ip), _d(lim),
                                        hard_tolerance, _d(cost), ctypes.byref(evals)),
               "time_optimize_hard")
    elif soft:
        der = np.ascontiguousarray([d for d, _ in soft], dtype=np.int32)
        lim = np.ascontiguousarray([v for _, v in soft], dtype=np.float64)
        L.orc_time_optimize_soft.argtypes = [ctypes.c_int] * 5 + [
            _u8p, _dp, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int, _ip,
            _dp, ctypes.c_double, ctypes.c_double, _dp, _ip]
        _check(L.orc_time_optimize_soft(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                        _d(vertices.vals), _d(t), time_penalty, increment,
                                        max_evals, len(der), der.ctypes.data_as(_ip), _d(lim),
                                        soft_weight, soft_maximum_cost, _d(cost),
                                        ctypes.byref(evals)), "time_optimize_soft")
    else:
        L.orc_time_optimize.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, ctypes.c_double,
                                                             ctypes.c_double, ctypes.c_int, _dp,
                                                             _ip]
        _check(L.orc_time_optimize(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                   _d(vertices.vals), _d(t), time_penalty, increment, max_evals,
                                   _d(cost), ctypes.byref(evals)), "time_optimize")
    return t, float(cost[0]), evals.value


def sbplx_test(lb, ub, x0, xstep, maxeval, ftol_rel=0.05, ftol_abs=-1.0):
    """orc_sbplx_test: the LN_SBPLX restatement (orc_sbplx.cpp) on its fixed
    test objective.  Returns (code, x, minf, nevals, history [nevals, n])."""
    n = len(x0)
    x = np.array(x0, dtype=np.float64)
    lb = np.ascontiguousarray(lb, dtype=np.float64)
    ub = np.ascontiguousarray(ub, dtype=np.float64)
    st = np.ascontiguousarray(xstep, dtype=np.float64)
    hist = np.zeros((maxeval, n))
    minf = np.zeros(1)
    nev = ctypes.c_int()
    L = lib()
    L.orc_sbplx_test.argtypes = [ctypes.c_int, _dp, _dp, _dp, _dp, ctypes.c_int,
                                 ctypes.c_double, ctypes.c_double, _dp, _ip, _dp]
    code = L.orc_sbplx_test(n, _d(lb), _d(ub), _d(x), _d(st), maxeval, ftol_rel, ftol_abs,
                            _d(minf), ctypes.byref(nev), _d(hist))
    return code, x, float(minf[0]), nev.value, hist[:nev.value]


def time_optimize_sbplx(N, r, vertices, times, max_evals, time_penalty=500.0, f_rel=0.05,
                        f_abs=-1.0, step_rel=0.1, soft=None, soft_weight=100.0,
                        soft_maximum_cost=1.0e12):
    """orc_time_optimize_sbplx: optimizeTime (nonlinear_impl:332-397) with
    the LN_SBPLX restatement on objectiveFunctionTime (linear inner solve):
    bounds [0.1, 2 T0], initial step step_rel T0, maxeval max_evals.
    Returns (times, cost, evals, result, history [evals, S])."""
    S, D, K = vertices.S, vertices.D, vertices.K
    t = np.array(times, dtype=np.float64)
    cost = np.zeros(1)
    evals, result = ctypes.c_int(), ctypes.c_int()
    hist = np.zeros((max_evals, S))
    der = np.ascontiguousarray([d for d, _ in (soft or [])] or [0], dtype=np.int32)
    lim = np.ascontiguousarray([v for _, v in (soft or [])] or [1.0], dtype=np.float64)
    L = lib()
    L.orc_time_optimize_sbplx.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double,
        ctypes.c_double, ctypes.c_int, _ip, _dp, ctypes.c_double, ctypes.c_double, _dp, _ip,
        _ip, _dp]
    _check(L.orc_time_optimize_sbplx(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                     _d(vertices.vals), _d(t), time_penalty, max_evals, f_rel,
                                     f_abs, step_rel, len(soft or []), der.ctypes.data_as(_ip),
                                     _d(lim), soft_weight, soft_maximum_cost, _d(cost),
                                     ctypes.byref(evals), ctypes.byref(result), _d(hist)),
           "time_optimize_sbplx")
    return t, float(cost[0]), evals.value, result.value, hist[:evals.value]


def bench_workload(kind, N, D, r, S, K, masks, vals, times, radii=None, param_i=0,
                   param_d=0.0, threads=1, seconds=10.0):
    """orc_bench_workload (kind 1 time optimisation, 2 tube, 3 sampling).
    Returns (units, seconds)."""
    L = lib()
    L.orc_bench_workload.argtypes = [ctypes.c_int] * 7 + [_u8p, _dp, _dp, _dp, ctypes.c_int,
                                                          ctypes.c_double, ctypes.c_int,
                                                          ctypes.c_double,
                                                          ctypes.POINTER(ctypes.c_int64), _dp]
    masks = np.ascontiguousarray(masks, dtype=np.uint8)
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    rad = None if radii is None else np.ascontiguousarray(radii, dtype=np.float64)
    units = ctypes.c_int64()
    sec = np.zeros(1)
    _check(L.orc_bench_workload(kind, N, D, r, S, K, masks.shape[0],
                                masks.ctypes.data_as(_u8p), _d(vals), _d(times),
                                _d(rad) if rad is not None else None, param_i, param_d, threads,
                                seconds, ctypes.byref(units), _d(sec)), "bench_workload")
    return units.value, float(sec[0])

def control_point_map(N, T):
    B = np.zeros((N, N))
    _check(lib().orc_control_point_map(N, T, _d(B)), "control_point_map")
    return B


def tube_num_constraints(N, S):
    return lib().orc_tube_num_constraints(N, S)


def tube_assemble(N, r, vertices, times, radii, times_cp=None, with_quad=True):
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    times_cp = times if times_cp is None else np.ascontiguousarray(times_cp, dtype=np.float64)
    radii = np.ascontiguousarray(radii, dtype=np.float64).reshape(S, 2)
    n = (S - 1) * (N // 2) * D
    m = tube_num_constraints(N, S)
    P = np.zeros((n, n))
    q = np.zeros(n)
    quad = np.zeros((m, n, n)) if with_quad else None
    lin = np.zeros((m, n))
    cst = np.zeros(m)
    nfree = ctypes.c_int()
    _check(lib().orc_tube_qcqp_assemble(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                        _d(vertices.vals), _d(times_cp), _d(times), _d(radii),
                                        _d(P), _d(q), _d(quad), _d(lin), _d(cst),
                                        ctypes.byref(nfree)), "tube_assemble")
    return dict(P=P, q=q, quad=quad, lin=lin, cst=cst, n=nfree.value)


def tube_residuals(N, r, vertices, times, radii, x, times_cp=None):
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    times_cp = times if times_cp is None else np.ascontiguousarray(times_cp, dtype=np.float64)
    radii = np.ascontiguousarray(radii, dtype=np.float64).reshape(S, 2)
    x = np.ascontiguousarray(x, dtype=np.float64)
    res = np.zeros(tube_num_constraints(N, S))
    _check(lib().orc_tube_residuals(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                    _d(vertices.vals), _d(times_cp), _d(times), _d(radii), _d(x),
                                    _d(res)), "tube_residuals")
    return res


def tube_solve(N, r, vertices, times, radii, times_cp=None, tol=1e-10, max_iter=100):
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    times_cp = times if times_cp is None else np.ascontiguousarray(times_cp, dtype=np.float64)
    radii = np.ascontiguousarray(radii, dtype=np.float64).reshape(S, 2)
    n = (S - 1) * (N // 2) * D
    x = np.zeros(n)
    coeffs = np.zeros((S, D, N))
    cost = np.zeros(1)
    iters = ctypes.c_int()
    rc = lib().orc_tube_qcqp_solve(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                   _d(vertices.vals), _d(times_cp), _d(times), _d(radii), tol,
                                   max_iter, _d(x), _d(coeffs), _d(cost), ctypes.byref(iters))
    _check(rc, "tube_solve")
    return dict(x=x, coeffs=coeffs, cost=float(cost[0]), iters=iters.value, status=rc)


def tube_time_cost(N, r, vertices, times, radii, times_cp=None, tol=1e-10, max_iter=100,
                   time_penalty=500.0, grad_mode=0, increment=0.1, soft=None,
                   soft_weight=100.0, soft_maximum_cost=1.0e12):
    """orc_tube_time_cost: objectiveFunctionTime with the QCQP inner solve.
    Returns (J, grad or None)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    times_cp = times if times_cp is None else np.ascontiguousarray(times_cp, dtype=np.float64)
    radii = np.ascontiguousarray(radii, dtype=np.float64).reshape(S, 2)
    cost = np.zeros(1)
    grad = np.zeros(S)
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_tube_time_cost.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int,
        ctypes.c_double, ctypes.c_int, _ip, _dp, ctypes.c_double, ctypes.c_double, _dp, _dp]
    _check(L.orc_tube_time_cost(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                _d(vertices.vals), _d(times_cp), _d(times), _d(radii), tol,
                                max_iter, time_penalty, grad_mode, increment, ns,
                                der.ctypes.data_as(_ip), _d(lim), soft_weight, soft_maximum_cost,
                                _d(cost), _d(grad)), "tube_time_cost")
    return float(cost[0]), (grad if grad_mode == 2 else None)


def tube_time_optimize(N, r, vertices, times, radii, max_evals, tol=1e-10, max_iter=100,
                       time_penalty=500.0, increment=0.1, soft=None, soft_weight=100.0,
                       soft_maximum_cost=1.0e12):
    """orc_tube_time_optimize: the mtg_tube_time_optimize algorithm.
    Returns (times, cost, evals)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    t = np.array(times, dtype=np.float64)
    radii = np.ascontiguousarray(radii, dtype=np.float64).reshape(S, 2)
    cost = np.zeros(1)
    evals = ctypes.c_int()
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_tube_time_optimize.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double,
        ctypes.c_int, ctypes.c_int, _ip, _dp, ctypes.c_double, ctypes.c_double, _dp,
        ctypes.POINTER(ctypes.c_int)]
    _check(L.orc_tube_time_optimize(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                    _d(vertices.vals), _d(radii), _d(t), tol, max_iter,
                                    time_penalty, increment, max_evals, ns,
                                    der.ctypes.data_as(_ip), _d(lim), soft_weight,
                                    soft_maximum_cost, _d(cost), ctypes.byref(evals)),
           "tube_time_optimize")
    return t, float(cost[0]), evals.value


def tube_time_optimize_sbplx(N, r, vertices, times, radii, max_evals, tol=1e-10, max_iter=100,
                             time_penalty=500.0, f_rel=0.05, f_abs=-1.0, step_rel=0.1,
                             soft=None, soft_weight=100.0, soft_maximum_cost=1.0e12):
    """orc_tube_time_optimize_sbplx: optimizeTime in the fork's QCQP form with
    LN_SBPLX (nonlinear_impl:332-397, 877-945).  Returns dict(times, cost,
    evals, result, history [evals, S])."""
    S, D, K = vertices.S, vertices.D, vertices.K
    t = np.array(times, dtype=np.float64)
    radii = np.ascontiguousarray(radii, dtype=np.float64).reshape(S, 2)
    cost = np.zeros(1)
    evals = ctypes.c_int()
    result = ctypes.c_int()
    hist = np.zeros((max_evals, S))
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_tube_time_optimize_sbplx.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int,
        ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, _ip, _dp,
        ctypes.c_double, ctypes.c_double, _dp, ctypes.POINTER(ctypes.c_int),
        ctypes.POINTER(ctypes.c_int), _dp]
    _check(L.orc_tube_time_optimize_sbplx(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                          _d(vertices.vals), _d(radii), _d(t), tol, max_iter,
                                          time_penalty, max_evals, f_rel, f_abs, step_rel, ns,
                                          der.ctypes.data_as(_ip), _d(lim), soft_weight,
                                          soft_maximum_cost, _d(cost), ctypes.byref(evals),
                                          ctypes.byref(result), _d(hist)),
           "tube_time_optimize_sbplx")
    return dict(times=t, cost=float(cost[0]), evals=evals.value, result=result.value,
                history=hist[:evals.value])


def evaluate_range(N, coeffs, times, t_start, t_end, dt, derivative, max_out=None):
    """Trajectory::evaluateRange (trajectory.cpp:74-134) on coeffs [S, D, N]."""
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    S, D, _ = coeffs.shape
    if max_out is None:
        max_out = int((t_end if t_end >= 0 else times.sum()) / dt) + 8
    out = np.zeros((max_out, D))
    tout = np.zeros(max_out)
    count = ctypes.c_int()
    L = lib()
    L.orc_evaluate_range.argtypes = [ctypes.c_int] * 3 + [_dp, _dp] + [ctypes.c_double] * 3 + [
        ctypes.c_int, ctypes.c_int, _dp, _dp, ctypes.POINTER(ctypes.c_int)]
    _check(L.orc_evaluate_range(N, D, S, _d(coeffs), _d(times), t_start, t_end, dt, derivative,
                                max_out, _d(out), _d(tout), ctypes.byref(count)),
           "evaluate_range")
    n = min(count.value, max_out)
    return out[:n], tout[:n], count.value


def max_magnitude(N, coeffs, times, derivative):
    """orc_max_magnitude: computeMaximumOfMagnitude (linear_impl:455-487) on
    coeffs [S, D, N].  Returns dict(time, value, segment, n_candidates)."""
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    S, D, _ = coeffs.shape
    t, v = np.zeros(1), np.zeros(1)
    seg, nc = ctypes.c_int(), ctypes.c_int()
    L = lib()
    L.orc_max_magnitude.argtypes = [ctypes.c_int] * 3 + [_dp, _dp, ctypes.c_int, _dp, _dp, _ip, _ip]
    _check(L.orc_max_magnitude(N, D, S, _d(coeffs), _d(times), derivative, _d(t), _d(v),
                               ctypes.byref(seg), ctypes.byref(nc)), "max_magnitude")
    return dict(time=float(t[0]), value=float(v[0]), segment=seg.value, n_candidates=nc.value)


def magnitude_candidates(N, coeffs, times, derivative):
    """orc_magnitude_candidates: per segment of coeffs [S, D, N] the list
    (t, |p^(derivative)(t)|) of Segment::computeMinMaxMagnitudeCandidates
    (0, T, real roots in [0, T]).  Returns a list of S (times, values) arrays."""
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    S, D, _ = coeffs.shape
    cap = 2 * N + 2
    ct, cv = np.zeros((S, cap)), np.zeros((S, cap))
    nc = np.zeros(S, dtype=np.int32)
    L = lib()
    L.orc_magnitude_candidates.argtypes = [ctypes.c_int] * 3 + [_dp, _dp, ctypes.c_int,
                                                                ctypes.c_int, _dp, _dp, _ip]
    _check(L.orc_magnitude_candidates(N, D, S, _d(coeffs), _d(times), derivative, cap, _d(ct),
                                      _d(cv), nc.ctypes.data_as(_ip)), "magnitude_candidates")
    return [(ct[s, :min(nc[s], cap)].copy(), cv[s, :min(nc[s], cap)].copy()) for s in range(S)]


def poly_roots(inc):
    """orc_poly_roots: all complex roots (companion-matrix eigenvalues)."""
    inc = np.ascontiguousarray(inc, dtype=np.float64)
    re, im = np.zeros(len(inc)), np.zeros(len(inc))
    L = lib()
    L.orc_poly_roots.argtypes = [ctypes.c_int, _dp, _dp, _dp]
    n = L.orc_poly_roots(len(inc), _d(inc), _d(re), _d(im))
    _check(0 if n >= 0 else n, "poly_roots")
    return re[:n] + 1j * im[:n]


def soft_constraint_cost(N, coeffs, times, derivatives, limits, weight=100.0,
                         maximum_cost=1.0e12):
    """orc_soft_constraint_cost (nonlinear_impl:2735-2766).  Returns
    (cost, maxima)."""
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    S, D, _ = coeffs.shape
    der = np.ascontiguousarray(derivatives, dtype=np.int32)
    lim = np.ascontiguousarray(limits, dtype=np.float64)
    maxima = np.zeros(len(der))
    cost = np.zeros(1)
    L = lib()
    L.orc_soft_constraint_cost.argtypes = [ctypes.c_int] * 3 + [_dp, _dp, ctypes.c_int, _ip, _dp,
                                                                ctypes.c_double, ctypes.c_double,
                                                                _dp, _dp]
    _check(L.orc_soft_constraint_cost(N, D, S, _d(coeffs), _d(times), len(der),
                                      der.ctypes.data_as(_ip), _d(lim), weight, maximum_cost,
                                      _d(maxima), _d(cost)), "soft_constraint_cost")
    return float(cost[0]), maxima


def _soft_arrays(soft):
    der = np.ascontiguousarray([d for d, _ in soft] if soft else [0], dtype=np.int32)
    lim = np.ascontiguousarray([v for _, v in soft] if soft else [1.0], dtype=np.float64)
    return (len(soft) if soft else 0), der, lim


def free_cost(N, r, vertices, times, dp, mode=0, time_penalty=500.0, soft=None,
              soft_weight=100.0, soft_maximum_cost=1.0e12):
    """orc_free_cost: objectiveFunctionFreeConstraints (mode 0: J_d [+ soft],
    gradient of J_d) / objectiveFunctionTimeAndConstraints (mode 1).
    dp: D x n_free.  Returns (J, grad or None)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    dp = np.ascontiguousarray(dp, dtype=np.float64)
    grad = np.zeros(dp.shape)
    cost = np.zeros(1)
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_free_cost.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, ctypes.c_int, ctypes.c_double, ctypes.c_int, _ip, _dp,
        ctypes.c_double, ctypes.c_double, _dp, _dp]
    _check(L.orc_free_cost(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p), _d(vertices.vals),
                           _d(times), _d(dp), mode, time_penalty, ns, der.ctypes.data_as(_ip),
                           _d(lim), soft_weight, soft_maximum_cost, _d(cost), _d(grad)),
           "free_cost")
    return float(cost[0]), (grad if mode == 0 else None)


def free_optimize(N, r, vertices, times, dp0, max_evals, lower=None, upper=None, soft=None,
                  soft_weight=100.0, soft_maximum_cost=1.0e12):
    """orc_free_optimize: the mtg_free_optimize algorithm on the oracle.
    Returns (dp, J, evals)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    times = np.ascontiguousarray(times, dtype=np.float64)
    dp = np.ascontiguousarray(dp0, dtype=np.float64).copy()
    lo = None if lower is None else np.ascontiguousarray(lower, dtype=np.float64)
    hi = None if upper is None else np.ascontiguousarray(upper, dtype=np.float64)
    cost = np.zeros(1)
    evals = ctypes.c_int()
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_free_optimize.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, _dp, _dp, ctypes.c_int, _ip, _dp, ctypes.c_double,
        ctypes.c_double, ctypes.c_int, _dp, ctypes.POINTER(ctypes.c_int)]
    _check(L.orc_free_optimize(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                               _d(vertices.vals), _d(times), _d(dp),
                               None if lo is None else _d(lo), None if hi is None else _d(hi),
                               ns, der.ctypes.data_as(_ip), _d(lim), soft_weight,
                               soft_maximum_cost, max_evals, _d(cost), ctypes.byref(evals)),
           "free_optimize")
    return dp, float(cost[0]), evals.value


def time_free_optimize(N, r, vertices, times, dp0, max_evals, time_penalty=500.0, increment=0.1,
                       soft=None, soft_weight=100.0, soft_maximum_cost=1.0e12):
    """orc_time_free_optimize: the mtg_time_free_optimize algorithm on the
    oracle.  Returns (times, dp, J, evals)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    t = np.ascontiguousarray(times, dtype=np.float64).copy()
    dp = np.ascontiguousarray(dp0, dtype=np.float64).copy()
    cost = np.zeros(1)
    evals = ctypes.c_int()
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_time_free_optimize.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, _ip, _dp,
        ctypes.c_double, ctypes.c_double, ctypes.c_int, _dp, ctypes.POINTER(ctypes.c_int)]
    _check(L.orc_time_free_optimize(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                    _d(vertices.vals), _d(dp), _d(t), time_penalty, increment,
                                    ns, der.ctypes.data_as(_ip), _d(lim), soft_weight,
                                    soft_maximum_cost, max_evals, _d(cost), ctypes.byref(evals)),
           "time_free_optimize")
    return t, dp, float(cost[0]), evals.value


def time_free_optimize_sbplx(N, r, vertices, times, dp0, max_evals, time_penalty=500.0,
                             f_rel=0.05, f_abs=-1.0, step_rel=0.1, soft=None, soft_weight=100.0,
                             soft_maximum_cost=1.0e12):
    """orc_time_free_optimize_sbplx: optimizeTimeAndFreeConstraints with
    LN_SBPLX over [T; d_p].  Returns dict(times, dp, cost, evals, result,
    history [evals, S + D np])."""
    S, D, K = vertices.S, vertices.D, vertices.K
    t = np.ascontiguousarray(times, dtype=np.float64).copy()
    dp = np.ascontiguousarray(dp0, dtype=np.float64).copy()
    n = S + dp.size
    cost = np.zeros(1)
    evals = ctypes.c_int()
    result = ctypes.c_int()
    hist = np.zeros((max_evals, n))
    ns, der, lim = _soft_arrays(soft)
    L = lib()
    L.orc_time_free_optimize_sbplx.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int, _ip, _dp, ctypes.c_double,
        ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp,
        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), _dp]
    _check(L.orc_time_free_optimize_sbplx(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                          _d(vertices.vals), _d(dp), _d(t), time_penalty, ns,
                                          der.ctypes.data_as(_ip), _d(lim), soft_weight,
                                          soft_maximum_cost, max_evals, f_rel, f_abs, step_rel,
                                          _d(cost), ctypes.byref(evals), ctypes.byref(result),
                                          _d(hist)), "time_free_optimize_sbplx")
    return dict(times=t, dp=dp, cost=float(cost[0]), evals=evals.value, result=result.value,
                history=hist[:evals.value])


def collision_cost(N, r, vertices, times, dp, occupancy, params, box_side=20):
    """orc_collision_cost: getCostAndGradientCollision on a dense grid.
    occupancy: float32 [nz, ny, nx]; params: dict of map_resolution,
    min_bound[3], max_bound[3], epsilon, robot_radius, coll_pot_multiplier,
    coll_check_time_increment.  Returns (J, collision, grad_coeffs [S, D, N],
    grad_free [D, np])."""
    S, D, K = vertices.S, vertices.D, vertices.K
    occ = np.ascontiguousarray(occupancy, dtype=np.float32)
    nz, ny, nx = occ.shape
    prm = np.array([params["map_resolution"], *params["min_bound"], *params["max_bound"],
                    params["epsilon"], params["robot_radius"], params["coll_pot_multiplier"],
                    params["coll_check_time_increment"]], dtype=np.float64)
    dp = np.ascontiguousarray(dp, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    cost = np.zeros(1)
    coll = ctypes.c_int()
    gc = np.zeros((S, D, N))
    gf = np.zeros(dp.shape)
    L = lib()
    L.orc_collision_cost.argtypes = [ctypes.c_int] * 5 + [
        _u8p, _dp, _dp, _dp, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int,
        ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.POINTER(ctypes.c_int), _dp, _dp]
    _check(L.orc_collision_cost(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                                _d(vertices.vals), _d(times), _d(dp),
                                occ.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nx, ny, nz,
                                _d(prm), box_side, _d(cost), ctypes.byref(coll), _d(gc), _d(gf)),
           "collision_cost")
    return float(cost[0]), coll.value, gc, gf


# Defaults of NonlinearOptimizationParameters for the collision objectives
# (polynomial_optimization_nonlinear.h:46-84), the same keys as the product's
# COLL_DEFAULTS.
COLL_DEFAULTS = dict(map_resolution=0.0, min_bound=(0.0, 0.0, 0.0), max_bound=(0.0, 0.0, 0.0),
                     epsilon=0.5, robot_radius=0.5, coll_pot_multiplier=1.0,
                     coll_check_time_increment=0.1, box_side=20, w_d=0.1, w_c=10.0, w_t=1.0,
                     w_sc=1.0, is_collision_safe=True, is_coll_raise_first_iter=True,
                     add_coll_raise=0.0, simple_numgrad_time=False,
                     simple_numgrad_constraints=False, increment_time=0.1, soft=(),
                     soft_weight=100.0, soft_maximum_cost=1.0e12, f_rel=0.05, f_abs=-1.0,
                     x_rel=-1.0, x_abs=-1.0, lbfgs_memory=10)


def _coll_arrays(params):
    d = dict(COLL_DEFAULTS, **params)
    prm = np.array([d["map_resolution"], *d["min_bound"], *d["max_bound"], d["epsilon"],
                    d["robot_radius"], d["coll_pot_multiplier"], d["coll_check_time_increment"],
                    d["w_d"], d["w_c"], d["w_t"], d["w_sc"], d["add_coll_raise"],
                    d["increment_time"], d["soft_weight"], d["soft_maximum_cost"], d["f_rel"],
                    d["f_abs"], d["x_rel"], d["x_abs"]], dtype=np.float64)
    soft = list(d["soft"] or [])
    ip = np.array([d["box_side"], int(d["is_collision_safe"]), int(d["is_coll_raise_first_iter"]),
                   int(d["simple_numgrad_time"]), int(d["simple_numgrad_constraints"]), len(soft),
                   d["lbfgs_memory"]], dtype=np.int32)
    der = np.array([s[0] for s in soft] + [0], dtype=np.int32)
    lim = np.array([s[1] for s in soft] + [1.0], dtype=np.float64)
    return prm, ip, der, lim


_COLL_COMMON = [ctypes.c_int] * 5 + [_u8p, _dp, _dp, ctypes.c_int]


def coll_cost(N, r, vertices, times, mode, x, occupancy, params, raise_ref=0.0):
    """orc_coll_cost: objectiveFunctionFreeConstraintsAndCollision (mode 0,
    x = d_p flattened D x np) / ...AndCollisionAndTime (mode 1, x = [T; d_p])
    on a dense grid.  Returns (J, grad [nv], terms [4], collision)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    occ = np.ascontiguousarray(occupancy, dtype=np.float32)
    nz, ny, nx = occ.shape
    prm, ip, der, lim = _coll_arrays(params)
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    times = np.ascontiguousarray(times, dtype=np.float64)
    cost = np.zeros(1)
    grad = np.zeros(x.size)
    terms = np.zeros(4)
    coll = ctypes.c_int()
    L = lib()
    L.orc_coll_cost.argtypes = _COLL_COMMON + [
        _dp, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _ip,
        _ip, _dp, ctypes.c_double, _dp, _dp, _dp, ctypes.POINTER(ctypes.c_int)]
    _check(L.orc_coll_cost(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p), _d(vertices.vals),
                           _d(times), mode, _d(x),
                           occ.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nx, ny, nz,
                           _d(prm), ip.ctypes.data_as(_ip), der.ctypes.data_as(_ip), _d(lim),
                           float(raise_ref), _d(cost), _d(grad), _d(terms), ctypes.byref(coll)),
           "coll_cost")
    return float(cost[0]), grad, terms, coll.value


def bench_coll(N, r, vertices, times, occupancy, params, X0, max_evals, threads=1,
               seconds=2.0):
    """orc_bench_coll: CPU rate of orc_coll_optimize (mode 0) cycling over the
    starts X0 [B, nv].  Returns (optimisations, seconds)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    occ = np.ascontiguousarray(occupancy, dtype=np.float32)
    nz, ny, nx = occ.shape
    prm, ip, der, lim = _coll_arrays(params)
    X0 = np.ascontiguousarray(X0, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    units = ctypes.c_int64()
    sec = np.zeros(1)
    L = lib()
    L.orc_bench_coll.argtypes = [ctypes.c_int] * 5 + [_u8p, _dp, _dp] + [
        ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _ip, _ip,
        _dp, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
        ctypes.POINTER(ctypes.c_int64), _dp]
    _check(L.orc_bench_coll(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                            _d(vertices.vals), _d(times),
                            occ.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nx, ny, nz,
                            _d(prm), ip.ctypes.data_as(_ip), der.ctypes.data_as(_ip), _d(lim),
                            X0.shape[0], X0.shape[1], _d(X0), max_evals, threads, seconds,
                            ctypes.byref(units), _d(sec)), "bench_coll")
    return units.value, float(sec[0])


def coll_optimize(N, r, vertices, times, mode, x0, occupancy, params, max_evals, lower=None,
                  upper=None, initial_step=None):
    """orc_coll_optimize: the mtg_coll_optimize algorithm (projected L-BFGS)
    on the collision objective.  Returns (x, J, evals, result, terms)."""
    S, D, K = vertices.S, vertices.D, vertices.K
    occ = np.ascontiguousarray(occupancy, dtype=np.float32)
    nz, ny, nx = occ.shape
    prm, ip, der, lim = _coll_arrays(params)
    x = np.array(x0, dtype=np.float64).reshape(-1)
    times = np.ascontiguousarray(times, dtype=np.float64)
    opt = [None if a is None else np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
           for a in (lower, upper, initial_step)]
    cost = np.zeros(1)
    terms = np.zeros(4)
    ev, res = ctypes.c_int(), ctypes.c_int()
    L = lib()
    L.orc_coll_optimize.argtypes = _COLL_COMMON + [
        ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _ip, _ip,
        _dp, _dp, _dp, _dp, ctypes.c_int, _dp, _dp, ctypes.POINTER(ctypes.c_int),
        ctypes.POINTER(ctypes.c_int), _dp]
    _check(L.orc_coll_optimize(N, D, r, S, K, vertices.mask.ctypes.data_as(_u8p),
                               _d(vertices.vals), _d(times), mode,
                               occ.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nx, ny, nz,
                               _d(prm), ip.ctypes.data_as(_ip), der.ctypes.data_as(_ip),
                               _d(lim), *[None if a is None else _d(a) for a in opt],
                               max_evals, _d(x), _d(cost), ctypes.byref(ev), ctypes.byref(res),
                               _d(terms)),
           "coll_optimize")
    return x, float(cost[0]), ev.value, res.value, terms
