"""ctypes binding of libmtg_hip.so (include/mtg_hip.h).

The shared library is the product: every compute call goes to the gfx950
kernels.  There is no CPU fallback; loading fails loudly when the library is
missing or was built without a usable HIP device.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MTG_LIB_PATH selects a diagnostic build (tools/stamps.py); default in-tree.
LIB_PATH = os.environ.get("MTG_LIB_PATH", os.path.join(_HERE, "libmtg_hip.so"))

_dp = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_ip = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p


class CollisionParams(ctypes.Structure):
    """mtg_collision_params (include/mtg_hip.h)."""
    _fields_ = [("map_resolution", ctypes.c_double), ("min_bound", ctypes.c_double * 3),
                ("max_bound", ctypes.c_double * 3), ("epsilon", ctypes.c_double),
                ("robot_radius", ctypes.c_double), ("coll_pot_multiplier", ctypes.c_double),
                ("coll_check_time_increment", ctypes.c_double), ("box_side", ctypes.c_int)]


def make_collision_params(map_resolution, min_bound, max_bound, epsilon=0.5, robot_radius=0.5,
                          coll_pot_multiplier=1.0, coll_check_time_increment=0.1, box_side=20):
    """NonlinearOptimizationParameters' collision fields (defaults of
    polynomial_optimization_nonlinear.h:46-84; side 20 of :1797)."""
    return CollisionParams(map_resolution, (ctypes.c_double * 3)(*min_bound),
                           (ctypes.c_double * 3)(*max_bound), epsilon, robot_radius,
                           coll_pot_multiplier, coll_check_time_increment, box_side)


class CollObjectiveParams(ctypes.Structure):
    """mtg_coll_params (include/mtg_hip.h)."""
    _fields_ = [("coll", CollisionParams), ("w_d", ctypes.c_double), ("w_c", ctypes.c_double),
                ("w_t", ctypes.c_double), ("w_sc", ctypes.c_double),
                ("is_collision_safe", ctypes.c_int), ("is_coll_raise_first_iter", ctypes.c_int),
                ("add_coll_raise", ctypes.c_double), ("simple_numgrad_time", ctypes.c_int),
                ("simple_numgrad_constraints", ctypes.c_int), ("increment_time", ctypes.c_double),
                ("n_soft", ctypes.c_int), ("soft_derivative", ctypes.c_int * 8),
                ("soft_limit", ctypes.c_double * 8), ("soft_weight", ctypes.c_double),
                ("soft_maximum_cost", ctypes.c_double), ("f_rel", ctypes.c_double),
                ("f_abs", ctypes.c_double), ("x_rel", ctypes.c_double),
                ("x_abs", ctypes.c_double), ("lbfgs_memory", ctypes.c_int)]


# Defaults of NonlinearOptimizationParameters for the collision objectives
# (polynomial_optimization_nonlinear.h:46-84, cost_weights :163).
COLL_DEFAULTS = dict(map_resolution=0.0, min_bound=(0.0, 0.0, 0.0), max_bound=(0.0, 0.0, 0.0),
                     epsilon=0.5, robot_radius=0.5, coll_pot_multiplier=1.0,
                     coll_check_time_increment=0.1, box_side=20, w_d=0.1, w_c=10.0, w_t=1.0,
                     w_sc=1.0, is_collision_safe=True, is_coll_raise_first_iter=True,
                     add_coll_raise=0.0, simple_numgrad_time=False,
                     simple_numgrad_constraints=False, increment_time=0.1, soft=(),
                     soft_weight=100.0, soft_maximum_cost=1.0e12, f_rel=0.05, f_abs=-1.0,
                     x_rel=-1.0, x_abs=-1.0, lbfgs_memory=10)


def make_coll_params(**kw):
    """mtg_coll_params from COLL_DEFAULTS updated by `kw` (soft: list of
    (derivative, maximum_value) magnitude constraints)."""
    unknown = set(kw) - set(COLL_DEFAULTS)
    if unknown:
        raise MTGError(f"unknown collision-objective parameters {sorted(unknown)}")
    d = dict(COLL_DEFAULTS, **kw)
    soft = list(d["soft"] or [])
    if len(soft) > 8:
        raise MTGError("at most 8 soft constraints")
    p = CollObjectiveParams()
    p.coll = make_collision_params(d["map_resolution"], d["min_bound"], d["max_bound"],
                                   d["epsilon"], d["robot_radius"], d["coll_pot_multiplier"],
                                   d["coll_check_time_increment"], d["box_side"])
    for k in ("w_d", "w_c", "w_t", "w_sc", "add_coll_raise", "increment_time", "soft_weight",
              "soft_maximum_cost", "f_rel", "f_abs", "x_rel", "x_abs"):
        setattr(p, k, float(d[k]))
    for k in ("is_collision_safe", "is_coll_raise_first_iter", "simple_numgrad_time",
              "simple_numgrad_constraints", "lbfgs_memory"):
        setattr(p, k, int(d[k]))
    p.n_soft = len(soft)
    for i, (der, v) in enumerate(soft):
        p.soft_derivative[i] = int(der)
        p.soft_limit[i] = float(v)
    return p


class TimeParams(ctypes.Structure):
    """mtg_time_params (include/mtg_hip.h)."""
    _fields_ = [("time_penalty", ctypes.c_double), ("increment", ctypes.c_double),
                ("w_d", ctypes.c_double), ("w_t", ctypes.c_double),
                ("grad_mode", ctypes.c_int), ("n_soft", ctypes.c_int),
                ("soft_derivative", ctypes.c_int * 8), ("soft_limit", ctypes.c_double * 8),
                ("soft_weight", ctypes.c_double), ("soft_maximum_cost", ctypes.c_double),
                ("hard_constraints", ctypes.c_int), ("hard_tolerance", ctypes.c_double),
                ("optimizer", ctypes.c_int), ("f_rel", ctypes.c_double),
                ("f_abs", ctypes.c_double), ("initial_stepsize_rel", ctypes.c_double)]

OPTIMIZERS = {"fd": 0, "descent": 0, "sbplx": 1}


def make_time_params(time_penalty=500.0, increment=0.1, w_d=0.1, w_t=1.0, grad_mode=0,
                     soft=None, soft_weight=100.0, soft_maximum_cost=1.0e12, hard=False,
                     hard_tolerance=0.1, optimizer="fd", f_rel=0.05, f_abs=-1.0,
                     initial_stepsize_rel=0.1):
    """soft: list of (derivative, maximum_value) magnitude constraints
    (addMaximumMagnitudeConstraint), evaluated as soft costs, or with
    hard=True as hard inequalities max - value <= hard_tolerance
    (use_soft_constraints = false).  optimizer: "fd" (projected
    central-difference descent) or "sbplx" (LN_SBPLX, the reference's
    default) with NLopt's f_rel / f_abs and initial_stepsize_rel
    (NonlinearOptimizationParameters defaults)."""
    p = TimeParams(time_penalty, increment, w_d, w_t, grad_mode)
    soft = list(soft or [])
    if len(soft) > 8:
        raise MTGError("at most 8 soft constraints")
    p.n_soft = len(soft)
    for i, (d, v) in enumerate(soft):
        p.soft_derivative[i] = int(d)
        p.soft_limit[i] = float(v)
    p.soft_weight = soft_weight
    p.soft_maximum_cost = soft_maximum_cost
    p.hard_constraints = 1 if hard else 0
    p.hard_tolerance = hard_tolerance
    if optimizer not in OPTIMIZERS:
        raise MTGError(f"optimizer must be one of {sorted(OPTIMIZERS)}")
    p.optimizer = OPTIMIZERS[optimizer]
    p.f_rel = f_rel
    p.f_abs = f_abs
    p.initial_stepsize_rel = initial_stepsize_rel
    return p


# Symbol -> (restype, argtypes).  Must match include/mtg_hip.h exactly; the
# CPU test suite checks that every declared symbol is exported.
SIGNATURES = {
    "mtg_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "mtg_version": (ctypes.c_int, []),
    "mtg_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "mtg_ctx_destroy": (ctypes.c_int, [_vp]),
    "mtg_ctx_device": (ctypes.c_int, [_vp]),
    "mtg_plan_create": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, _u8p, ctypes.POINTER(_vp)]),
    "mtg_plan_destroy": (ctypes.c_int, [_vp]),
    "mtg_plan_counts": (ctypes.c_int, [_vp, _ip, _ip]),
    "mtg_plan_set_kernel": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mtg_free_cost": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp,
                                     ctypes.POINTER(TimeParams), ctypes.c_int, _vp, _vp, _vp,
                                     _vp]),
    "mtg_free_optimize": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp,
                                         ctypes.POINTER(TimeParams), ctypes.c_int, _vp, _vp,
                                         _vp, _vp]),
    "mtg_time_free_optimize": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp,
                                              ctypes.POINTER(TimeParams), ctypes.c_int, _vp,
                                              _vp, _vp, _vp]),
    "mtg_time_free_optimize_ex": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp,
                                                 ctypes.POINTER(TimeParams), ctypes.c_int, _vp,
                                                 _vp, _vp, _vp, _vp]),
    "mtg_plan_kernel": (ctypes.c_int, [_vp]),
    "mtg_collision_cost": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(CollisionParams), _vp, _vp, _vp, _vp,
                                          _vp]),
    "mtg_coll_workspace_bytes": (ctypes.c_int64, [_vp, ctypes.c_int64, ctypes.c_int,
                                                  ctypes.POINTER(CollObjectiveParams),
                                                  ctypes.c_int]),
    "mtg_coll_field_bytes": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "mtg_coll_field": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(CollisionParams), _vp, _vp]),
    "mtg_coll_cost": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, _vp, _vp,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                     ctypes.POINTER(CollObjectiveParams), _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "mtg_coll_optimize": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, _vp, _vp,
                                         _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         _vp, ctypes.POINTER(CollObjectiveParams), ctypes.c_int,
                                         _vp,
                                         _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "mtg_coll_optimize_trace": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, _vp,
                                               _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, _vp,
                                               ctypes.POINTER(CollObjectiveParams), ctypes.c_int,
                                               _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t,
                                               _vp]),
    "mtg_min_max_magnitude": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp, _vp,
                                             _vp, _vp, _vp, _vp, _vp]),
    "mtg_plan_kernel_for_batch": (ctypes.c_int, [_vp, ctypes.c_int64]),
    "mtg_linear_solve": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mtg_linear_solve_host": (ctypes.c_int, [_vp, ctypes.c_int64, _dp, _dp, _dp, _dp, _dp,
                                             _i32p]),
    "mtg_coeffs_from_constraints": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp,
                                                   _vp, _vp, _vp]),
    "mtg_segment_matrices": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                            _vp, _vp, _vp, _vp, _vp, _vp]),
    "mtg_time_cost": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, ctypes.POINTER(TimeParams),
                                     _vp, _vp, _vp, _vp]),
    "mtg_time_optimize": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp,
                                         ctypes.POINTER(TimeParams), ctypes.c_int, _vp, _vp,
                                         _vp, _vp, _vp]),
    "mtg_time_optimize_ex": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp,
                                            ctypes.POINTER(TimeParams), ctypes.c_int, _vp, _vp,
                                            _vp, _vp, _vp, _vp]),
    "mtg_tube_num_constraints": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "mtg_tube_residuals": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp]),
    "mtg_tube_solve": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, ctypes.c_double,
                                      ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mtg_tube_time_workspace_bytes": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int,
                                                       ctypes.c_int64,
                                                       ctypes.POINTER(TimeParams),
                                                       ctypes.c_int]),
    "mtg_tube_time_cost": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int64, _vp, _vp, _vp, _vp, _vp,
                                          ctypes.c_double, ctypes.c_int,
                                          ctypes.POINTER(TimeParams), _vp, _vp, _vp, _vp,
                                          ctypes.c_size_t, _vp]),
    "mtg_tube_time_optimize": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int64, _vp, _vp, _vp, _vp,
                                              ctypes.c_double, ctypes.c_int,
                                              ctypes.POINTER(TimeParams), ctypes.c_int, _vp,
                                              _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "mtg_tube_time_optimize_ex": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp,
                                                 _vp, ctypes.c_double, ctypes.c_int,
                                                 ctypes.POINTER(TimeParams), ctypes.c_int, _vp,
                                                 _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "mtg_select_local": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "mtg_select_workspace_bytes": (ctypes.c_int64, [_vp, ctypes.c_int64]),
    "mtg_linear_solve_select": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, _vp,
                                               ctypes.c_int64, ctypes.c_int, _vp, _vp,
                                               ctypes.c_size_t, _vp]),
    "mtg_select_global": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "mtg_linear_solve_select_prev": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp,
                                                     _vp, _vp, ctypes.c_int64, ctypes.c_int64,
                                                     ctypes.c_int, _vp, _vp]),
    "mtg_select_global_steps": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                _vp, _vp]),
    "mtg_sample_trajectories": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int64, _vp, _vp, ctypes.c_double,
                                               ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                               ctypes.c_int, _vp, _vp, _vp, _vp]),
    "mtg_max_magnitude": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                         _vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "mtg_magnitude_candidates": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int64, _vp, _vp, ctypes.c_int,
                                                ctypes.c_int, _vp, _vp, _vp, _vp]),
    "mtg_soft_constraint_cost": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int64, _vp, _vp, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int), _dp,
                                                ctypes.c_double, ctypes.c_double, _vp, _vp,
                                                _vp]),
    "mtg_generate_random_problems": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int64, ctypes.c_uint64,
                                                    ctypes.c_double, ctypes.c_double,
                                                    ctypes.c_double, _u8p, _dp, _dp, _dp]),
}

_lib = None


class MTGError(RuntimeError):
    pass


def lib():
    """Load libmtg_hip.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MTGError(
                f"{LIB_PATH} not found: build it with `python __graft_entry__.py build` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().mtg_status_string(rc).decode()
        raise MTGError(f"{what} failed: {msg} ({rc})")
    return rc
