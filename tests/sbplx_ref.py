"""An independent pure-Python restatement of NLopt's LN_SBPLX (Rowan's
Subplex with NLopt's bounded Nelder-Mead), used only to pin the oracle's
C++ restatement (oracle/orc_sbplx.cpp) evaluation for evaluation.

Same published algorithm and constants, same tie rules (simplex ordered by
(value, point index); the progress permutation a stable sort by decreasing
|dx|), written as a flat event loop rather than nested routines.  NLopt
itself is absent, so parity with it stays unpinned.
"""
import math

PSI, OMEGA, NSMIN, NSMAX = 0.25, 0.1, 2, 5
ALPHA, BETA, GAMMA, DELTA = 1.0, 0.5, 2.0, 0.5
FAILURE, SUCCESS, FTOL, XTOL, MAXEVAL = -1, 1, 3, 4, 5


class _Stop(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


def _close(a, b):
    return abs(a - b) <= 1e-13 * (abs(a) + abs(b))


def _pin(v, lo, hi):
    return lo if v < lo else (hi if v > hi else v)


def _reflect(c, scale, xold, lb, ub):
    new = [_pin(ci + scale * (ci - xi), l, u) for ci, xi, l, u in zip(c, xold, lb, ub)]
    same_c = all(_close(a, b) for a, b in zip(new, c))
    same_old = all(_close(a, b) for a, b in zip(new, xold))
    return new, not (same_c or same_old)


def test_fn(x):
    n = len(x)
    s = 0.0
    for i in range(n):
        yi = x[i] - 0.3 * (i + 1)
        yj = x[i + 1] - 0.3 * (i + 2) if i + 1 < n else 0.0
        s += (1.0 + i) * yi * yi + 0.5 * yi * yj + 0.1 * yi * yi * yi * yi
    return s


def sbplx(f, lb, ub, x0, xstep0, maxeval, ftol_rel, ftol_abs):
    """Returns (code, best x, best f, evaluation history)."""
    n = len(x0)
    # NLopt refuses a start outside the bounds before any evaluation
    # (NLOPT_INVALID_ARGS; optimizeTime returns nlopt::FAILURE)
    if any(lo > hi or x < lo or x > hi for x, lo, hi in zip(x0, lb, ub)):
        return FAILURE, list(x0), float("nan"), []
    st = {"x": list(x0), "minf": None, "nevals": 0, "hist": []}

    def evaluate(point):
        st["hist"].append(list(point))
        return f(point)

    def count(point_sub, val, sub_x):
        # NLopt's CHECK_EVAL inside the subspace solver
        st["nevals"] += 1
        if val <= st["minf"]:
            st["minf"] = val
            sub_x[:] = point_sub
        if maxeval > 0 and st["nevals"] >= maxeval:
            raise _Stop(MAXEVAL)

    def nm(perm, lo_b, hi_b, sx, sstep):
        """Nelder-Mead on the coordinates perm; sx in/out; returns fdiff."""
        m = len(perm)
        full = lambda s: [s[perm.index(k)] if k in perm else st["x"][k]  # noqa: E731
                          for k in range(n)]
        vals = [st["minf"]]
        pts = [list(sx)]
        fdiff = math.inf
        for i in range(m):
            pt = list(sx)
            pt[i] += sstep[i]
            if pt[i] > hi_b[i]:
                pt[i] = hi_b[i] if hi_b[i] - sx[i] > abs(sstep[i]) * 0.1 else sx[i] - abs(sstep[i])
            if pt[i] < lo_b[i]:
                if sx[i] - lo_b[i] > abs(sstep[i]) * 0.1:
                    pt[i] = lo_b[i]
                else:
                    pt[i] = sx[i] + abs(sstep[i])
                    if pt[i] > hi_b[i]:
                        far = hi_b[i] if hi_b[i] - sx[i] > sx[i] - lo_b[i] else lo_b[i]
                        pt[i] = 0.5 * (far + sx[i])
            if _close(pt[i], sx[i]):
                raise _Stop(FAILURE)
            v = evaluate(full(pt))
            pts.append(pt)
            vals.append(v)
            count(pt, v, sx)
        diam0 = 0.0
        while True:
            order = sorted(range(m + 1), key=lambda i: (vals[i], i))
            lo, hi = order[0], order[-1]
            pred = order[-2] if m > 0 else None  # an empty subspace stops below
            fdiff = vals[hi] - vals[lo]
            st["fdiff"] = fdiff
            if diam0 == 0.0:
                diam0 = sum(abs(a - b) for a, b in zip(pts[lo], pts[hi]))
            cen = [0.0] * m
            for i in range(m + 1):
                if i != hi:
                    for j in range(m):
                        cen[j] += pts[i][j]
            cen = [cj * (1.0 / m) for cj in cen]
            if sum(abs(a - b) for a, b in zip(pts[lo], pts[hi])) < PSI * diam0:
                return XTOL
            xr, ok = _reflect(cen, ALPHA, pts[hi], lo_b, hi_b)
            if not ok:
                return XTOL
            fr = evaluate(full(xr))
            count(xr, fr, sx)
            fh = vals[hi]
            if fr < vals[lo]:
                xe, ok = _reflect(cen, GAMMA, pts[hi], lo_b, hi_b)
                pts[hi] = xe
                if not ok:
                    return XTOL
                fe = evaluate(full(xe))
                count(xe, fe, sx)
                if fe >= fr:
                    pts[hi], vals[hi] = xr, fr
                else:
                    vals[hi] = fe
            elif fr < vals[pred]:
                pts[hi], vals[hi] = xr, fr
            else:
                xc, ok = _reflect(cen, -BETA if fh <= fr else BETA, pts[hi], lo_b, hi_b)
                if not ok:
                    return XTOL
                fc = evaluate(full(xc))
                count(xc, fc, sx)
                if fc < fr and fc < fh:
                    pts[hi], vals[hi] = xc, fc
                else:
                    for i in range(m + 1):
                        if i == lo:
                            continue
                        xs_, ok = _reflect(pts[lo], -DELTA, pts[i], lo_b, hi_b)
                        pts[i] = xs_
                        if not ok:
                            return XTOL
                        vals[i] = evaluate(full(xs_))
                        count(xs_, vals[i], sx)

    st["minf"] = evaluate(st["x"])
    st["nevals"] = 1
    if maxeval > 0 and maxeval <= 1:
        return MAXEVAL, st["x"], st["minf"], st["hist"]
    xstep = list(xstep0)
    dx = [0.0] * n
    try:
        while True:
            xprev = list(st["x"])
            perm = sorted(range(n), key=lambda k: -abs(dx[k]))  # stable
            normdx = sum(abs(d) for d in dx)
            # partition into subspaces (Rowan's goodness)
            parts = []
            i, normi = 0, 0.0
            while i + NSMIN < n:
                norm = normi + sum(abs(dx[perm[k]]) for k in range(i, i + NSMIN - 1))
                best, size = -math.inf, NSMIN
                for k in range(i + NSMIN - 1, min(i + NSMAX, n)):
                    norm += abs(dx[perm[k]])
                    rest = n - k - 1
                    if -(-rest // NSMAX) > rest // NSMIN:
                        continue
                    g = (norm / (k + 1) - (normdx - norm) / (n - (k + 1))) if k + 1 < n \
                        else normdx / n
                    if g > best:
                        best, size = g, k + 1 - i
                for k in range(i, i + size):
                    normi += abs(dx[perm[k]])
                parts.append(perm[i:i + size])
                # the subspace runs before the next one is chosen; the
                # choice only reads dx, so the order is unaffected
                i += size
            parts.append(perm[i:])
            fdiff_max = 0.0
            for sub in parts:
                sx = [st["x"][k] for k in sub]
                ss = [xstep[k] for k in sub]
                try:
                    code = nm(sub, [lb[k] for k in sub], [ub[k] for k in sub], sx, ss)
                finally:
                    for k, v in zip(sub, sx):
                        st["x"][k] = v
                fdiff_max = max(fdiff_max, st.get("fdiff", math.inf))
                if code != XTOL:
                    raise _Stop(code)
            a, b = st["minf"] + fdiff_max, st["minf"]
            if not math.isinf(a) and (abs(b - a) < ftol_abs or
                                      abs(b - a) < ftol_rel * (abs(b) + abs(a)) * 0.5 or
                                      (ftol_rel > 0 and a == b)):
                return FTOL, st["x"], st["minf"], st["hist"]
            dx = [xk - pk for xk, pk in zip(st["x"], xprev)]
            if len(parts) == 1:
                scale = PSI
            else:
                scale = sum(abs(d) for d in dx) / sum(abs(s) for s in xstep)
                scale = min(max(scale, OMEGA), 1.0 / OMEGA)
            xstep = [-(s * scale) if d == 0.0 else math.copysign(s * scale, d)
                     for s, d in zip(xstep, dx)]
    except _Stop as e:
        code = XTOL if e.code == FAILURE else e.code
        return code, st["x"], st["minf"], st["hist"]
