"""GPU candidate lists of the magnitude extrema (mtg_magnitude_candidates):
Segment::computeMinMaxMagnitudeCandidates (segment.cpp:82-161) per segment,
the list computeMaximumOfMagnitude returns (linear_impl:455-487), against
the oracle's restatement (companion-matrix roots standing in for RPOLY,
pinned to numpy.roots in test_oracle.py).

The two root finders agree on simple real roots; a multiple root (the
rest-to-rest start and end vertices make f vanish to high order there) comes
out of an eigenvalue solver as a cluster whose members the reference's
|Im| > DBL_EPSILON test keeps or drops by rounding, while the Bernstein
search lists it once.  So the comparison is: endpoints exact, every device
root is a root of f, every simple oracle root is found by the device, the
values are |p^(k)| at the times, and the maximum over the list equals
mtg_max_magnitude's.
"""
import numpy as np
import pytest
from numpy.polynomial import polynomial as P

from helpers import standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _problems(oracle, N, D, S, seeds):
    vs = [standard_vertices(N, S, D, s) for s in seeds]
    times = np.stack([oracle.estimate_segment_times(v, 3.0, 5.0) for v in vs])
    coeffs = np.stack([oracle.linear_solve(N, N // 2 - 1, v, t)["coeffs"]
                       for v, t in zip(vs, times)])
    return coeffs, times


def _f(c, k):
    """Coefficients of f = sum_d p_d^(k) p_d^(k+1) (D > 1) or p^(k+1) (D = 1)."""
    if c.shape[0] == 1:
        return P.polyder(c[0], k + 1)
    f = np.zeros(1)
    for d in range(c.shape[0]):
        f = P.polyadd(f, P.polymul(P.polyder(c[d], k) if k else c[d], P.polyder(c[d], k + 1)))
    return f


def _mag(c, t, k):
    return np.sqrt(sum(P.polyval(t, P.polyder(c[d], k) if k else c[d]) ** 2
                       for d in range(c.shape[0])))


@pytest.mark.parametrize("N,D,S", [(10, 3, 10), (10, 1, 5), (8, 2, 4), (12, 3, 3), (6, 4, 6)])
def test_candidates_vs_oracle(ctx, dev, oracle, N, D, S):
    import mav_tube_trajectory_generation_amd as mtg
    seeds = list(range(900, 908))
    coeffs, times = _problems(oracle, N, D, S, seeds)
    cd, td = torch.from_numpy(coeffs).to(dev), torch.from_numpy(times).to(dev)
    for k in range(0, min(4, N - 2) + 1):
        out = mtg.magnitude_candidates(cd, td, k)
        mx = mtg.max_magnitude(cd, td, k)
        torch.cuda.synchronize()
        ct, cv, cn = (out[x].cpu().numpy() for x in ("time", "value", "count"))
        C = ct.shape[2]
        assert C == 2 * (N - k) - 1
        for b in range(len(seeds)):
            best = 0.0  # Extremum() = {0, 0, 0}; strict '<' (linear_impl:474)
            ref = oracle.magnitude_candidates(N, coeffs[b], times[b], k)
            for s in range(S):
                n = int(cn[b, s])
                T = times[b, s]
                c = coeffs[b, s]
                assert 2 <= n <= C
                t, v = ct[b, s, :n], cv[b, s, :n]
                assert t[0] == 0.0 and t[1] == T  # t_start, t_end first (polynomial.cpp:44-45)
                roots = t[2:]
                assert np.all(np.diff(roots) > 0) and np.all((roots > 0) & (roots < T))
                f = _f(c, k)
                scale = np.sum(np.abs(f) * np.maximum(T, 1.0) ** np.arange(len(f)))
                for r in roots:  # every device root is a root of f
                    assert abs(P.polyval(r, f)) <= 1e-9 * scale, (N, D, S, k, b, s, r)
                # every simple oracle root inside (0, T) is found
                fd = P.polyder(f)
                for r in ref[s][0][2:]:
                    if r <= 1e-9 * T or r >= T * (1 - 1e-9):
                        continue
                    if abs(P.polyval(r, fd)) * T < 1e-6 * scale:
                        continue  # multiple / near-multiple root
                    assert roots.size and np.min(np.abs(roots - r)) <= 1e-7 * T, \
                        (N, D, S, k, b, s, r, roots)
                # values are the magnitude at the times (to the rounding of the
                # Horner sums: near-zero magnitudes at rest vertices are noise)
                mscale = sum(np.sum(np.abs(P.polyder(c[d], k) if k else c[d]) *
                                    np.maximum(T, 1.0) ** np.arange(N - k)) for d in range(D))
                for tt, vv in zip(t, v):
                    m = _mag(c, tt, k)
                    assert abs(vv - m) <= 1e-9 * m + 1e-13 * mscale, (k, b, s, tt, vv, m)
                # ...and the reference's endpoints agree exactly in value
                assert abs(v[0] - ref[s][1][0]) <= 1e-12 * abs(v[0]) + 1e-14 * mscale
                for vv in v:
                    best = vv if best < vv else best
            last = _mag(coeffs[b, S - 1], times[b, S - 1], k)
            best = last if best < last else best
            assert abs(best - mx["value"][b].item()) <= 1e-12 * max(best, 1e-300), (k, b)


def test_candidates_overflow_and_bad_time(ctx, dev, oracle):
    """A list longer than max_candidates stores its head: count reports the
    full count (as the C ABI), stored the entries written; a negative or NaN
    segment time gives no candidates."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S = 10, 3, 4
    coeffs, times = _problems(oracle, N, D, S, [31, 32])
    full = mtg.magnitude_candidates(torch.from_numpy(coeffs).to(dev),
                                    torch.from_numpy(times).to(dev), 1)
    short = mtg.magnitude_candidates(torch.from_numpy(coeffs).to(dev),
                                     torch.from_numpy(times).to(dev), 1, max_candidates=3)
    torch.cuda.synchronize()
    n_full = full["count"].cpu().numpy()
    assert np.array_equal(full["found"].cpu().numpy(), n_full)
    assert np.array_equal(short["found"].cpu().numpy(), n_full)
    assert np.array_equal(short["count"].cpu().numpy(), n_full)  # unclamped, as the C ABI
    assert np.array_equal(short["stored"].cpu().numpy(), np.minimum(n_full, 3))
    assert np.array_equal(short["time"].cpu().numpy()[..., :2], full["time"].cpu().numpy()[..., :2])
    assert (n_full > 3).any()  # the cap was exercised
    bad = times.copy()
    bad[0, 1] = -1.0
    bad[1, 2] = np.nan
    out = mtg.magnitude_candidates(torch.from_numpy(coeffs).to(dev), torch.from_numpy(bad).to(dev),
                                   1)
    torch.cuda.synchronize()
    n = out["count"].cpu().numpy()
    assert n[0, 1] == 0 and n[1, 2] == 0 and n[0, 0] >= 2


def test_candidates_rejects_bad_arguments(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    c = torch.zeros((1, 2, 3, 10), dtype=torch.float64, device=dev)
    t = torch.ones((1, 2), dtype=torch.float64, device=dev)
    with pytest.raises(mtg.MTGError):
        mtg.magnitude_candidates(c, t, 1, max_candidates=1)
    with pytest.raises(mtg.MTGError):
        mtg.magnitude_candidates(c, t, 9)
