// mtg_extrema_device.h — device core of the magnitude-extremum search
// (computeMaximumOfMagnitude, linear_impl:455-487; see mtg_extrema.hip for
// the method), shared by the batched extremum kernel and the time-allocation
// kernels' soft-constraint objective (objectiveFunctionTime with
// use_soft_constraints, nonlinear_impl:907-913).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_internal.h"
#ifdef MTG_STAMPS
#include "mtg_device.h"  // g_mtg_stamps
#endif

namespace mtg {

constexpr int kExtParts = 8;       // dyadic parts per segment (power of 2)
constexpr int kExtMaxLevel = 30;   // node width 2^-30 of the segment: cluster
constexpr int kExtRefineIters = 80;

__host__ __device__ constexpr double ext_falling(int k, int i) {
  double p = 1.0;
  for (int m = 0; m < k; ++m) p *= static_cast<double>(i - m);
  return p;
}

__host__ __device__ constexpr double ext_binom(int n, int k) {
  double r = 1.0;
  for (int i = 1; i <= k; ++i) r = r * static_cast<double>(n - k + i) / static_cast<double>(i);
  return r;
}

// |p^(K)(t)|^2 over the D dimensions of one segment (Polynomial::evaluate,
// polynomial.h:135-149: Horner over base(K, i) c_i).
template <int N, int K>
__device__ inline double ext_mag2(const double* c, int D, double t) {
  double sq = 0.0;
#pragma unroll
  for (int d = 0; d < kMaxD; ++d) {
    if (d >= D) break;
    const double* cd = c + d * N;
    double v = ext_falling(K, N - 1) * cd[N - 1];
#pragma unroll
    for (int i = N - 2; i >= K; --i) v = fma(v, t, ext_falling(K, i) * cd[i]);
    sq = fma(v, v, sq);
  }
  return sq;
}

// Candidate list output of the search (kEmit): every candidate (t, |p^(K)|)
// in visiting order, t = 0, T, then the roots ascending; n counts all of
// them (entries past cap are not stored).  single: the candidates of a
// one-dimensional magnitude are the roots of p^(K+1) alone, as the
// reference takes them (Polynomial::computeMinMaxCandidates on the
// derivative, segment.cpp:123-129), not those of p^(K) p^(K+1).
// Diagnostic counters of one lane's search (STAMPS build): nodes visited,
// Laguerre iterations, the phase clock's last mark.
struct ExtStats {
  int nodes = 0, iters = 0, maxit = 0;
  unsigned long long mark = 0;
};

struct ExtEmit {
  double* t;
  double* v;
  int cap;
  int n;
  bool single;
};

// One lane's share of segment s: the endpoint candidates (part 0: t = 0,
// last part: t = T) and the real roots of f = sum_d p_d^(K) p_d^(K+1) in its
// dyadic part [part / 2^log2parts, (part + 1) / 2^log2parts) of the segment.
// c: the segment's D x N coefficients (LDS), T: its time.  Updates best_v
// (|p^(K)|^2) and best_t with strict '>' in candidate order; with kMin also
// min_v / min_t with strict '<' (the minimum of Trajectory::
// computeMinMaxMagnitude, trajectory.cpp:184-220; caller starts min_v at
// +inf).  lb: a value |p^(K)|^2 attains somewhere on the trajectory (0 if
// none is known); without kMin, nodes whose upper bound lies below it are
// pruned, which never drops the trajectory's maximum.
template <int N, int K, bool kMin = false, bool kEmit = false>
__device__ __attribute__((always_inline)) inline void ext_segment_search(const double* c, int D, double T, int part, int parts,
                                          int log2parts, double& best_v, double& best_t,
                                          double& min_v, double& min_t, double lb = 0.0,
                                          ExtEmit* em = nullptr, ExtStats* stats = nullptr) {
  static_assert(!kEmit || kMin, "the candidate list needs the exhaustive (kMin) search");
  auto emit = [&](double v, double t) {
    if constexpr (kEmit) {
      if (em->n < em->cap) {
        em->t[em->n] = t;
        em->v[em->n] = sqrt(v);
      }
      ++em->n;
    }
  };
  auto take = [&](double v, double t) {
    emit(v, t);
    if (v > best_v) {
      best_v = v;
      best_t = t;
    }
    if constexpr (kMin) {
      if (v < min_v) {
        min_v = v;
        min_t = t;
      }
    }
  };
  constexpr int ND = N - K;        // terms of p^(K)
  constexpr int NDD = ND - 1;      // terms of p^(K+1)
  constexpr int M = ND + NDD - 2;  // degree of f
  // Endpoint candidates first (the reference lists 0, 0, T, roots).
  if (part == 0) {
    best_v = ext_mag2<N, K>(c, D, 0.0);
    best_t = 0.0;
    emit(best_v, 0.0);
    if constexpr (kMin) {
      min_v = best_v;
      min_t = 0.0;
    }
  }
  if (part == parts - 1) take(ext_mag2<N, K>(c, D, T), T);
  // f(t) = sum_d conv(p_d^(K), p_d^(K+1)), then q(u) = f(T u) on [0, 1].
  double q[M + 1];
#pragma unroll
  for (int j = 0; j <= M; ++j) q[j] = 0.0;
#pragma unroll
  for (int d = 0; d < kMaxD; ++d) {
    if (d >= D) break;
    const double* cd = c + d * N;
    double dv[ND], ddv[NDD];
#pragma unroll
    for (int j = 0; j < ND; ++j) dv[j] = ext_falling(K, j + K) * cd[j + K];
    if constexpr (kEmit) {
      if (em->single) {  // f = p^(K+1)
#pragma unroll
        for (int j = 0; j < ND; ++j) dv[j] = j == 0 ? 1.0 : 0.0;
      }
    }
#pragma unroll
    for (int j = 0; j < NDD; ++j) ddv[j] = ext_falling(K + 1, j + K + 1) * cd[j + K + 1];
#pragma unroll
    for (int a = 0; a < ND; ++a)
#pragma unroll
      for (int e = 0; e < NDD; ++e) q[a + e] = fma(dv[a], ddv[e], q[a + e]);
  }
  {
    double tp = T;
#pragma unroll
    for (int j = 1; j <= M; ++j) {
      q[j] *= tp;
      tp *= T;
    }
  }
  // The lane's part [u0, u0 + w0] of [0, 1] in the local variable v in
  // [0, 1]: q(u0 + w0 v) by a Taylor shift (synthetic division) and an exact
  // power-of-two scaling.  The part's Bernstein coefficients then come from
  // one conversion instead of two de Casteljau splits of the segment's.
  const double w0 = ldexp(1.0, -log2parts);
  const double u0 = part * w0;
  if (part > 0) {
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = M - 1; j >= i; --j) q[j] = fma(u0, q[j + 1], q[j]);
  }
  if (log2parts > 0) {
    double wp = w0;
#pragma unroll
    for (int j = 1; j <= M; ++j) {
      q[j] *= wp;
      wp *= w0;
    }
  }
  // Bernstein coefficients on the part: beta_i = sum_{j<=i} C(i,j)/C(M,j)
  // q_j, normalised to max |beta| = 1.
  double beta[M + 1];
  double mx = 0.0;
#pragma unroll
  for (int i = 0; i <= M; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j <= i; ++j) acc = fma(ext_binom(i, j) / ext_binom(M, j), q[j], acc);
    beta[i] = acc;
    mx = fmax(mx, fabs(acc));
  }
#ifdef MTG_STAMPS
  if (stats) MTG_TACC(471, stats->mark);
#endif
  if (mx > 0.0) {
    const double inv = 1.0 / mx;
#pragma unroll
    for (int i = 0; i <= M; ++i) {
      beta[i] *= inv;
      q[i] *= inv;
    }
    // Depth-first walk of the dyadic tree under the part (local level 0;
    // global level = level + log2parts).  Bracket tolerances are the global
    // 1e-12 in local units.
    const double tol = ldexp(1.0e-12, log2parts);
    const double hw = T * w0 * mx;  // d t / d v times the normalisation
    const int max_level = kExtMaxLevel - log2parts;
    int level = 0, idx = 0;
    for (;;) {
      if (stats) ++stats->nodes;
      const double w = ldexp(1.0, -level);
      const double a = idx * w;
      const double e = a + w;
      // Node coefficients: left part of a split at e, then the right part
      // of that at a / e.
      double bb[M + 1];
#pragma unroll
      for (int i = 0; i <= M; ++i) bb[i] = beta[i];
      if (e < 1.0) {
#pragma unroll
        for (int r = 1; r <= M; ++r)
#pragma unroll
          for (int i = M; i >= r; --i) bb[i] = fma(e, bb[i] - bb[i - 1], bb[i - 1]);
      }
      if (a > 0.0) {
        const double u = a / e;
#pragma unroll
        for (int r = 1; r <= M; ++r)
#pragma unroll
          for (int i = 0; i <= M - r; ++i) bb[i] = fma(u, bb[i + 1] - bb[i], bb[i]);
      }
      // Prune (maximum only): g = |p^(K)|^2 has g' = 2 f, so on the node
      // g <= g(t_a) + 2 (t_e - t_a) max(0, max_i beta_i) mx (convex hull of
      // the Bernstein coefficients).  A node whose bound is below a value g
      // attains on the trajectory cannot hold the maximum; the 1e-12 margin
      // keeps rounding from pruning the node that does.
      bool pruned = false;
      if constexpr (!kMin) {
        double bmax = 0.0;
#pragma unroll
        for (int i = 0; i <= M; ++i) bmax = fmax(bmax, bb[i]);
        lb = fmax(lb, best_v);
        const double ta = fma(w0, a, u0) * T;
        const double ub = fma(2.0 * (e - a) * hw, bmax, ext_mag2<N, K>(c, D, ta));
        pruned = ub < lb * (1.0 - 1.0e-12);
      }
      // Sign variations (zeros skipped), first / last nonzero signs.
      int var = 0;
      double first = 0.0, last = 0.0;
#pragma unroll
      for (int i = 0; i <= M; ++i) {
        const double x = bb[i];
        const bool nz = x != 0.0;
        var += (nz && last != 0.0 && ((x > 0.0) != (last > 0.0))) ? 1 : 0;
        first = (first == 0.0) ? x : first;
        last = nz ? x : last;
      }
      // One sign change from - to + inside the node is a strict local minimum
      // of g, below g at the node's ends, so never the maximum: maximum-only
      // searches skip its refinement (a root exactly at the left end is
      // still taken below).
      bool local_min = false;
      if constexpr (!kMin) local_min = var == 1 && first < 0.0;
      if (pruned || local_min) var = 0;
      double root = -1.0;
      if (!pruned && bb[0] == 0.0 && (a > 0.0 || part > 0)) {  // root exactly at the node's left end
        const double ua = fma(w0, a, u0);
        take(ext_mag2<N, K>(c, D, ua * T), ua * T);
      }
      bool descend = false;
      if (var == 1) {
        // Laguerre's method safeguarded by the bracket (bisection when a
        // step leaves it); lo keeps the sign of q just right of a.  Laguerre
        // models the other roots as one cluster, which is what the
        // high-multiplicity roots at rest-to-rest vertices look like, so it
        // converges in a few steps where Newton crawls.  Stops at the
        // rounding floor of the Horner evaluation.
        double lo = a, hi = e, x = 0.5 * (a + e);
        const bool pos_lo = first > 0.0;
        int its = 0;  // this call's iterations (diagnostic counters)
        for (int it = 0; it < kExtRefineIters; ++it) {
          ++its;
          if (stats) ++stats->iters;
          double fx = q[M], d1 = 0.0, d2 = 0.0, ab = fabs(q[M]);
#pragma unroll
          for (int j = M - 1; j >= 0; --j) {
            d2 = fma(d2, x, d1);
            d1 = fma(d1, x, fx);
            fx = fma(fx, x, q[j]);
            ab = fma(ab, x, fabs(q[j]));
          }
          if (fabs(fx) <= 32.0 * 2.220446049250313e-16 * ab) break;
          if ((fx > 0.0) == pos_lo) lo = x; else hi = x;
          const double rf = 1.0 / fx;
          const double G = d1 * rf;
          const double H = G * G - 2.0 * d2 * rf;
          const double rad = fmax((M - 1) * (M * H - G * G), 0.0);
          const double sq = sqrt(rad);
          const double den = G >= 0.0 ? G + sq : G - sq;
          double xn = den != 0.0 ? x - M / den : 0.5 * (lo + hi);
          if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
          const bool done = fabs(xn - x) <= tol || hi - lo <= tol;
          x = xn;
          if (done) break;
        }
        if (stats) stats->maxit = stats->maxit > its ? stats->maxit : its;
        root = x;
      } else if (var > 1) {
        if (level >= max_level) root = 0.5 * (a + e);  // unresolved cluster
        else descend = true;
      }
      if (root >= 0.0) {
        const double ur = fma(w0, root, u0);
        take(ext_mag2<N, K>(c, D, ur * T), ur * T);
      }
      if (descend) {
        ++level;
        idx *= 2;
        continue;
      }
      while (level > 0 && (idx & 1)) {
        idx >>= 1;
        --level;
      }
      if (level == 0) break;
      ++idx;
    }
  }
#ifdef MTG_STAMPS
  if (stats) MTG_TACC(472, stats->mark);
#endif
}

// max_t |p^(K)(t)| over a whole trajectory by one wave (all 64 lanes call):
// coeffs S x D x N and times S in LDS; work items (segment, part) strided
// over the lanes.  Returns the maximum on every lane.
template <int N, int K>
__device__ __attribute__((always_inline)) inline double ext_trajectory_max_wave(const double* coeffs, const double* times,
                                                 int S, int D, int lane) {
  int parts = 8, log2parts = 3;
  while (parts > 1 && S * parts > 64) {
    parts >>= 1;
    --log2parts;
  }
#ifdef MTG_STAMPS
  ExtStats st_{};
  MTG_TACC(511, st_.mark);
#endif
  // Lower bound for the pruning: |p^(K)|^2 at every part's right end.
  double lb = 0.0;
  for (int item = lane; item < S * parts; item += 64) {
    const int s = item >> log2parts, part = item & (parts - 1);
    lb = fmax(lb, ext_mag2<N, K>(coeffs + s * D * N, D, ldexp(times[s] * (part + 1), -log2parts)));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lb = fmax(lb, __shfl_xor(lb, off, 64));
  double best = 0.0;
#ifdef MTG_STAMPS
  // Diagnostic build: per-lane node and Laguerre-iteration counts of
  // workgroup 0 (stamp slots 320 + lane, 384 + lane) and phase cycles of
  // lane 0 (470 bound, 471 setup, 472 tree walk, 473 reduction).
  MTG_TACC(470, st_.mark);
  ExtStats* pst = &st_;
#else
  ExtStats* pst = nullptr;
#endif
  for (int item = lane; item < S * parts; item += 64) {
    const int s = item >> log2parts, part = item & (parts - 1);
    double v = -1.0, t = 0.0, mv = 0.0, mt = 0.0;
    ext_segment_search<N, K>(coeffs + s * D * N, D, times[s], part, parts, log2parts, v, t, mv,
                             mt, lb, nullptr, pst);
    best = fmax(best, v);
  }
#ifdef MTG_STAMPS
  MTG_TACC(511, st_.mark);
  if (blockIdx.x == 0) {
    atomicAdd(&g_mtg_stamps[320 + lane], static_cast<unsigned long long>(st_.nodes));
    atomicAdd(&g_mtg_stamps[384 + lane], static_cast<unsigned long long>(st_.iters));
    atomicMax(&g_mtg_stamps[448 + lane], static_cast<unsigned long long>(st_.maxit));
  }
#endif
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) best = fmax(best, __shfl_xor(best, off, 64));
#ifdef MTG_STAMPS
  MTG_TACC(473, st_.mark);
#endif
  return sqrt(best);
}

// Runtime-derivative dispatch (POSITION..SNAP, nonlinear_impl:2697-2724).
template <int N>
__device__ __attribute__((always_inline)) inline double ext_trajectory_max_wave_k(int K, const double* coeffs,
                                                   const double* times, int S, int D, int lane) {
  switch (K) {
    case 0: return ext_trajectory_max_wave<N, 0>(coeffs, times, S, D, lane);
    case 1: return ext_trajectory_max_wave<N, 1>(coeffs, times, S, D, lane);
    case 2: return ext_trajectory_max_wave<N, 2>(coeffs, times, S, D, lane);
    case 3:
      if constexpr (N >= 5) return ext_trajectory_max_wave<N, 3>(coeffs, times, S, D, lane);
      return 0.0;
    case 4:
      if constexpr (N >= 6) return ext_trajectory_max_wave<N, 4>(coeffs, times, S, D, lane);
      return 0.0;
    default: return 0.0;
  }
}

// ---------------------------------------------------------------------------
// Soft-constraint maxima, value only (the time kernels' soft objective,
// evaluateMaximumMagnitudeAsSoftConstraint, nonlinear_impl:2735-2766): the
// maximum of |p^(K_c)| over the trajectory for every constraint c at once.
// The wave's lanes take (constraint, segment, part) items, so both of the
// usual two constraints share one pass instead of running one search each.
// K is per lane at run time: p^(K) is read from the segment's coefficients
// through a per-constraint table of falling factorials (zero past N-1-K), and
// every polynomial is held at the degree of KMIN, the smallest K of the
// constraints (the extra leading coefficients are zero).
//
// Only the value is needed, so a local maximum is refined by a safeguarded
// Newton iteration on f = sum_d p_d^(K) p_d^(K+1) from the crossing of the
// Bernstein control polygon, stopped once a step is below 1e-9 of the part:
// at a simple root of f, |p^(K)|^2 is flat, so the value is then exact to
// rounding (a t error e gives a value error of order e^2).
template <int N, int KMIN>
struct ExtSoft {
  static constexpr int NK = N - KMIN;    // terms of p^(K), zero-padded
  static constexpr int MF = 2 * NK - 3;  // degree of f

  // Coefficients of p_d^(K) on segment row c (D x N): a[j] = fk[j] c[j + K].
  __device__ static void deriv(const double* cd, const double* fk, int K, double (&a)[NK]) {
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int i = j + K < N ? j + K : N - 1;
      a[j] = fk[j] * cd[i];
    }
  }

  // |p^(K)(t)|^2.
  __device__ static double mag2(const double* c, const double* fk, int K, int D, double t) {
    double sq = 0.0;
#pragma unroll
    for (int d = 0; d < kMaxD; ++d) {
      if (d >= D) break;
      double a[NK];
      deriv(c + d * N, fk, K, a);
      double v = a[NK - 1];
#pragma unroll
      for (int j = NK - 2; j >= 0; --j) v = fma(v, t, a[j]);
      sq = fma(v, v, sq);
    }
    return sq;
  }

  // |p^(K)(0)|^2: the constant terms only.
  __device__ static double mag2_at0(const double* c, const double* fk, int K, int D) {
    double sq = 0.0;
#pragma unroll
    for (int d = 0; d < kMaxD; ++d) {
      if (d >= D) break;
      const double v = fk[0] * c[d * N + (K < N ? K : N - 1)];
      sq = fma(v, v, sq);
    }
    return sq;
  }

  // Bernstein coefficients of q on [0, 1]: beta_i = sum_j C(i, j) / C(MF, j)
  // q_j, the scaled q_j through the binomial transform as Pascal additions
  // (MF + 1 constants instead of (MF + 1)(MF + 2) / 2 ratios held in
  // registers).
  __device__ static void bernstein(double (&bb)[MF + 1]) {
#pragma unroll
    for (int j = 0; j <= MF; ++j) bb[j] *= 1.0 / ext_binom(MF, j);
#pragma unroll
    for (int k = 1; k <= MF; ++k)
#pragma unroll
      for (int i = MF; i >= k; --i) bb[i] += bb[i - 1];
  }

  // A node's Bernstein coefficients bb of f on [a, e] (part coordinate u):
  // pruned (g <= g(t_a) + 2 (t_e - t_a) max(0, max_i bb_i) mx cannot reach
  // lb), the sign variations (zeros skipped), the first nonzero sign, and the
  // control polygon's first + to - step (its index ci and coefficients b0, b1).
  struct Scan {
    bool pruned;
    int var, ci;
    double first, b0, b1;
  };
  __device__ static Scan scan(const double (&bb)[MF + 1], double a, double e, double ga, double hw,
                              double lb) {
    Scan r;
    double bmax = 0.0;
#pragma unroll
    for (int i = 0; i <= MF; ++i) bmax = fmax(bmax, bb[i]);
    r.pruned = fma(2.0 * (e - a) * hw, bmax, ga) < lb * (1.0 - 1.0e-12);
    int var = 0;
    double first = 0.0, last = 0.0;
    bool found = false;
    int ci = 0;  // an int select: no double constants held in registers
    double b0 = 1.0, b1 = -1.0;
#pragma unroll
    for (int i = 0; i <= MF; ++i) {
      const double x = bb[i];
      const bool nz = x != 0.0;
      var += (nz && last != 0.0 && ((x > 0.0) != (last > 0.0))) ? 1 : 0;
      first = (first == 0.0) ? x : first;
      last = nz ? x : last;
      if (i < MF) {
        const bool cross = !found && x > 0.0 && !(bb[i + 1] > 0.0);
        ci = cross ? i : ci;
        b0 = cross ? x : b0;
        b1 = cross ? bb[i + 1] : b1;
        found = found || cross;
      }
    }
    r.var = var;
    r.first = first;
    r.ci = ci;
    r.b0 = b0;
    r.b1 = b1;
    return r;
  }

  // The local maximum of g on a node [a, e] with one + to - sign change of
  // f: Laguerre's method (the actual degree of f for this lane's K) on q
  // (f in the part coordinate), started at the control polygon's zero
  // crossing and safeguarded by the bracket, with approximate reciprocals
  // and square root: cubic convergence from the polygon start, and the
  // bracket keeps every step valid.  Stops at the rounding floor of the
  // Horner sum or once a step is below kTol of the part: the error is then
  // of order kTol^3, and the value's error of order its square times the
  // part's width (below rounding).  Returns g there.
  __device__ static double refine(const double (&q)[MF + 1], const double* c, const double* fk,
                                  int K, int D, double T, double w0, double u0, double a, double e,
                                  const Scan& sc, ExtStats* stats) {
    const double dn = sc.b0 - sc.b1;
    const double r0 = __builtin_amdgcn_rcp(dn);
    const double fr = sc.b0 * fma(r0, fma(-dn, r0, 1.0), r0);
    int ci = sc.ci;
    __asm__ volatile("" : "+v"(ci));  // converted here, not as a select chain of doubles
    const double x0 = fma(e - a, (static_cast<double>(ci) + fr) * (1.0 / MF), a);
    constexpr double kTol = 1.0e-7;
    const double nd = static_cast<double>(2 * (N - K) - 3);
    double lo = a, hi = e, x = x0;
    int its = 0;
    for (int it = 0; it < 64; ++it) {
      ++its;
      if (stats) ++stats->iters;
      double fx = q[MF], d1 = 0.0, d2 = 0.0, ab = fabs(q[MF]);
#pragma unroll
      for (int j = MF - 1; j >= 0; --j) {
        d2 = fma(d2, x, d1);
        d1 = fma(d1, x, fx);
        fx = fma(fx, x, q[j]);
        ab = fma(ab, x, fabs(q[j]));
      }
      if (fabs(fx) <= 32.0 * 2.220446049250313e-16 * ab) break;
      if (fx > 0.0) lo = x; else hi = x;
      const double s0 = __builtin_amdgcn_rcp(fx);
      const double rf = fma(s0, fma(-fx, s0, 1.0), s0);
      const double G = d1 * rf;
      const double H = G * G - 2.0 * d2 * rf;
      const double rad = fmax((nd - 1.0) * (nd * H - G * G), 0.0);
      const double sq = __builtin_amdgcn_sqrt(rad);
      const double den = G >= 0.0 ? G + sq : G - sq;
      const double t0 = __builtin_amdgcn_rcp(den);
      const double rden = fma(t0, fma(-den, t0, 1.0), t0);
      double xn = den != 0.0 ? fma(-nd, rden, x) : 0.5 * (lo + hi);
      if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
      const bool done = fabs(xn - x) <= kTol || hi - lo <= kTol;
      x = xn;
      if (done) break;
    }
    if (stats) stats->maxit = stats->maxit > its ? stats->maxit : its;
    return mag2(c, fk, K, D, fma(w0, x, u0) * T);
  }

  // Largest |p^(K)|^2 on part p of P of a segment (coefficients c, time T)
  // that can matter: the part's end values gl, gr and the local maxima
  // inside it whose bound reaches lb, a value attained on the trajectory
  // (nodes bounded below it are pruned; a 1e-12 margin keeps rounding from
  // pruning the node that holds the maximum).  At most two coefficient
  // arrays are live at any point (q and one node's), which keeps the time
  // kernels that inline the search at two waves per SIMD.
  __device__ static double part_max(const double* c, const double* fk, int K, int D, double T,
                                    int p, int P, double gl, double gr, double lb,
                                    ExtStats* stats = nullptr) {
    double best = fmax(gl, gr);
#ifdef MTG_STAMPS
    unsigned long long m0_ = 0;
    MTG_TACC(511, m0_);
#endif
    double q[MF + 1];
#pragma unroll
    for (int j = 0; j <= MF; ++j) q[j] = 0.0;
#pragma unroll
    for (int d = 0; d < kMaxD; ++d) {
      if (d >= D) break;
      double a[NK];
      deriv(c + d * N, fk, K, a);
#pragma unroll
      for (int i = 0; i < NK; ++i)
#pragma unroll
        for (int e = 0; e + 1 < NK; ++e) q[i + e] = fma(a[i], (e + 1) * a[e + 1], q[i + e]);
    }
    // q(u) = f(T (u0 + w0 u)) on the part, u in [0, 1].  (w0 opaque: its
    // powers below would otherwise be hoisted out of every enclosing loop
    // and held in 28 registers.)
    double w0 = 1.0 / P;
    __asm__ volatile("" : "+v"(w0));
    const double u0 = p * w0;
    {
      double tp = T;
#pragma unroll
      for (int j = 1; j <= MF; ++j) {
        q[j] *= tp;
        tp *= T;
      }
    }
    if (p > 0) {
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = MF - 1; j >= i; --j) q[j] = fma(u0, q[j + 1], q[j]);
    }
    if (P > 1) {
      double wp = w0;
#pragma unroll
      for (int j = 1; j <= MF; ++j) {
        q[j] *= wp;
        wp *= w0;
      }
    }
    double beta[MF + 1];
#pragma unroll
    for (int j = 0; j <= MF; ++j) beta[j] = q[j];
    bernstein(beta);
    double mx = 0.0;
#pragma unroll
    for (int i = 0; i <= MF; ++i) mx = fmax(mx, fabs(beta[i]));
    if (!(mx > 0.0)) return best;  // f = 0: g constant on the part
    const double inv = 1.0 / mx;
#pragma unroll
    for (int i = 0; i <= MF; ++i) {
      beta[i] *= inv;
      q[i] *= inv;
    }
    const double hw = T * w0 * mx;  // dt / du times the normalisation
#ifdef MTG_STAMPS
    MTG_TACC(471, m0_);  // setup of the part (lane 0)
#endif
    // Root node [0, 1]: g(0) of the part is gl, already in best.
    if (stats) ++stats->nodes;
    const Scan rs = scan(beta, 0.0, 1.0, gl, hw, lb);
#ifdef MTG_STAMPS
    MTG_TACC(474, m0_);  // node: bound, sign scan
#endif
    // One sign change from + to - is a local maximum of g; from - to + a
    // local minimum, never the maximum.
    if (!rs.pruned && rs.var == 1 && rs.first > 0.0)
      best = fmax(best, refine(q, c, fk, K, D, T, w0, u0, 0.0, 1.0, rs, stats));
#ifdef MTG_STAMPS
    MTG_TACC(476, m0_);  // refinement + value
#endif
    if (rs.pruned || rs.var <= 1) return best;
    // Descent (rare): a node's coefficients come from q (Taylor shift to a,
    // scale by its width, Bernstein conversion), so only q and one node's
    // coefficients are live.
    int level = 1, idx = 0;
    for (;;) {
      // Keeps mag2's coefficient reads (LDS) in the loop rather than hoisted
      // into registers.
      __asm__ volatile("" ::: "memory");
      if (stats) ++stats->nodes;
      const double w = ldexp(1.0, -level);
      const double a = idx * w;
      const double e = a + w;
      double bb[MF + 1];
#pragma unroll
      for (int i = 0; i <= MF; ++i) bb[i] = q[i];
      if (a > 0.0) {
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int j = MF - 1; j >= i; --j) bb[j] = fma(a, bb[j + 1], bb[j]);
      }
      {
        double wp = w;
#pragma unroll
        for (int j = 1; j <= MF; ++j) {
          bb[j] *= wp;
          wp *= w;
        }
      }
      bernstein(bb);
      const double ga = mag2(c, fk, K, D, fma(w0, a, u0) * T);
      const Scan sc = scan(bb, a, e, ga, hw, lb);
      if (!sc.pruned && bb[0] == 0.0 && (a > 0.0 || p > 0)) best = fmax(best, ga);
      if (!sc.pruned && sc.var == 1 && sc.first > 0.0)
        best = fmax(best, refine(q, c, fk, K, D, T, w0, u0, a, e, sc, stats));
      if (!sc.pruned && sc.var > 1) {
        if (level >= kExtMaxLevel) {
          best = fmax(best, mag2(c, fk, K, D, fma(w0, 0.5 * (a + e), u0) * T));
        } else {
          ++level;
          idx *= 2;
          continue;
        }
      }
      while (level > 0 && (idx & 1)) {
        idx >>= 1;
        --level;
      }
      if (level == 0) break;
      ++idx;
    }
    return best;
  }
};

// Maxima of |p^(K_c)| over the trajectory for the nc soft constraints (all
// 64 lanes call; one wave per workgroup).  coeffs S x D x N and times S in
// LDS; scratch (LDS) holds nc * N + 2 * nc doubles: the falling-factorial
// rows and per-constraint bounds and maxima.  On return out[c] (LDS, every
// lane) is max |p^(K_c)|.  Ks: the constraints' derivative orders (0..4),
// indexed with compile-time indices only.
template <int N, int KMIN>
__device__ __attribute__((always_inline)) inline void ext_soft_maxima_wave(
    const double* coeffs, const double* times, int S, int D, int lane, int nc,
    const int (&Ks)[kMaxSoftConstraints], double* scratch, double* out) {
  using X = ExtSoft<N, KMIN>;
#ifdef MTG_STAMPS
  unsigned long long mark_ = 0;
  MTG_TACC(511, mark_);
#endif
  double* fall = scratch;            // nc x N
  double* lbv = scratch + nc * N;    // nc bounds (bit patterns of non-negative doubles)
  auto Kof = [&](int ci) {
    int K = 0;
#pragma unroll
    for (int cc = 0; cc < kMaxSoftConstraints; ++cc) K = cc == ci ? Ks[cc] : K;
    return K;
  };
  for (int i = lane; i < nc * N; i += 64) {
    const int ci = i / N, j = i % N, K = Kof(ci);
    double f = 0.0;
    if (j + K < N) {
      f = 1.0;
      for (int m = 0; m < K; ++m) f *= static_cast<double>(j + K - m);
    }
    fall[i] = f;
  }
  for (int i = lane; i < 2 * nc; i += 64) (i < nc ? lbv : out)[i < nc ? i : i - nc] = 0.0;
  __syncthreads();
  const int per = nc * S;
  int P = 64 / per;
  P = P < 1 ? 1 : (P > kExtParts ? kExtParts : P);
  const int items = per * P;
  for (int base = 0; base < items; base += 64) {
    const int item = base + lane;
    const bool act = item < items;
    const int it = act ? item : 0;
    const int ci = it / (S * P), s = (it / P) % S, p = it % P;
    const int K = Kof(ci);
    const double* c = coeffs + s * D * N;
    const double* fk = fall + ci * N;
    const double T = times[s];
    const double ta = T * p / P, te = p == P - 1 ? T : T * (p + 1) / P;
    // g at the part's right end; at its left end: the constant terms at a
    // segment start, else the previous item's right end (the same
    // polynomial at the same t, computed by lane - 1 of this round).
    const double gr = X::mag2(c, fk, K, D, te);
    double gl = __shfl(gr, (lane + 63) & 63, 64);
    if (p == 0) gl = X::mag2_at0(c, fk, K, D);
    else if (lane == 0) gl = X::mag2(c, fk, K, D, ta);
    if (act)
      atomicMax(reinterpret_cast<unsigned long long*>(lbv + ci),
                static_cast<unsigned long long>(__double_as_longlong(fmax(gl, gr))));
    __syncthreads();
#ifdef MTG_STAMPS
    MTG_TACC(470, mark_);  // tables + part-end values + bounds
#endif
    if (act) {
      const double lb = lbv[ci];
#ifdef MTG_STAMPS
      ExtStats es{};
      const double m = X::part_max(c, fk, K, D, T, p, P, gl, gr, lb, &es);
      if (blockIdx.x == 0) {
        atomicAdd(&g_mtg_stamps[320 + lane], static_cast<unsigned long long>(es.nodes));
        atomicAdd(&g_mtg_stamps[384 + lane], static_cast<unsigned long long>(es.iters));
        atomicMax(&g_mtg_stamps[256 + lane], static_cast<unsigned long long>(es.maxit));
      }
#else
      const double m = X::part_max(c, fk, K, D, T, p, P, gl, gr, lb);
#endif
      atomicMax(reinterpret_cast<unsigned long long*>(out + ci),
                static_cast<unsigned long long>(__double_as_longlong(m)));
    }
#ifdef MTG_STAMPS
    MTG_TACC(472, mark_);  // part searches
#endif
    __syncthreads();
  }
  for (int i = lane; i < nc; i += 64) out[i] = sqrt(out[i]);
  __syncthreads();
#ifdef MTG_STAMPS
  MTG_TACC(473, mark_);  // results
#endif
}

// Runtime KMIN dispatch.
template <int N>
__device__ __attribute__((always_inline)) inline void ext_soft_maxima_wave_k(
    int kmin, const double* coeffs, const double* times, int S, int D, int lane, int nc,
    const int (&Ks)[kMaxSoftConstraints], double* scratch, double* out) {
  switch (kmin) {
    case 0: ext_soft_maxima_wave<N, 0>(coeffs, times, S, D, lane, nc, Ks, scratch, out); break;
    case 1: ext_soft_maxima_wave<N, 1>(coeffs, times, S, D, lane, nc, Ks, scratch, out); break;
    case 2: ext_soft_maxima_wave<N, 2>(coeffs, times, S, D, lane, nc, Ks, scratch, out); break;
    case 3:
      if constexpr (N >= 5) ext_soft_maxima_wave<N, 3>(coeffs, times, S, D, lane, nc, Ks, scratch, out);
      break;
    default:
      if constexpr (N >= 6) ext_soft_maxima_wave<N, 4>(coeffs, times, S, D, lane, nc, Ks, scratch, out);
      break;
  }
}

}  // namespace mtg
