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
                                          ExtEmit* em = nullptr, int* nodes = nullptr,
                                          int* iters = nullptr) {
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
      if (nodes) ++*nodes;
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
        for (int it = 0; it < kExtRefineIters; ++it) {
          if (iters) ++*iters;
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
  // workgroup 0 (stamp slots 320 + lane, 384 + lane).
  int n_nodes = 0, n_iters = 0;
  int* pn = &n_nodes;
  int* pi = &n_iters;
#else
  int* pn = nullptr;
  int* pi = nullptr;
#endif
  for (int item = lane; item < S * parts; item += 64) {
    const int s = item >> log2parts, part = item & (parts - 1);
    double v = -1.0, t = 0.0, mv = 0.0, mt = 0.0;
    ext_segment_search<N, K>(coeffs + s * D * N, D, times[s], part, parts, log2parts, v, t, mv,
                             mt, lb, nullptr, pn, pi);
    best = fmax(best, v);
  }
#ifdef MTG_STAMPS
  if (blockIdx.x == 0) {
    atomicAdd(&g_mtg_stamps[320 + lane], static_cast<unsigned long long>(n_nodes));
    atomicAdd(&g_mtg_stamps[384 + lane], static_cast<unsigned long long>(n_iters));
  }
#endif
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) best = fmax(best, __shfl_xor(best, off, 64));
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

}  // namespace mtg
