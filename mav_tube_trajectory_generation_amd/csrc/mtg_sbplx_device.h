// mtg_sbplx_device.h — the reference's default time optimiser on the device:
// NLopt's LN_SBPLX (Rowan's Subplex with NLopt's bounded Nelder-Mead as the
// subspace solver), NonlinearOptimizationParameters::algorithm = LN_SBPLX
// (polynomial_optimization_nonlinear.h:61), configured at
// impl/polynomial_optimization_nonlinear_impl.h:95-101 (ftol_rel = f_rel,
// ftol_abs = f_abs, maxeval = max_iterations) and driven by optimizeTime
// (:332-397: initial step initial_stepsize_rel T0, bounds [0.1, 2 T0]).
//
// The time kernels (mtg_time_std.hip, mtg_kernels.hip), the free-derivative
// and time kernel (mtg_free.hip) and the tube-QCQP time optimiser
// (mtg_tube_time.hip) evaluate the objective at one call site in a loop; this
// machine decides the next point.  Its state (state_bytes(n): a fixed part
// plus six n-vectors and the permutation) lives in LDS, or in the caller's
// global workspace for the tube optimiser, and one lane advances it:
// init() / init_box() set the first point (the start), resume(f) takes the
// value of the point it asked for and writes the next one into T (or sets
// done).  The control flow is NLopt's
// (sbplx.c, nldrmd.c) unrolled into resume states; the CPU restatement it is
// checked against evaluation for evaluation is oracle/orc_sbplx.cpp
// (tests/test_time_sbplx_gpu.py).  Tie rules as the oracle: simplex order
// (value, point index), progress permutation a stable sort by decreasing
// |dx|.  The x tolerances are not restated (the reference disables them).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtg {
namespace sbplx {

constexpr int kNsMin = 2, kNsMax = 5;
constexpr double kPsi = 0.25, kOmega = 0.1;
constexpr double kAlpha = 1.0, kBeta = 0.5, kGamma = 2.0, kDelta = 0.5;
// nlopt_result codes
constexpr int kFailure = -1, kFtol = 3, kXtol = 4, kMaxEval = 5;

// The fixed part of the state; the n-sized arrays follow it (state_bytes(n)):
// x, xprev, dx, xstep, lb, ub (n doubles each), then the permutation p (n
// ints).  The subspace solver's arrays are fixed (ns <= kNsMax).
struct State {
  double pts[kNsMax + 1][kNsMax + 1];  // simplex: value, then the point
  double xs[kNsMax], lbs[kNsMax], ubs[kNsMax], sstep[kNsMax], c[kNsMax], xcur[kNsMax];
  double minf, fdiff, fdiff_max, normi, normdx, init_diam, fr, ftol_rel, ftol_abs;
  int n, maxeval, nevals, pc, result, done, i, is, ns, nsubs, k, lo, hi, last;
};
constexpr size_t kHdrBytes = (sizeof(State) + 15) / 16 * 16;
// Bytes of the state of an n-variable problem (16-byte multiple).
__host__ __device__ constexpr size_t state_bytes(int n) {
  return kHdrBytes + ((sizeof(double) * 6 + sizeof(int)) * static_cast<size_t>(n) + 15) / 16 * 16;
}
// Array k (0 x, 1 xprev, 2 dx, 3 xstep, 4 lb, 5 ub) of the state.
__device__ inline double* arr(State* s, int k) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(s) + kHdrBytes) + k * s->n;
}
__device__ inline const double* arr(const State* s, int k) {
  return reinterpret_cast<const double*>(reinterpret_cast<const char*>(s) + kHdrBytes) +
         k * s->n;
}
// NLopt's x: the best point (valid once done).
__device__ inline const double* best_x(const State* s) { return arr(s, 0); }

enum Pc {
  kFirst, kOuter, kSubsel, kNmInit, kNmInitGot, kNmIter, kNmReflGot, kNmExpGot, kNmConGot,
  kNmShrink, kNmShrGot
};

__device__ inline bool close_to(double a, double b) {
  return fabs(a - b) <= 1e-13 * (fabs(a) + fabs(b));
}

// xnew = c + scale (c - xold) pinned to [lb, ub]; false if it coincides
// with c or xold (nldrmd's reflectpt).  xnew may alias xold.
__device__ inline bool reflect(int n, double* xnew, const double* c, double scale,
                               const double* xold, const double* lb, const double* ub) {
  bool equalc = true, equalold = true;
  for (int i = 0; i < n; ++i) {
    double v = c[i] + scale * (c[i] - xold[i]);
    v = v < lb[i] ? lb[i] : v;
    v = v > ub[i] ? ub[i] : v;
    equalc = equalc && close_to(v, c[i]);
    equalold = equalold && close_to(v, xold[i]);
    xnew[i] = v;
  }
  return !(equalc || equalold);
}

// The machine (lane 0 only; the caller synchronises the workgroup after
// each call before T or done are read).
struct Machine {
  State* s;

  __device__ double* x() { return arr(s, 0); }
  __device__ double* xprev() { return arr(s, 1); }
  __device__ double* dx() { return arr(s, 2); }
  __device__ double* xstep() { return arr(s, 3); }
  __device__ double* lb() { return arr(s, 4); }
  __device__ double* ub() { return arr(s, 5); }
  __device__ int* p() { return reinterpret_cast<int*>(arr(s, 6)); }

  // Start from the times in T (S values): lb 0.1, ub 2 T0, steps
  // step_rel T0 (optimizeTime, nonlinear_impl:343-358, 370-378).
  __device__ void init(int n, const double* T, double step_rel, int maxeval, double ftol_rel,
                       double ftol_abs) {
    s->n = n;
    for (int i = 0; i < n; ++i) {
      x()[i] = T[i];
      lb()[i] = 0.1;  // kOptimizationTimeLowerBound
      ub()[i] = 2.0 * T[i];
      xstep()[i] = step_rel * T[i];
    }
    start(maxeval, ftol_rel, ftol_abs);
  }
  // Start from x0 with bounds [lb, ub] and initial steps (each n values; the
  // caller's arrays may be the ones the kernel evaluates at).
  __device__ void init_box(int n, const double* x0, const double* lo, const double* hi,
                           const double* step, int maxeval, double ftol_rel, double ftol_abs) {
    s->n = n;
    for (int i = 0; i < n; ++i) {
      x()[i] = x0[i];
      lb()[i] = lo[i];
      ub()[i] = hi[i];
      xstep()[i] = step[i];
    }
    start(maxeval, ftol_rel, ftol_abs);
  }
  // Common tail of init / init_box.  NLopt refuses a start outside its
  // bounds (or lb > ub) before the first evaluation (nlopt_optimize:
  // NLOPT_INVALID_ARGS, which nlopt::opt::optimize throws and optimizeTime
  // turns into nlopt::FAILURE, nonlinear_impl:389-394), and a zero initial
  // step (nlopt_set_initial_step, thrown at set_initial_step, :376 / :682):
  // the machine is then done at once with result kFailure, no evaluation,
  // x = x0, minf NaN.  The caller checks `done` before its first evaluation.
  // start() can also be called directly after the caller has filled n, x,
  // lb, ub and xstep (e.g. by all lanes of a wave).
  __device__ void start(int maxeval, double ftol_rel, double ftol_abs) {
    const int n = s->n;
    s->maxeval = maxeval;
    s->ftol_rel = ftol_rel;
    s->ftol_abs = ftol_abs;
    bool ok = true;
    for (int i = 0; i < n; ++i) {
      dx()[i] = 0.0;
      ok = ok && !(lb()[i] > ub()[i] || x()[i] < lb()[i] || x()[i] > ub()[i]);
      ok = ok && xstep()[i] != 0.0;  // nlopt_set_initial_step: "zero step size"
    }
    s->nevals = 0;
    s->done = 0;
    s->result = 0;
    s->minf = HUGE_VAL;
    s->pc = kFirst;  // the caller's point array already holds the first point
    if (!ok) {
      s->minf = __builtin_nan("");
      finish(kFailure);
    }
  }

  __device__ double& pf(int i) { return s->pts[i][0]; }
  __device__ double* pp(int i) { return &s->pts[i][1]; }

  // The full point for the subspace point xsub: x with the subspace
  // coordinates replaced (sbplx's subspace_func).  T equals x outside the
  // current subspace at every request (x changes only in nm_return, which
  // writes the subspace's final coordinates into T as well), so only the
  // subspace's ns <= 5 coordinates are written, not all n.
  __device__ void request(const double* xsub, double* T, int next) {
    for (int k = 0; k < s->ns; ++k) T[p()[s->is + k]] = xsub[k];
    s->pc = next;
  }
  // NLopt's CHECK_EVAL: count; keep the best subspace point; stop at maxeval.
  __device__ bool check_eval(const double* xc, double fc) {
    ++s->nevals;
    if (fc <= s->minf) {
      s->minf = fc;
      for (int k = 0; k < s->ns; ++k) s->xs[k] = xc[k];
    }
    return s->maxeval > 0 && s->nevals >= s->maxeval;
  }
  __device__ void finish(int code) {
    s->result = code;
    s->done = 1;
  }
  __device__ bool before(int a, int b) {
    return pf(a) < pf(b) || (pf(a) == pf(b) && a < b);
  }

  // The subspace solver returned `code`: write its best point back, then
  // the next subspace, the sweep's termination tests and step update.
  // Returns true when the machine continues (pc set), false when finished.
  __device__ void nm_return(int code, double* T) {
    if (s->fdiff > s->fdiff_max) s->fdiff_max = s->fdiff;
    for (int k = 0; k < s->ns; ++k) {
      const int q = p()[s->is + k];
      x()[q] = s->xs[k];
      T[q] = s->xs[k];  // keeps T == x outside the next subspace (request)
    }
    if (code == kFailure) return finish(kXtol);
    if (code != kXtol) return finish(code);
    if (!s->last) {
      s->i += s->ns;
      s->pc = kSubsel;
      return;
    }
    // ftol on (minf + the sweep's largest spread, minf): nlopt's relstop
    const double vold = s->minf + s->fdiff_max, vnew = s->minf;
    if (!isinf(vold)) {
      const double d = fabs(vnew - vold);
      if (d < s->ftol_abs || d < s->ftol_rel * (fabs(vnew) + fabs(vold)) * 0.5 ||
          (s->ftol_rel > 0 && vnew == vold))
        return finish(kFtol);
    }
    const int n = s->n;
    for (int k = 0; k < n; ++k) dx()[k] = x()[k] - xprev()[k];
    double scale;
    if (s->nsubs == 1) {
      scale = kPsi;
    } else {
      double stepnorm = 0.0, dxnorm = 0.0;
      for (int k = 0; k < n; ++k) {
        stepnorm += fabs(xstep()[k]);
        dxnorm += fabs(dx()[k]);
      }
      scale = dxnorm / stepnorm;
      scale = scale < kOmega ? kOmega : scale;
      scale = scale > 1.0 / kOmega ? 1.0 / kOmega : scale;
    }
    for (int k = 0; k < n; ++k)
      xstep()[k] = dx()[k] == 0.0 ? -(xstep()[k] * scale) : copysign(xstep()[k] * scale, dx()[k]);
    s->pc = kOuter;
  }

  // f: the value at the point last requested.  Advances to the next request
  // (written to T) or finishes.
  __device__ void resume(double f, double* T) {
    const int n = s->n;
    for (;;) {
      switch (s->pc) {
        case kFirst: {
          s->minf = f;
          s->nevals = 1;
          if (s->maxeval > 0 && s->nevals >= s->maxeval) return finish(kMaxEval);
          s->pc = kOuter;
          break;
        }
        case kOuter: {
          for (int k = 0; k < n; ++k) xprev()[k] = x()[k];
          s->fdiff_max = 0.0;
          s->nsubs = 0;
          // stable insertion sort of the indices by decreasing |dx|
          for (int k = 0; k < n; ++k) {
            const int v = k;
            const double key = fabs(dx()[v]);
            int j = k;
            while (j > 0 && fabs(dx()[p()[j - 1]]) < key) {
              p()[j] = p()[j - 1];
              --j;
            }
            p()[j] = v;
          }
          double nd = 0.0;
          for (int k = 0; k < n; ++k) nd += fabs(dx()[k]);
          s->normdx = nd;
          s->normi = 0.0;
          s->i = 0;
          s->pc = kSubsel;
          break;
        }
        case kSubsel: {
          const int i = s->i;
          int size;
          if (i + kNsMin < n) {
            // Rowan's figure of merit: the size with the sharpest drop in
            // the average |dx|, the remainder still partitionable
            const int nk = i + kNsMax > n ? n : i + kNsMax;
            double best = -HUGE_VAL, norm = s->normi;
            size = kNsMin;
            for (int k = i; k < i + kNsMin - 1; ++k) norm += fabs(dx()[p()[k]]);
            for (int k = i + kNsMin - 1; k < nk; ++k) {
              norm += fabs(dx()[p()[k]]);
              const int rest = n - k - 1;
              if ((rest + kNsMax - 1) / kNsMax > rest / kNsMin) continue;
              const double g = k + 1 < n ? norm / (k + 1) - (s->normdx - norm) / (n - (k + 1))
                                         : s->normdx / n;
              if (g > best) {
                best = g;
                size = (k + 1) - i;
              }
            }
            for (int k = i; k < i + size; ++k) s->normi += fabs(dx()[p()[k]]);
            s->last = 0;
          } else {
            size = n - i;
            s->last = 1;
          }
          s->is = i;
          s->ns = size;
          ++s->nsubs;
          for (int k = 0; k < size; ++k) {
            const int q = p()[i + k];
            s->xs[k] = x()[q];
            s->sstep[k] = xstep()[q];
            s->lbs[k] = lb()[q];
            s->ubs[k] = ub()[q];
          }
          // Nelder-Mead from xs, f(xs) = minf
          s->fdiff = HUGE_VAL;
          pf(0) = s->minf;
          for (int k = 0; k < size; ++k) pp(0)[k] = s->xs[k];
          s->k = 0;
          s->pc = kNmInit;
          break;
        }
        case kNmInit: {
          const int m = s->ns, k = s->k;
          if (k < m) {
            double* pt = pp(k + 1);
            for (int j = 0; j < m; ++j) pt[j] = s->xs[j];  // the current best
            const double xk = s->xs[k], st = s->sstep[k], lo = s->lbs[k], hi = s->ubs[k];
            double v = xk + st;
            if (v > hi) v = hi - xk > fabs(st) * 0.1 ? hi : xk - fabs(st);
            if (v < lo) {
              if (xk - lo > fabs(st) * 0.1) {
                v = lo;
              } else {
                v = xk + fabs(st);
                if (v > hi) v = 0.5 * ((hi - xk > xk - lo ? hi : lo) + xk);
              }
            }
            pt[k] = v;
            if (close_to(v, xk)) {
              nm_return(kFailure, T);
              if (s->done) return;
              break;
            }
            return request(pt, T, kNmInitGot);
          }
          s->init_diam = 0.0;
          s->pc = kNmIter;
          break;
        }
        case kNmInitGot: {
          const int k = s->k;
          pf(k + 1) = f;
          if (check_eval(pp(k + 1), f)) return nm_return(kMaxEval, T);
          s->k = k + 1;
          s->pc = kNmInit;
          break;
        }
        case kNmIter: {
          const int m = s->ns;
          int lo = 0, hi = 0;
          for (int i = 1; i <= m; ++i) {
            if (before(i, lo)) lo = i;
            if (before(hi, i)) hi = i;
          }
          s->lo = lo;
          s->hi = hi;
          const double* xl = pp(lo);
          const double* xh = pp(hi);
          s->fdiff = pf(hi) - pf(lo);
          if (s->init_diam == 0.0) {
            double d = 0.0;
            for (int j = 0; j < m; ++j) d += fabs(xl[j] - xh[j]);
            s->init_diam = d;
          }
          for (int j = 0; j < m; ++j) s->c[j] = 0.0;
          for (int i = 0; i <= m; ++i)
            if (i != hi)
              for (int j = 0; j < m; ++j) s->c[j] += pp(i)[j];
          for (int j = 0; j < m; ++j) s->c[j] *= 1.0 / m;
          double diam = 0.0;
          for (int j = 0; j < m; ++j) diam += fabs(xl[j] - xh[j]);
          if (diam < kPsi * s->init_diam) {
            nm_return(kXtol, T);
            if (s->done) return;
            break;
          }
          if (!reflect(m, s->xcur, s->c, kAlpha, xh, s->lbs, s->ubs)) {
            nm_return(kXtol, T);
            if (s->done) return;
            break;
          }
          return request(s->xcur, T, kNmReflGot);
        }
        case kNmReflGot: {
          const int m = s->ns, lo = s->lo, hi = s->hi;
          s->fr = f;
          if (check_eval(s->xcur, f)) return nm_return(kMaxEval, T);
          const double fr = f;
          if (fr < pf(lo)) {  // expansion
            if (!reflect(m, pp(hi), s->c, kGamma, pp(hi), s->lbs, s->ubs)) {
              nm_return(kXtol, T);
              if (s->done) return;
              break;
            }
            return request(pp(hi), T, kNmExpGot);
          }
          int pred = -1;  // the second highest
          for (int i = 0; i <= m; ++i)
            if (i != hi && (pred < 0 || before(pred, i))) pred = i;
          if (fr < pf(pred)) {  // accept the reflection
            for (int j = 0; j < m; ++j) pp(hi)[j] = s->xcur[j];
            pf(hi) = fr;
            s->pc = kNmIter;
            break;
          }
          // contraction: inside if fh <= fr, outside otherwise
          const double fh = pf(hi);
          if (!reflect(m, s->xcur, s->c, fh <= fr ? -kBeta : kBeta, pp(hi), s->lbs, s->ubs)) {
            nm_return(kXtol, T);
            if (s->done) return;
            break;
          }
          return request(s->xcur, T, kNmConGot);
        }
        case kNmExpGot: {
          const int m = s->ns, hi = s->hi;
          if (check_eval(pp(hi), f)) return nm_return(kMaxEval, T);
          if (f >= s->fr) {
            for (int j = 0; j < m; ++j) pp(hi)[j] = s->xcur[j];
            pf(hi) = s->fr;
          } else {
            pf(hi) = f;
          }
          s->pc = kNmIter;
          break;
        }
        case kNmConGot: {
          const int m = s->ns, hi = s->hi;
          if (check_eval(s->xcur, f)) return nm_return(kMaxEval, T);
          if (f < s->fr && f < pf(hi)) {
            for (int j = 0; j < m; ++j) pp(hi)[j] = s->xcur[j];
            pf(hi) = f;
            s->pc = kNmIter;
            break;
          }
          s->k = 0;  // shrink toward the lowest point
          s->pc = kNmShrink;
          break;
        }
        case kNmShrink: {
          const int m = s->ns, lo = s->lo;
          int k = s->k;
          if (k == lo) ++k;
          if (k > m) {
            s->pc = kNmIter;
            break;
          }
          s->k = k;
          if (!reflect(m, pp(k), pp(lo), -kDelta, pp(k), s->lbs, s->ubs)) {
            nm_return(kXtol, T);
            if (s->done) return;
            break;
          }
          return request(pp(k), T, kNmShrGot);
        }
        case kNmShrGot: {
          const int k = s->k;
          pf(k) = f;
          if (check_eval(pp(k), f)) return nm_return(kMaxEval, T);
          s->k = k + 1;
          s->pc = kNmShrink;
          break;
        }
        default:
          return finish(kFailure);
      }
    }
  }
};

}  // namespace sbplx
}  // namespace mtg
