// ORACLE — test infrastructure only (tests/, bench.py's cpu_baseline).
//
// A CPU restatement of NLopt's LN_SBPLX, the reference's default optimiser
// (NonlinearOptimizationParameters::algorithm = nlopt::LN_SBPLX,
// polynomial_optimization_nonlinear.h:61, configured at
// impl/polynomial_optimization_nonlinear_impl.h:95-101 and driven by
// optimizeTime, :332-397, on objectiveFunctionTime, :877-945).
//
// NLopt is a third-party dependency absent from /root/reference and from
// this image (version unpinned: cmake/FindNLOPT.cmake only asks pkg-config
// for "nlopt").  What follows restates its published algorithm: Rowan's
// Subplex (T. Rowan, "Functional Stability Analysis of Numerical
// Algorithms", PhD thesis, UT Austin 1990) as NLopt re-implements it
// (sbplx.c), with NLopt's bounded Nelder-Mead (nldrmd.c: reflections pinned
// to the bounds after Richardson & Kuester 1973) as the subspace solver.
//   * constants: psi = 0.25, omega = 0.1, subspace sizes nsmin = 2,
//     nsmax = 5; Nelder-Mead alpha = 1, beta = 0.5, gamma = 2, delta = 0.5;
//   * stopping: maxeval (every objective evaluation counts, the first one
//     included), ftol_rel / ftol_abs on (minf + the largest simplex spread
//     of the sweep, minf); the reference disables the x tolerances
//     (x_rel = x_abs = -1), so no x test is restated;
//   * tie rules where NLopt leaves them to its containers: the simplex is
//     ordered by (f, point index) (NLopt's red-black tree breaks ties by the
//     point's address, i.e. its index), and the progress vector's
//     permutation is a stable sort by decreasing |dx| (NLopt hands it to
//     qsort_r, whose order of equal keys is the C library's).
// Parity with NLopt itself is therefore unpinned; tests/test_sbplx.py pins
// this restatement against an independent NumPy restatement, and the device
// optimiser (mtg_sbplx_device.h) against this one.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <vector>

#include "orc_sbplx.h"

namespace {

constexpr double kPsi = 0.25, kOmega = 0.1;
constexpr int kNsMin = 2, kNsMax = 5;
constexpr double kAlpha = 1.0, kBeta = 0.5, kGamma = 2.0, kDelta = 0.5;

// nlopt's relstop(vold, vnew, reltol, abstol)
bool relstop(double vold, double vnew, double reltol, double abstol) {
  if (std::isinf(vold)) return false;
  const double d = std::fabs(vnew - vold);
  return d < abstol || d < reltol * (std::fabs(vnew) + std::fabs(vold)) * 0.5 ||
         (reltol > 0 && vnew == vold);
}

// nldrmd's close(): equal up to floating-point precision.
bool close_to(double a, double b) { return std::fabs(a - b) <= 1e-13 * (std::fabs(a) + std::fabs(b)); }

struct Stop {
  int nevals = 0;
  int maxeval = 0;
  double ftol_rel = 0.0, ftol_abs = 0.0;
  bool evals_done() const { return maxeval > 0 && nevals >= maxeval; }
};

// xnew = c + scale (c - xold), pinned to [lb, ub]; false when xnew
// coincides with c or with xold (nldrmd's reflectpt).  xnew may alias xold.
bool reflect(int n, double* xnew, const double* c, double scale, const double* xold,
             const double* lb, const double* ub) {
  bool equalc = true, equalold = true;
  for (int i = 0; i < n; ++i) {
    double v = c[i] + scale * (c[i] - xold[i]);
    if (v < lb[i]) v = lb[i];
    if (v > ub[i]) v = ub[i];
    equalc = equalc && close_to(v, c[i]);
    equalold = equalold && close_to(v, xold[i]);
    xnew[i] = v;
  }
  return !(equalc || equalold);
}

using Fn = std::function<double(const double*)>;

// One subspace: Nelder-Mead of dimension n on f from x (f(x) = *minf),
// stopping when the simplex's diameter has shrunk by psi (nldrmd_minimize_
// with psi > 0).  On return x is the best point seen and *fdiff the spread
// fh - fl of the last simplex.
int nelder_mead(int n, const Fn& f, const double* lb, const double* ub, double* x, double* minf,
                const double* xstep, Stop* stop, double* fdiff) {
  const int np = n + 1;
  std::vector<double> pts(static_cast<size_t>(np) * np);  // row i: f, then the point
  std::vector<double> c(n), xcur(n);
  auto P = [&](int i) { return pts.data() + static_cast<size_t>(i) * np; };
  *fdiff = HUGE_VAL;
  // CHECK_EVAL: count, keep the best point, stop at maxeval.
  auto check_eval = [&](const double* xc, double fc) -> int {
    ++stop->nevals;
    if (fc <= *minf) {
      *minf = fc;
      std::memcpy(x, xc, sizeof(double) * n);
    }
    return stop->evals_done() ? kSbplxMaxEval : 0;
  };
  P(0)[0] = *minf;
  std::memcpy(P(0) + 1, x, sizeof(double) * n);
  for (int i = 0; i < n; ++i) {
    double* pt = P(i + 1);
    std::memcpy(pt + 1, x, sizeof(double) * n);  // the current best point
    pt[1 + i] += xstep[i];
    if (pt[1 + i] > ub[i]) {
      if (ub[i] - x[i] > std::fabs(xstep[i]) * 0.1)
        pt[1 + i] = ub[i];
      else
        pt[1 + i] = x[i] - std::fabs(xstep[i]);
    }
    if (pt[1 + i] < lb[i]) {
      if (x[i] - lb[i] > std::fabs(xstep[i]) * 0.1) {
        pt[1 + i] = lb[i];
      } else {
        pt[1 + i] = x[i] + std::fabs(xstep[i]);
        if (pt[1 + i] > ub[i]) pt[1 + i] = 0.5 * ((ub[i] - x[i] > x[i] - lb[i] ? ub[i] : lb[i]) + x[i]);
      }
    }
    if (close_to(pt[1 + i], x[i])) return kSbplxFailure;
    pt[0] = f(pt + 1);
    if (int r = check_eval(pt + 1, pt[0])) return r;
  }
  double init_diam = 0.0;
  // simplex order: by value, ties by point index
  auto before = [&](int a, int b) { return P(a)[0] < P(b)[0] || (P(a)[0] == P(b)[0] && a < b); };
  for (;;) {
    int lo = 0, hi = 0;
    for (int i = 1; i < np; ++i) {
      if (before(i, lo)) lo = i;
      if (before(hi, i)) hi = i;
    }
    const double fl = P(lo)[0];
    double fh = P(hi)[0];
    double* xl = P(lo) + 1;
    double* xh = P(hi) + 1;
    *fdiff = fh - fl;
    if (init_diam == 0.0)
      for (int i = 0; i < n; ++i) init_diam += std::fabs(xl[i] - xh[i]);
    // centroid of every point but the highest
    std::fill(c.begin(), c.end(), 0.0);
    for (int i = 0; i < np; ++i)
      if (i != hi)
        for (int j = 0; j < n; ++j) c[j] += P(i)[1 + j];
    for (int j = 0; j < n; ++j) c[j] *= 1.0 / n;
    double diam = 0.0;
    for (int i = 0; i < n; ++i) diam += std::fabs(xl[i] - xh[i]);
    if (diam < kPsi * init_diam) return kSbplxXtol;
    if (!reflect(n, xcur.data(), c.data(), kAlpha, xh, lb, ub)) return kSbplxXtol;
    const double fr = f(xcur.data());
    if (int r = check_eval(xcur.data(), fr)) return r;
    if (fr < fl) {  // expansion
      if (!reflect(n, xh, c.data(), kGamma, xh, lb, ub)) return kSbplxXtol;
      fh = f(xh);
      if (int r = check_eval(xh, fh)) return r;
      if (fh >= fr) {
        fh = fr;
        std::memcpy(xh, xcur.data(), sizeof(double) * n);
      }
    } else {
      int pred = -1;  // the second highest
      for (int i = 0; i < np; ++i)
        if (i != hi && (pred < 0 || before(pred, i))) pred = i;
      if (fr < P(pred)[0]) {  // accept the reflection
        std::memcpy(xh, xcur.data(), sizeof(double) * n);
        fh = fr;
      } else {  // contraction: outside if fr < fh, inside otherwise
        if (!reflect(n, xcur.data(), c.data(), fh <= fr ? -kBeta : kBeta, xh, lb, ub))
          return kSbplxXtol;
        const double fc = f(xcur.data());
        if (int r = check_eval(xcur.data(), fc)) return r;
        if (fc < fr && fc < fh) {
          std::memcpy(xh, xcur.data(), sizeof(double) * n);
          fh = fc;
        } else {  // shrink toward the lowest point, then restart
          for (int i = 0; i < np; ++i) {
            if (i == lo) continue;
            double* pt = P(i);
            if (!reflect(n, pt + 1, xl, -kDelta, pt + 1, lb, ub)) return kSbplxXtol;
            pt[0] = f(pt + 1);
            if (int r = check_eval(pt + 1, pt[0])) return r;
          }
          continue;
        }
      }
    }
    P(hi)[0] = fh;
  }
}

}  // namespace

int orc_sbplx_run(int n, const std::function<double(const double*)>& f, const double* lb,
                  const double* ub, double* x, double* minf, const double* xstep0, int maxeval,
                  double ftol_rel, double ftol_abs, int* nevals) {
  Stop stop;
  stop.maxeval = maxeval;
  stop.ftol_rel = ftol_rel;
  stop.ftol_abs = ftol_abs;
  int ret = kSbplxSuccess;
  // NLopt refuses a start outside the bounds (or lb > ub) before evaluating
  // anything (nlopt_optimize returns NLOPT_INVALID_ARGS; nlopt::opt::optimize
  // throws and optimizeTime returns nlopt::FAILURE, nonlinear_impl:389-394):
  // x unchanged, no evaluation.
  for (int i = 0; i < n; ++i)
    if (lb[i] > ub[i] || x[i] < lb[i] || x[i] > ub[i]) {
      *minf = std::numeric_limits<double>::quiet_NaN();
      if (nevals) *nevals = 0;
      return kSbplxFailure;
    }
  *minf = f(x);
  ++stop.nevals;
  std::vector<double> xstep(xstep0, xstep0 + n), xprev(n), dx(n, 0.0);
  std::vector<double> xs(n), xsstep(n), lbs(n), ubs(n), xfull(n);
  std::vector<int> p(n);
  int is = 0, ns = 0;
  // f over the subspace p[is .. is+ns): the current point with those
  // coordinates replaced (sbplx's subspace_func).
  const Fn fsub = [&](const double* xsub) {
    std::memcpy(xfull.data(), x, sizeof(double) * n);
    for (int k = 0; k < ns; ++k) xfull[p[is + k]] = xsub[k];
    return f(xfull.data());
  };
  auto run_subspace = [&](int start, int size, double* fdiff) {
    is = start;
    ns = size;
    for (int k = 0; k < ns; ++k) {
      xs[k] = x[p[is + k]];
      xsstep[k] = xstep[p[is + k]];
      lbs[k] = lb[p[is + k]];
      ubs[k] = ub[p[is + k]];
    }
    const int r = nelder_mead(ns, fsub, lbs.data(), ubs.data(), xs.data(), minf, xsstep.data(),
                              &stop, fdiff);
    for (int k = 0; k < ns; ++k) x[p[is + k]] = xs[k];
    return r;
  };
  if (stop.evals_done()) {
    ret = kSbplxMaxEval;
  } else {
    for (;;) {
      std::memcpy(xprev.data(), x, sizeof(double) * n);
      double normi = 0.0, normdx = 0.0, fdiff = 0.0, fdiff_max = 0.0;
      int nsubs = 0;
      std::iota(p.begin(), p.end(), 0);
      std::stable_sort(p.begin(), p.end(),
                       [&](int a, int b) { return std::fabs(dx[a]) > std::fabs(dx[b]); });
      for (int i = 0; i < n; ++i) normdx += std::fabs(dx[i]);
      int i = 0, r = 0;
      for (; i + kNsMin < n; i += ns) {
        // the subspace starting at i: the size that maximises Rowan's
        // figure of merit (a sudden drop in the average |dx|), leaving a
        // remainder that can still be partitioned
        int nk = i + kNsMax > n ? n : i + kNsMax;
        double goodness_best = -HUGE_VAL, norm = normi;
        int size = kNsMin;
        for (int k = i; k < i + kNsMin - 1; ++k) norm += std::fabs(dx[p[k]]);
        for (int k = i + kNsMin - 1; k < nk; ++k) {
          norm += std::fabs(dx[p[k]]);
          const int rest = n - k - 1;
          if ((rest + kNsMax - 1) / kNsMax > rest / kNsMin) continue;
          const double goodness = k + 1 < n
                                      ? norm / (k + 1) - (normdx - norm) / (n - (k + 1))
                                      : normdx / n;
          if (goodness > goodness_best) {
            goodness_best = goodness;
            size = (k + 1) - i;
          }
        }
        for (int k = i; k < i + size; ++k) normi += std::fabs(dx[p[k]]);
        ++nsubs;
        r = run_subspace(i, size, &fdiff);
        if (fdiff > fdiff_max) fdiff_max = fdiff;
        if (r != kSbplxXtol) break;
      }
      if (r == 0 || r == kSbplxXtol) {  // the last subspace
        ++nsubs;
        r = run_subspace(i, n - i, &fdiff);
        if (fdiff > fdiff_max) fdiff_max = fdiff;
      }
      if (r == kSbplxFailure) {
        ret = kSbplxXtol;
        break;
      }
      if (r != kSbplxXtol) {
        ret = r;
        break;
      }
      if (relstop(*minf + fdiff_max, *minf, stop.ftol_rel, stop.ftol_abs)) {
        ret = kSbplxFtol;
        break;
      }
      for (int k = 0; k < n; ++k) dx[k] = x[k] - xprev[k];
      double scale;
      if (nsubs == 1) {
        scale = kPsi;
      } else {
        double stepnorm = 0.0, dxnorm = 0.0;
        for (int k = 0; k < n; ++k) {
          stepnorm += std::fabs(xstep[k]);
          dxnorm += std::fabs(dx[k]);
        }
        scale = dxnorm / stepnorm;
        if (scale < kOmega) scale = kOmega;
        if (scale > 1.0 / kOmega) scale = 1.0 / kOmega;
      }
      for (int k = 0; k < n; ++k)
        xstep[k] = dx[k] == 0.0 ? -(xstep[k] * scale) : std::copysign(xstep[k] * scale, dx[k]);
    }
  }
  if (nevals) *nevals = stop.nevals;
  return ret;
}

namespace {
// A fixed test objective for pinning the restatement (tests/test_sbplx.py):
// a rotated, shifted ill-conditioned quadratic plus a quartic term.
double test_fn(int n, const double* x) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    const double yi = x[i] - 0.3 * (i + 1);
    const double yj = i + 1 < n ? x[i + 1] - 0.3 * (i + 2) : 0.0;
    s += (1.0 + i) * yi * yi + 0.5 * yi * yj + 0.1 * yi * yi * yi * yi;
  }
  return s;
}
}  // namespace

extern "C" int orc_sbplx_test(int n, const double* lb, const double* ub, double* x,
                              const double* xstep, int maxeval, double ftol_rel,
                              double ftol_abs, double* minf, int* nevals, double* history) {
  int k = 0;
  auto f = [&](const double* xx) {
    if (history && k < maxeval) std::memcpy(history + static_cast<size_t>(k) * n, xx, sizeof(double) * n);
    ++k;
    return test_fn(n, xx);
  };
  return orc_sbplx_run(n, f, lb, ub, x, minf, xstep, maxeval, ftol_rel, ftol_abs, nevals);
}
