// ORACLE — test infrastructure only.  NLopt LN_SBPLX restated
// (orc_sbplx.cpp); result codes are NLopt's nlopt_result values.
#pragma once
#include <functional>

constexpr int kSbplxFailure = -1;  // NLOPT_FAILURE (degenerate simplex; start out of bounds)
constexpr int kSbplxSuccess = 1;   // NLOPT_SUCCESS
constexpr int kSbplxFtol = 3;      // NLOPT_FTOL_REACHED
constexpr int kSbplxXtol = 4;      // NLOPT_XTOL_REACHED
constexpr int kSbplxMaxEval = 5;   // NLOPT_MAXEVAL_REACHED

// Minimise f over [lb, ub] from x (in/out: the best point) with initial
// steps xstep0; *minf the best value.  Returns the nlopt_result code.
int orc_sbplx_run(int n, const std::function<double(const double*)>& f, const double* lb,
                  const double* ub, double* x, double* minf, const double* xstep0, int maxeval,
                  double ftol_rel, double ftol_abs, int* nevals);
