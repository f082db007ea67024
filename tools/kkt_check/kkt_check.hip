// Standalone check of the tube kernel's block factorisation + solve
// (Tube<N>::factor / solve, unconstrained KKT = I_3 (x) P blocks) against a
// dense Cholesky solve on the host.  Build: see tools/kkt_check/build.sh.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../mav_tube_trajectory_generation_amd/csrc/mtg_tube_device.h"

using namespace mtg;
constexpr int N = 10, M = 5, BS = 15;

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k(int S, const double* Pd, const double* Po, const double* Gc,
                  const double* bet, const double* rhs, double* x, int* fail) {
  extern __shared__ double smem[];
  const TubeLayout L = make_tube_layout(N, S);
  Tube<N> t{S, 4, S - 1, tube_ncon(N, S), &L, smem, static_cast<int>(threadIdx.x)};
  const int nv = S - 1;
  for (int i = threadIdx.x; i < nv * M * M; i += 64) smem[L.Pd + i] = Pd[i];
  for (int i = threadIdx.x; i < (nv - 1) * M * M; i += 64) smem[L.Po + i] = Po[i];
  for (int i = threadIdx.x; i < nv * BS; i += 64) smem[L.rhs + i] = rhs[i];
  for (int i = threadIdx.x; i < S * N * 9; i += 64) smem[L.Gc + i] = Gc[i];
  for (int i = threadIdx.x; i < S * N * M; i += 64) smem[L.bet + i] = bet[i];
  int* f = reinterpret_cast<int*>(smem + L.ndouble);
  if (threadIdx.x == 0) *f = 0;
  __syncthreads();
  // IPM-like sequence: unconstrained factor + solve, then the constrained
  // factor and two solves (the second must be the checked one).
  t.factor(f, false);
  __syncthreads();
  t.solve(L.rhs, L.dx);
  __syncthreads();
  t.factor(f, true);
  __syncthreads();
  for (int i = threadIdx.x; i < nv * BS; i += 64) smem[L.rhs + i] = 0.5 * rhs[i];
  __syncthreads();
  t.solve(L.rhs, L.dx);
  __syncthreads();
  for (int i = threadIdx.x; i < nv * BS; i += 64) smem[L.rhs + i] = rhs[i];
  __syncthreads();
  t.solve(L.rhs, L.x);
  __syncthreads();
  for (int i = threadIdx.x; i < nv * BS; i += 64) x[i] = smem[L.x + i];
  if (threadIdx.x == 0) *fail = *f;
}

int main() {
  const int S = 10, nv = S - 1, n = nv * BS;
  std::mt19937 g(3);
  std::normal_distribution<double> nd;
  std::vector<double> Pd(nv * M * M), Po((nv - 1) * M * M), rhs(n), x(n);
  for (int a = 0; a < nv; ++a) {
    double X[M * M];
    for (auto& v : X) v = nd(g);
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < M; ++j) {
        double s = (i == j) ? 6.0 : 0.0;
        for (int k = 0; k < M; ++k) s += X[i * M + k] * X[j * M + k];
        Pd[a * M * M + i * M + j] = s;
      }
  }
  for (auto& v : Po) v = 0.5 * nd(g);
  for (auto& v : rhs) v = nd(g);
  std::vector<double> Gc(S * N * 9), bet(S * N * M);
  for (int cp = 0; cp < S * N; ++cp) {
    double Y[9];
    for (auto& v : Y) v = nd(g);
    const double scale = std::pow(10.0, 6.0 * (cp % 7) / 6.0);  // ill-conditioned mix
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s2 = 0.0;
        for (int q = 0; q < 3; ++q) s2 += Y[i * 3 + q] * Y[j * 3 + q];
        Gc[cp * 9 + i * 3 + j] = scale * s2;
      }
  }
  for (auto& v : bet) v = nd(g);
  // dense K (vertex-major blocks (a, d, m)), K x = rhs
  std::vector<double> K(n * n, 0.0);
  for (int a = 0; a < nv; ++a)
    for (int d = 0; d < 3; ++d)
      for (int m = 0; m < M; ++m)
        for (int m2 = 0; m2 < M; ++m2) {
          K[(a * BS + d * M + m) * n + a * BS + d * M + m2] = Pd[a * M * M + m * M + m2];
          if (a < nv - 1) {
            const double p = Po[a * M * M + m * M + m2];
            K[(a * BS + d * M + m) * n + (a + 1) * BS + d * M + m2] = p;
            K[((a + 1) * BS + d * M + m2) * n + a * BS + d * M + m] = p;
          }
        }
  for (int a = 0; a < nv; ++a) {
    const int u = a + 1;
    for (int q = 0; q < N; ++q) {
      const int i = q < M ? u - 1 : u, j = q < M ? q + M : q - M, cp = i * N + j;
      for (int d = 0; d < 3; ++d)
        for (int m = 0; m < M; ++m)
          for (int d2 = 0; d2 < 3; ++d2)
            for (int m2 = 0; m2 < M; ++m2)
              K[(a * BS + d * M + m) * n + a * BS + d2 * M + m2] +=
                  Gc[cp * 9 + d * 3 + d2] * bet[cp * M + m] * bet[cp * M + m2];
    }
  }
  // host Gaussian elimination
  std::vector<double> A = K, b = rhs;
  for (int c = 0; c < n; ++c)
    for (int i = c + 1; i < n; ++i) {
      const double f = A[i * n + c] / A[c * n + c];
      for (int j = c; j < n; ++j) A[i * n + j] -= f * A[c * n + j];
      b[i] -= f * b[c];
    }
  std::vector<double> xr(n);
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < n; ++j) s -= A[i * n + j] * xr[j];
    xr[i] = s / A[i * n + i];
  }
  double *dPd, *dPo, *dr, *dx, *dG, *dB;
  hipMalloc(&dG, Gc.size() * 8);
  hipMalloc(&dB, bet.size() * 8);
  hipMemcpy(dG, Gc.data(), Gc.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, bet.data(), bet.size() * 8, hipMemcpyHostToDevice);
  int* df;
  hipMalloc(&dPd, Pd.size() * 8);
  hipMalloc(&dPo, Po.size() * 8);
  hipMalloc(&dr, n * 8);
  hipMalloc(&dx, n * 8);
  hipMalloc(&df, 4);
  hipMemcpy(dPd, Pd.data(), Pd.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dPo, Po.data(), Po.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dr, rhs.data(), n * 8, hipMemcpyHostToDevice);
  const size_t bytes = make_tube_layout(N, S).bytes() + 16;
  hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), bytes, 0, S, dPd, dPo, dG, dB, dr, dx, df);
  int fl = -1;
  hipMemcpy(x.data(), dx, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(&fl, df, 4, hipMemcpyDeviceToHost);
  double err = 0.0, nr = 0.0;
  for (int i = 0; i < n; ++i) {
    err = std::fmax(err, std::fabs(x[i] - xr[i]));
    nr = std::fmax(nr, std::fabs(xr[i]));
  }
  std::printf("fail=%d  max|x - x_ref| = %.3e  (max|x_ref| = %.3e)\n", fl, err, nr);
  for (int i = 0; i < 6; ++i) std::printf("  %d: %.12f %.12f\n", i, x[i], xr[i]);
  return err <= 1e-6 * nr ? 0 : 1;
}
