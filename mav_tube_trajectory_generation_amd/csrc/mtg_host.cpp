// mtg_host.cpp — host side of the C ABI (include/mtg_hip.h): device
// context, plans (constraint pattern + constant tables), argument checks and
// the batched input generator.  Kernels live in mtg_kernels.hip / mtg_tube.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "mtg_internal.h"
#include "mtg_sbplx_device.h"
#include "mav_tube_trajectory_generation_amd/vertex.h"

struct mtg_ctx {
  int device = 0;
  std::mutex mu;
  std::map<std::pair<int, int>, double*> tables;  // (N, r) -> H(1), A(1)^-1
};

// Persistent staging of the host-memory entry point (mtg_linear_solve_host),
// created on first use and grown on demand: a pinned, device-mapped host
// buffer, a device buffer of the same layout and a non-blocking stream of
// the plan's own.  Small calls (the single-trajectory shim: up to
// kZeroCopyBytes) run zero-copy: the kernel reads its inputs from and writes
// its outputs to the mapped host buffer, so a steady-state call is one launch
// and a wait on that stream.  Larger calls copy in and out by DMA (one H2D
// copy, one launch, one D2H copy).  No allocation, no device-wide
// synchronisation.  Layout (bytes, each part 256-aligned): inputs
// [fixed_vals | times], outputs [coeffs | cost | free_vals | status].
constexpr size_t kZeroCopyBytes = 64 * 1024;
struct mtg_staging {
  std::mutex mu;
  hipStream_t stream = nullptr;
  char* host = nullptr;
  char* hdev = nullptr;  // device address of the mapped host buffer
  char* dev = nullptr;
  size_t bytes = 0;
  ~mtg_staging() {
    if (stream) (void)hipStreamDestroy(stream);
    if (host) (void)hipHostFree(host);
    if (dev) (void)hipFree(dev);
  }
};

struct mtg_plan {
  mtg_ctx* ctx = nullptr;
  mtg::PlanDev dev{};
  int* d_slots = nullptr;
  int* d_free_map = nullptr;
  int* d_fixed_map = nullptr;
  std::unique_ptr<mtg_staging> stage{new mtg_staging};
};

namespace {

using mtg::PlanDev;

int from_hip(hipError_t e) { return e == hipSuccess ? MTG_OK : MTG_ERR_HIP; }

// The launch helpers report hipGetLastError() after their launches, and the
// runtime keeps the last error of ANY failed HIP call on this thread (the
// caller's, or another library's) until it is read.  The entry points that
// launch work (and so read that slot afterwards) clear it first, so a stale
// error is never returned as this call's MTG_ERR_HIP; getters, size queries,
// the host-only generator and the create / destroy calls (which check their
// HIP calls' return values directly) leave the caller's pending error alone.  Round 4's failed graph captures were exactly
// that: an experiment's event-record call failed inside the capture and the
// next mtg_linear_solve reported it ("Graph capture").
void clear_stale_error() { (void)hipGetLastError(); }

bool valid_N(int N) { return N >= 4 && N <= 12 && N % 2 == 0; }

// Constant tables for (N, r), computed in long double (layout: H(1) N*N,
// A(1)^-1 N*N, C^-1 M*M):
//   A(1)  = setupMappingMatrix(1)                (linear_impl:101-111)
//   Q(1)  = computeQuadraticCostJacobian(r, 1)   (linear_impl:557-573)
//   H(1)  = A(1)^-T Q(1) A(1)^-1                 (linear_impl:318)
// H(T) and A(T)^-1 follow by the exact time-scaling identity (mtg_device.h).
void build_tables(int N, int r, std::vector<double>* out) {
  typedef long double ld;
  const int M = N / 2;
  auto falling = [](int n, int i) -> ld {
    if (i < n) return 0;
    ld p = 1;
    for (int m = 0; m < n; ++m) p *= (i - m);
    return p;
  };
  std::vector<ld> A(N * N, 0), Ai(N * N, 0), Q(N * N, 0), H(N * N, 0);
  for (int l = 0; l < M; ++l) {
    A[l * N + l] = falling(l, l);
    for (int j = l; j < N; ++j) A[(M + l) * N + j] = falling(l, j);
  }
  // Gauss-Jordan with partial pivoting.
  std::vector<ld> W(A), I(N * N, 0);
  for (int i = 0; i < N; ++i) I[i * N + i] = 1;
  for (int k = 0; k < N; ++k) {
    int p = k;
    for (int i = k + 1; i < N; ++i)
      if (std::fabs(W[i * N + k]) > std::fabs(W[p * N + k])) p = i;
    for (int j = 0; j < N; ++j) {
      std::swap(W[k * N + j], W[p * N + j]);
      std::swap(I[k * N + j], I[p * N + j]);
    }
    const ld piv = W[k * N + k];
    for (int j = 0; j < N; ++j) {
      W[k * N + j] /= piv;
      I[k * N + j] /= piv;
    }
    for (int i = 0; i < N; ++i) {
      if (i == k) continue;
      const ld f = W[i * N + k];
      if (f == 0) continue;
      for (int j = 0; j < N; ++j) {
        W[i * N + j] -= f * W[k * N + j];
        I[i * N + j] -= f * I[k * N + j];
      }
    }
  }
  Ai = I;
  for (int j = r; j < N; ++j)
    for (int k = r; k < N; ++k)
      Q[j * N + k] = 2 * falling(r, j) * falling(r, k) / static_cast<ld>(j + k - 2 * r + 1);
  // H = Ai^T Q Ai.
  std::vector<ld> QA(N * N, 0);
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < N; ++k)
      for (int j = 0; j < N; ++j) QA[i * N + j] += Q[i * N + k] * Ai[k * N + j];
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < N; ++k)
      for (int j = 0; j < N; ++j) H[i * N + j] += Ai[k * N + i] * QA[k * N + j];
  // Bezier control-point map (qcqp_impl:280-297): B_ul(T) = diag(T^-l) C
  // with C[l][j] = n!/(n-l)! (-1)^(l+j) binom(l, j), n = N-1, so
  // B_ul^-1(T) = C^-1 diag(T^l); C^-1 by forward substitution.
  std::vector<ld> C(M * M, 0), Ci(M * M, 0);
  for (int l = 0; l < M; ++l)
    for (int j = 0; j <= l; ++j) {
      ld binom = 1;
      for (int t = 0; t < j; ++t) binom = binom * (l - t) / (t + 1);
      C[l * M + j] = falling(l, N - 1) * (((l + j) & 1) ? -1 : 1) * binom;
    }
  for (int c = 0; c < M; ++c)
    for (int i = 0; i < M; ++i) {
      ld s = (i == c) ? 1 : 0;
      for (int k = 0; k < i; ++k) s -= C[i * M + k] * Ci[k * M + c];
      Ci[i * M + c] = s / C[i * M + i];
    }
  // Symmetrise (exact in real arithmetic).
  out->assign(2 * N * N + M * M, 0.0);
  for (int i = 0; i < M * M; ++i) (*out)[2 * N * N + i] = static_cast<double>(Ci[i]);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      (*out)[i * N + j] = static_cast<double>((H[i * N + j] + H[j * N + i]) / 2);
      (*out)[N * N + i * N + j] = static_cast<double>(Ai[i * N + j]);
    }
}

// Makes `device` current for the calling thread while in scope and restores
// the caller's device afterwards: allocations and the plan's staging stream
// land on the context's device whatever device the thread had selected.
struct DeviceScope {
  int prev = -1;
  bool ok = false;
  explicit DeviceScope(int device) {
    ok = hipGetDevice(&prev) == hipSuccess && hipSetDevice(device) == hipSuccess;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int get_tables(mtg_ctx* ctx, int N, int r, const double** out) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  auto key = std::make_pair(N, r);
  auto it = ctx->tables.find(key);
  if (it != ctx->tables.end()) {
    *out = it->second;
    return MTG_OK;
  }
  std::vector<double> host;
  build_tables(N, r, &host);
  double* d = nullptr;
  DeviceScope dev(ctx->device);
  if (!dev.ok) return MTG_ERR_HIP;
  if (hipMalloc(&d, host.size() * sizeof(double)) != hipSuccess) return MTG_ERR_HIP;
  if (hipMemcpy(d, host.data(), host.size() * sizeof(double), hipMemcpyHostToDevice) !=
      hipSuccess) {
    (void)hipFree(d);
    return MTG_ERR_HIP;
  }
  ctx->tables[key] = d;
  *out = d;
  return MTG_OK;
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return n ? hipMalloc(&p, n * sizeof(T)) : hipSuccess; }
};

}  // namespace

extern "C" {

const char* mtg_status_string(int status) {
  switch (status) {
    case MTG_OK: return "ok";
    case MTG_ERR_INVALID_ARG: return "invalid argument";
    case MTG_ERR_NO_DEVICE: return "no HIP device";
    case MTG_ERR_HIP: return "HIP runtime error";
    case MTG_ERR_UNSUPPORTED: return "unsupported size (LDS budget)";
    case MTG_ERR_NUMERIC: return "numerical failure in at least one trajectory";
    default: return "unknown status";
  }
}

int mtg_version(void) { return 100; }

int mtg_ctx_create(int device, mtg_ctx** out) {
  if (!out) return MTG_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MTG_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return MTG_ERR_INVALID_ARG;
  if (hipSetDevice(device) != hipSuccess) return MTG_ERR_HIP;
  mtg_ctx* c = new mtg_ctx;
  c->device = device;
  *out = c;
  return MTG_OK;
}

int mtg_ctx_destroy(mtg_ctx* ctx) {
  if (!ctx) return MTG_ERR_INVALID_ARG;
  DeviceScope dev(ctx->device);
  for (auto& kv : ctx->tables) (void)hipFree(kv.second);
  delete ctx;
  return MTG_OK;
}

int mtg_ctx_device(const mtg_ctx* ctx) { return ctx ? ctx->device : MTG_ERR_INVALID_ARG; }

int mtg_plan_create(mtg_ctx* ctx, int N, int D, int r, int S, const uint8_t* fixed_mask,
                    mtg_plan** out) {
  if (!ctx || !out || !fixed_mask) return MTG_ERR_INVALID_ARG;
  *out = nullptr;
  if (!valid_N(N) || D < 1 || D > mtg::kMaxD || r < 0 || r > N / 2 - 1 || S < 1)
    return MTG_ERR_INVALID_ARG;
  if (mtg::linear_lds_bytes(N, S, D) > static_cast<size_t>(mtg::kMaxLdsBytes))
    return MTG_ERR_UNSUPPORTED;
  const int M = N / 2;
  // setupConstraintReorderingMatrix (linear_impl:171-252): fixed and free
  // constraints each numbered in (vertex, derivative) order.
  std::vector<int> slots((S + 1) * M), free_map, fixed_map;
  int nf = 0, np = 0;
  uint64_t fmask = 0;
  const bool use_mask = (S + 1) * M <= 64;
  for (int v = 0; v <= S; ++v)
    for (int k = 0; k < M; ++k) {
      if (fixed_mask[v * M + k]) {
        slots[v * M + k] = nf++;
        fixed_map.push_back(v * M + k);
        if (use_mask) fmask |= 1ull << (v * M + k);
      } else {
        slots[v * M + k] = -(np + 1);
        free_map.push_back(v * M + k);
        ++np;
      }
    }
  const double* tab = nullptr;
  int rc = get_tables(ctx, N, r, &tab);
  if (rc) return rc;
  std::unique_ptr<mtg_plan> p(new mtg_plan);
  p->ctx = ctx;
  DeviceScope dev(ctx->device);
  if (!dev.ok) return MTG_ERR_HIP;
  if (hipMalloc(&p->d_slots, slots.size() * sizeof(int)) != hipSuccess) return MTG_ERR_HIP;
  if (hipMalloc(&p->d_free_map, (free_map.size() + 1) * sizeof(int)) != hipSuccess) {
    (void)hipFree(p->d_slots);
    return MTG_ERR_HIP;
  }
  if (hipMalloc(&p->d_fixed_map, (fixed_map.size() + 1) * sizeof(int)) != hipSuccess) {
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_free_map);
    return MTG_ERR_HIP;
  }
  hipError_t e = hipMemcpy(p->d_slots, slots.data(), slots.size() * sizeof(int),
                           hipMemcpyHostToDevice);
  if (e == hipSuccess && np)
    e = hipMemcpy(p->d_free_map, free_map.data(), free_map.size() * sizeof(int),
                  hipMemcpyHostToDevice);
  if (e == hipSuccess && nf)
    e = hipMemcpy(p->d_fixed_map, fixed_map.data(), fixed_map.size() * sizeof(int),
                  hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_free_map);
    (void)hipFree(p->d_fixed_map);
    return MTG_ERR_HIP;
  }
  // Standard pattern (createRandomVertices / makeStartOrEnd, vertex.cpp:
  // 27-82, 147-153): start and end fully fixed, intermediate positions only.
  bool std_pattern = S >= 2 && S <= mtg::kMaxStdS;
  for (int v = 0; v <= S && std_pattern; ++v)
    for (int k = 0; k < M; ++k) {
      const bool want = (v == 0 || v == S) ? true : (k == 0);
      if ((fixed_mask[v * M + k] != 0) != want) std_pattern = false;
    }
  p->dev = PlanDev{N, D, r, S, nf, np, tab, p->d_slots, p->d_free_map, p->d_fixed_map,
                   fmask, use_mask ? 1 : 0, std_pattern ? 1 : 0, MTG_KERNEL_AUTO};
  *out = p.release();
  return MTG_OK;
}

int mtg_plan_destroy(mtg_plan* plan) {
  if (!plan) return MTG_ERR_INVALID_ARG;
  DeviceScope dev(plan->ctx->device);
  plan->stage.reset();  // its stream and buffers belong to the plan's device
  (void)hipFree(plan->d_slots);
  (void)hipFree(plan->d_free_map);
  (void)hipFree(plan->d_fixed_map);
  delete plan;
  return MTG_OK;
}

int mtg_plan_set_kernel(mtg_plan* plan, int kernel) {
  if (!plan || kernel < MTG_KERNEL_AUTO || kernel > MTG_KERNEL_LANE_PAIR)
    return MTG_ERR_INVALID_ARG;
  if (kernel == MTG_KERNEL_STANDARD && !plan->dev.std_pattern) return MTG_ERR_UNSUPPORTED;
  if (kernel >= MTG_KERNEL_LANE) {
    mtg::PlanDev probe = plan->dev;
    probe.kernel = MTG_KERNEL_AUTO;
    if (!mtg::has_linear_lane(probe)) return MTG_ERR_UNSUPPORTED;
  }
  plan->dev.kernel = kernel;
  return MTG_OK;
}

int mtg_plan_kernel(const mtg_plan* plan) {
  if (!plan) return MTG_ERR_INVALID_ARG;
  if (plan->dev.kernel >= MTG_KERNEL_LANE) return plan->dev.kernel;
  return mtg::use_std_kernel(plan->dev) ? MTG_KERNEL_STANDARD : MTG_KERNEL_GENERIC;
}

int mtg_plan_kernel_for_batch(const mtg_plan* plan, int64_t B) {
  if (!plan || B < 0) return MTG_ERR_INVALID_ARG;
  return mtg::linear_kernel_for_batch(plan->dev, B);
}

int mtg_plan_counts(const mtg_plan* plan, int* n_fixed, int* n_free) {
  if (!plan) return MTG_ERR_INVALID_ARG;
  if (n_fixed) *n_fixed = plan->dev.nf;
  if (n_free) *n_free = plan->dev.np;
  return MTG_OK;
}

int mtg_linear_solve(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                     const double* times, double* coeffs, double* cost, double* free_vals,
                     int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || B < 0 || B > 0x7fffffff || !times || !coeffs) return MTG_ERR_INVALID_ARG;
  if (plan->dev.nf > 0 && !fixed_vals) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_linear_solve(plan->dev, B, fixed_vals, times, coeffs, cost,
                                           free_vals, status,
                                           static_cast<hipStream_t>(stream)));
}

int mtg_linear_solve_host(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                          const double* times, double* coeffs, double* cost,
                          double* free_vals, int32_t* status) {
  clear_stale_error();
  if (!plan || B < 0 || B > 0x7fffffff || !times || !coeffs) return MTG_ERR_INVALID_ARG;
  if (plan->dev.nf > 0 && !fixed_vals) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  const PlanDev& pl = plan->dev;
  const size_t nfv = static_cast<size_t>(B) * pl.D * pl.nf;
  const size_t nt = static_cast<size_t>(B) * pl.S;
  const size_t nc = static_cast<size_t>(B) * pl.S * pl.D * pl.N;
  const size_t npv = static_cast<size_t>(B) * pl.D * pl.np;
  auto up = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t o_t = up(nfv * sizeof(double)), o_out = up(o_t + nt * sizeof(double));
  const size_t o_cost = up(o_out + nc * sizeof(double));
  const size_t o_free = up(o_cost + B * sizeof(double));
  const size_t o_st = up(o_free + npv * sizeof(double));
  const size_t total = up(o_st + B * sizeof(int32_t));
  mtg_staging& sg = *plan->stage;
  std::lock_guard<std::mutex> lock(sg.mu);
  DeviceScope dev(plan->ctx->device);
  if (!dev.ok) return MTG_ERR_HIP;
  if (!sg.stream) {
    if (hipStreamCreateWithFlags(&sg.stream, hipStreamNonBlocking) != hipSuccess) {
      sg.stream = nullptr;
      return MTG_ERR_HIP;
    }
  }
  if (sg.bytes < total) {
    if (sg.host) (void)hipHostFree(sg.host);
    if (sg.dev) (void)hipFree(sg.dev);
    sg.host = sg.hdev = sg.dev = nullptr;
    sg.bytes = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&sg.host), total, hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&sg.hdev), sg.host, 0) !=
            hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&sg.dev), total) != hipSuccess)
      return MTG_ERR_HIP;
    sg.bytes = total;
  }
  if (nfv) std::memcpy(sg.host, fixed_vals, nfv * sizeof(double));
  std::memcpy(sg.host + o_t, times, nt * sizeof(double));
  const bool zc = total <= kZeroCopyBytes;
  char* base = zc ? sg.hdev : sg.dev;
  if (!zc &&
      hipMemcpyAsync(sg.dev, sg.host, o_out, hipMemcpyHostToDevice, sg.stream) != hipSuccess)
    return MTG_ERR_HIP;
  auto d = [&](size_t off) { return reinterpret_cast<double*>(base + off); };
  int rc = from_hip(mtg::launch_linear_solve(
      pl, B, nfv ? d(0) : nullptr, d(o_t), d(o_out), d(o_cost), npv ? d(o_free) : nullptr,
      reinterpret_cast<int32_t*>(base + o_st), sg.stream));
  if (rc) return rc;
  if (!zc && hipMemcpyAsync(sg.host + o_out, sg.dev + o_out, total - o_out,
                            hipMemcpyDeviceToHost, sg.stream) != hipSuccess)
    return MTG_ERR_HIP;
  if (hipStreamSynchronize(sg.stream) != hipSuccess) return MTG_ERR_HIP;
  std::memcpy(coeffs, sg.host + o_out, nc * sizeof(double));
  if (cost) std::memcpy(cost, sg.host + o_cost, B * sizeof(double));
  if (free_vals && npv) std::memcpy(free_vals, sg.host + o_free, npv * sizeof(double));
  const int32_t* st = reinterpret_cast<const int32_t*>(sg.host + o_st);
  if (status) std::memcpy(status, st, B * sizeof(int32_t));
  for (int64_t b = 0; b < B; ++b)
    if (st[b] != MTG_TRAJ_OK) return MTG_ERR_NUMERIC;
  return MTG_OK;
}

int mtg_coeffs_from_constraints(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                                const double* free_vals, const double* times, double* coeffs,
                                double* cost, int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || B < 0 || B > 0x7fffffff || !times || !coeffs) return MTG_ERR_INVALID_ARG;
  if ((plan->dev.nf > 0 && !fixed_vals) || (plan->dev.np > 0 && !free_vals))
    return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_coeffs_from_constraints(plan->dev, B, fixed_vals, free_vals,
                                                      times, coeffs, cost, status,
                                                      static_cast<hipStream_t>(stream)));
}

int mtg_sample_trajectories(int N, int D, int S, int64_t B, const double* coeffs,
                            const double* times, double t_start, double t_end, double dt,
                            int n_max, int max_derivative, double* samples,
                            double* sample_times, int32_t* n_samples, void* stream) {
  clear_stale_error();
  if (!valid_N(N) || D < 1 || D > mtg::kMaxD || S < 1 || S > mtg::kMaxSampleS || B < 0 ||
      B > 65535 || n_max < 0 || max_derivative < 0 || max_derivative >= N || !(dt > 0.0) ||
      !(t_start >= 0.0))
    return MTG_ERR_INVALID_ARG;
  if (B == 0 || n_max == 0) return MTG_OK;
  if (!coeffs || !times || !samples) return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_sample(N, D, S, B, coeffs, times, t_start, t_end, dt, n_max,
                                     max_derivative, samples, sample_times, n_samples,
                                     static_cast<hipStream_t>(stream)));
}

int mtg_magnitude_candidates(int N, int D, int S, int64_t B, const double* coeffs,
                             const double* times, int derivative, int max_candidates,
                             double* cand_time, double* cand_value, int32_t* n_candidates,
                             void* stream) {
  clear_stale_error();
  if (!valid_N(N) || D < 1 || D > mtg::kMaxD || S < 1 || B < 0 || derivative < 0 ||
      derivative > mtg::kMaxExtremaDerivative || N - derivative - 1 <= 0 || max_candidates < 2)
    return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!coeffs || !times || !cand_time || !cand_value || !n_candidates) return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_magnitude_candidates(N, D, B * S, derivative, coeffs, times,
                                                   max_candidates, cand_time, cand_value,
                                                   n_candidates,
                                                   static_cast<hipStream_t>(stream)));
}

int mtg_max_magnitude(int N, int D, int S, int64_t B, const double* coeffs,
                      const double* times, int derivative, double* max_time,
                      double* max_value, int32_t* max_segment, void* stream) {
  clear_stale_error();
  if (!valid_N(N) || D < 1 || D > mtg::kMaxD || S < 1 || S > 256 || B < 0 || derivative < 0 ||
      derivative > mtg::kMaxExtremaDerivative || N - derivative - 1 <= 0)
    return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!coeffs || !times) return MTG_ERR_INVALID_ARG;
  const mtg::SoftCostArgs none{};
  return from_hip(mtg::launch_max_magnitude(N, D, S, B, derivative, coeffs, times, max_time,
                                            max_value, max_segment, 1, 0, none,
                                            static_cast<hipStream_t>(stream)));
}

// The map / potential / sampling parameters shared by the collision entry
// points.
static bool valid_collision_params(const mtg_collision_params& p, int nx, int ny, int nz) {
  return p.map_resolution > 0.0 && p.epsilon > 0.0 && p.coll_check_time_increment > 0.0 &&
         p.robot_radius >= 0.0 && p.box_side >= 1 && p.box_side <= 256 && nx >= 0 && ny >= 0 &&
         nz >= 0;
}

int mtg_collision_cost(const mtg_plan* plan, int64_t B, const double* coeffs,
                       const double* times, const float* occupancy, int nx, int ny, int nz,
                       const mtg_collision_params* params, double* cost, int32_t* collision,
                       double* grad_coeffs, double* grad_free, void* stream) {
  clear_stale_error();
  if (!plan || !params || B < 0 || B > 0x7fffffff || plan->dev.D != 3) return MTG_ERR_INVALID_ARG;
  const mtg_collision_params& p = *params;
  if (!valid_collision_params(p, nx, ny, nz)) return MTG_ERR_INVALID_ARG;
  if (mtg::collision_lds_bytes(plan->dev.N, plan->dev.S) > 65536) return MTG_ERR_UNSUPPORTED;
  if (B == 0) return MTG_OK;
  if (!coeffs || !times || (!occupancy && static_cast<int64_t>(nx) * ny * nz > 0))
    return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_collision_cost(plan->dev, B, coeffs, times, occupancy, nx, ny, nz,
                                             p, cost, collision, grad_coeffs, grad_free,
                                             static_cast<hipStream_t>(stream)));
}

int mtg_min_max_magnitude(int N, int D, int S, int64_t B, const double* coeffs,
                          const double* times, int derivative, double* min_time,
                          double* min_value, int32_t* min_segment, double* max_time,
                          double* max_value, int32_t* max_segment, void* stream) {
  clear_stale_error();
  if (!valid_N(N) || D < 1 || D > mtg::kMaxD || S < 1 || S > 256 || B < 0 || derivative < 0 ||
      derivative > mtg::kMaxExtremaDerivative || N - derivative - 1 <= 0)
    return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!coeffs || !times) return MTG_ERR_INVALID_ARG;
  const mtg::SoftCostArgs none{};
  const mtg::MinOut mino{min_time, min_value, min_segment};
  return from_hip(mtg::launch_max_magnitude(N, D, S, B, derivative, coeffs, times, max_time,
                                            max_value, max_segment, 1, 0, none,
                                            static_cast<hipStream_t>(stream), &mino));
}

int mtg_soft_constraint_cost(int N, int D, int S, int64_t B, const double* coeffs,
                             const double* times, int n_constraints, const int* derivatives,
                             const double* limits, double weight, double maximum_cost,
                             double* maxima, double* cost, void* stream) {
  clear_stale_error();
  if (!valid_N(N) || D < 1 || D > mtg::kMaxD || S < 1 || S > 256 || B < 0 ||
      n_constraints < 1 || n_constraints > mtg::kMaxSoftConstraints || !derivatives ||
      !limits)
    return MTG_ERR_INVALID_ARG;
  mtg::SoftSpec spec{};
  spec.n = n_constraints;
  spec.weight = weight;
  spec.maximum_cost = maximum_cost;
  for (int c = 0; c < n_constraints; ++c) {
    // addMaximumMagnitudeConstraint: CHECK_GE(derivative, 0), CHECK_GE(value, 0)
    if (derivatives[c] < 0 || derivatives[c] > mtg::kMaxExtremaDerivative ||
        N - derivatives[c] - 1 <= 0 || !(limits[c] >= 0.0))
      return MTG_ERR_INVALID_ARG;
    spec.derivative[c] = derivatives[c];
    spec.limit[c] = limits[c];
  }
  if (B == 0) return MTG_OK;
  if (!coeffs || !times || !maxima || !cost) return MTG_ERR_INVALID_ARG;
  if (B > 0x7fffffff) return MTG_ERR_INVALID_ARG;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  // Small batches are latency-bound: all constraints in one launch (measured
  // 69.6 -> 43.8 us at B = 1024, 2 constraints).  Large batches are
  // throughput-bound and pack 3 trajectories per workgroup in the
  // per-constraint kernel (74 vs 48 M evaluations/s at B = 65 536).
  return from_hip(mtg::launch_soft_cost_any(N, D, S, B, coeffs, times, spec, maxima, cost, st));
}

static bool valid_coll_params(const mtg_plan* plan, int mode, const mtg_coll_params* p) {
  if (!plan || !p || (mode != 0 && mode != 1) || plan->dev.D != 3 || plan->dev.np < 1)
    return false;
  if (p->lbfgs_memory < 1 || p->lbfgs_memory > 16 || p->n_soft < 0 ||
      p->n_soft > mtg::kMaxSoftConstraints)
    return false;
  if (mode == 1 && !(p->increment_time > 0.0)) return false;
  for (int c = 0; c < p->n_soft; ++c)
    if (p->soft_derivative[c] < 0 || p->soft_derivative[c] > mtg::kMaxExtremaDerivative ||
        plan->dev.N - p->soft_derivative[c] - 1 <= 0 || !(p->soft_limit[c] > 0.0))
      return false;
  if (mtg::collision_lds_bytes(plan->dev.N, plan->dev.S) > 65536) return false;
  return true;
}

int64_t mtg_coll_workspace_bytes(const mtg_plan* plan, int64_t B, int mode,
                                 const mtg_coll_params* params, int optimize) {
  if (B < 0 || !valid_coll_params(plan, mode, params)) return MTG_ERR_INVALID_ARG;
  if (mtg::coll_problems(plan->dev, B, mode, *params) > 0x7fffffff) return MTG_ERR_INVALID_ARG;
  return static_cast<int64_t>(
      mtg::coll_workspace_bytes(plan->dev, B, mode, *params, optimize != 0));
}

int64_t mtg_coll_field_bytes(int nx, int ny, int nz) {
  if (nx < 0 || ny < 0 || nz < 0) return MTG_ERR_INVALID_ARG;
  return static_cast<int64_t>(nx) * ny * nz * mtg::kFieldSlots * sizeof(uint16_t);
}

int mtg_coll_field(const float* occupancy, int nx, int ny, int nz,
                   const mtg_collision_params* params, uint16_t* field, void* stream) {
  clear_stale_error();
  if (!params || !valid_collision_params(*params, nx, ny, nz) ||
      !mtg::coll_field_supported(params->box_side))
    return MTG_ERR_INVALID_ARG;
  if (static_cast<int64_t>(nx) * ny * nz == 0) return MTG_OK;
  if (!occupancy || !field) return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_coll_field(occupancy, nx, ny, nz, params->box_side, field,
                                         static_cast<hipStream_t>(stream)));
}

int mtg_coll_cost(const mtg_plan* plan, int64_t B, int mode, const double* fixed_vals,
                  const double* x, const double* times, const float* occupancy, int nx,
                  int ny, int nz, const uint16_t* near_field, const mtg_coll_params* params,
                  const double* raise_ref,
                  double* cost, double* grad, double* terms, int32_t* collision,
                  int32_t* status, void* workspace, size_t workspace_bytes, void* stream) {
  clear_stale_error();
  if (B < 0 || !valid_coll_params(plan, mode, params) ||
      !valid_collision_params(params->coll, nx, ny, nz))
    return MTG_ERR_INVALID_ARG;
  if (mtg::coll_problems(plan->dev, B, mode, *params) > 0x7fffffff) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!fixed_vals || !x || (mode == 0 && !times) || !workspace ||
      (!occupancy && static_cast<int64_t>(nx) * ny * nz > 0))
    return MTG_ERR_INVALID_ARG;
  return mtg::coll_cost(plan->dev, B, mode, fixed_vals, x, times, occupancy, nx, ny, nz,
                        near_field, *params, raise_ref, cost, grad, terms, collision, status, workspace,
                        workspace_bytes, static_cast<hipStream_t>(stream));
}

int mtg_coll_optimize_trace(const mtg_plan* plan, int64_t B, int mode, const double* fixed_vals,
                            double* x_io, const double* times, const double* lower,
                            const double* upper, const double* initial_step,
                            const float* occupancy, int nx, int ny, int nz,
                            const uint16_t* near_field, const mtg_coll_params* params,
                            int max_evals, double* cost, int32_t* evals, int32_t* result,
                            int32_t* status, double* terms, double* x_history, void* workspace,
                            size_t workspace_bytes, void* stream) {
  clear_stale_error();
  if (B < 0 || max_evals < 1 || !valid_coll_params(plan, mode, params) ||
      !valid_collision_params(params->coll, nx, ny, nz))
    return MTG_ERR_INVALID_ARG;
  if (mtg::coll_problems(plan->dev, B, mode, *params) > 0x7fffffff) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!fixed_vals || !x_io || (mode == 0 && !times) || !workspace ||
      (!occupancy && static_cast<int64_t>(nx) * ny * nz > 0))
    return MTG_ERR_INVALID_ARG;
  return mtg::coll_optimize(plan->dev, B, mode, fixed_vals, x_io, times, lower, upper,
                            initial_step, occupancy, nx, ny, nz, near_field, *params, max_evals,
                            cost, evals,
                            result, status, terms, x_history, workspace, workspace_bytes,
                            static_cast<hipStream_t>(stream));
}

int mtg_coll_optimize(const mtg_plan* plan, int64_t B, int mode, const double* fixed_vals,
                      double* x_io, const double* times, const double* lower,
                      const double* upper, const double* initial_step, const float* occupancy,
                      int nx, int ny, int nz, const uint16_t* near_field,
                      const mtg_coll_params* params, int max_evals,
                      double* cost, int32_t* evals, int32_t* result, int32_t* status,
                      double* terms, void* workspace, size_t workspace_bytes, void* stream) {
  clear_stale_error();
  return mtg_coll_optimize_trace(plan, B, mode, fixed_vals, x_io, times, lower, upper,
                                 initial_step, occupancy, nx, ny, nz, near_field, params,
                                 max_evals, cost, evals, result, status, terms, nullptr, workspace,
                                 workspace_bytes, stream);
}

int mtg_select_local(const double* costs, int64_t count, int64_t start, int rank, double* out,
                     void* stream) {
  clear_stale_error();
  if (count < 0 || start < 0 || rank < 0 || !out || (count > 0 && !costs))
    return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_select_local(costs, count, start, rank, out,
                                           static_cast<hipStream_t>(stream)));
}

// Workspace of the fused selection: the counter, then the per-workgroup
// (cost, index) partials, 256-byte aligned.
static size_t select_ws_layout(const mtg_plan* plan, int64_t B, size_t* off_cost,
                               size_t* off_idx) {
  const int64_t parts = mtg::select_partials(plan->dev, B);
  *off_cost = 0;
  *off_idx = (sizeof(double) * static_cast<size_t>(parts) + 255) & ~size_t(255);
  return parts > 0 ? *off_idx + sizeof(int64_t) * static_cast<size_t>(parts) : 0;
}

int64_t mtg_select_workspace_bytes(const mtg_plan* plan, int64_t B) {
  if (!plan || B < 0) return MTG_ERR_INVALID_ARG;
  size_t a, b;
  return static_cast<int64_t>(select_ws_layout(plan, B, &a, &b));
}

int mtg_linear_solve_select(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                            const double* times, double* coeffs, double* cost,
                            double* free_vals, int32_t* status, int64_t start, int rank,
                            double* triple, void* workspace, size_t workspace_bytes,
                            void* stream) {
  clear_stale_error();
  if (!plan || B < 0 || B > 0x7fffffff || start < 0 || rank < 0 || !triple)
    return MTG_ERR_INVALID_ARG;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0) return from_hip(mtg::launch_select_local(nullptr, 0, start, rank, triple, st));
  if (!fixed_vals || !times || !coeffs || !cost) return MTG_ERR_INVALID_ARG;
  size_t oc, oi;
  const size_t need = select_ws_layout(plan, B, &oc, &oi);
  if (need > workspace_bytes || (need > 0 && !workspace)) return MTG_ERR_INVALID_ARG;
  char* w = static_cast<char*>(workspace);
  mtg::SelectArgs sel;
  sel.start = start;
  sel.rank = rank;
  sel.out = triple;
  sel.part_cost = reinterpret_cast<double*>(w + oc);
  sel.part_idx = reinterpret_cast<int64_t*>(w + oi);
  return from_hip(mtg::launch_linear_solve(plan->dev, B, fixed_vals, times, coeffs, cost,
                                           free_vals, status, st, sel));
}

int mtg_linear_solve_select_prev(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                                 const double* times, double* coeffs, double* cost,
                                 double* free_vals, int32_t* status, const double* prev_cost,
                                 int64_t prev_count, int64_t prev_start, int rank,
                                 double* prev_triple, void* stream) {
  clear_stale_error();
  if (!plan || B < 0 || B > 0x7fffffff || rank < 0 || prev_count < 0 || prev_start < 0)
    return MTG_ERR_INVALID_ARG;
  if (prev_cost && !prev_triple) return MTG_ERR_INVALID_ARG;
  if (prev_cost && cost && prev_cost == cost) return MTG_ERR_INVALID_ARG;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  if (B == 0) {  // no solve launch to ride on
    if (!prev_cost) return MTG_OK;
    return from_hip(mtg::launch_select_local(prev_cost, prev_count, prev_start, rank,
                                             prev_triple, st));
  }
  if (!times || !coeffs || (plan->dev.nf > 0 && !fixed_vals)) return MTG_ERR_INVALID_ARG;
  mtg::SelectArgs sel;
  sel.rank = rank;
  if (prev_cost) {
    sel.prev_cost = prev_cost;
    sel.prev_count = prev_count;
    sel.prev_start = prev_start;
    sel.prev_out = prev_triple;
  }
  return from_hip(mtg::launch_linear_solve(plan->dev, B, fixed_vals, times, coeffs, cost,
                                           free_vals, status, st, sel));
}

int mtg_select_global_steps(const double* triples, int world, int G, int n, double* out,
                            void* stream) {
  clear_stale_error();
  if (world < 1 || G < 1 || n < 0 || n > G || (n > 0 && (!triples || !out)))
    return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_select_global_steps(triples, world, G, n, out,
                                                  static_cast<hipStream_t>(stream)));
}

int mtg_select_global(const double* triples, int world, double* out, void* stream) {
  clear_stale_error();
  if (world < 1 || !triples || !out) return MTG_ERR_INVALID_ARG;
  return from_hip(mtg::launch_select_global(triples, world, out,
                                            static_cast<hipStream_t>(stream)));
}

int mtg_segment_matrices(mtg_ctx* ctx, int N, int r, int64_t n, const double* times,
                         double* Q, double* A, double* Ainv, double* H, void* stream) {
  clear_stale_error();
  if (!ctx || !valid_N(N) || r < 0 || r > N / 2 - 1 || n < 0 || (n && !times))
    return MTG_ERR_INVALID_ARG;
  if (n == 0) return MTG_OK;
  const double* tab = nullptr;
  int rc = get_tables(ctx, N, r, &tab);
  if (rc) return rc;
  return from_hip(mtg::launch_segment_matrices(N, r, n, tab, times, Q, A, Ainv, H,
                                               static_cast<hipStream_t>(stream)));
}

// Soft constraints of mtg_time_params: addMaximumMagnitudeConstraint's
// CHECK_GE(derivative, 0), CHECK_GE(maximum_value, 0) (nonlinear_impl:849-850),
// the POSITION..SNAP switch (:2697-2724), N - derivative - 1 > 0
// (linear_impl:400) and a nonzero limit (the cost divides by it, :2754).
// allow_hard: the entry point implements hard_constraints (mtg_time_cost /
// mtg_time_optimize); elsewhere hard_constraints must be 0.
static bool valid_soft(const mtg_plan* plan, const mtg_time_params* p, bool allow_hard = false) {
  if (p->n_soft < 0 || p->n_soft > mtg::kMaxSoftConstraints) return false;
  if (p->hard_constraints != 0 && (!allow_hard || p->hard_constraints != 1)) return false;
  if (p->hard_constraints && !(p->hard_tolerance >= 0.0 && p->hard_tolerance < 1e300))
    return false;
  if (p->n_soft > 0 && plan->dev.S > 256) return false;
  for (int c = 0; c < p->n_soft; ++c) {
    const int k = p->soft_derivative[c];
    if (k < 0 || k > mtg::kMaxExtremaDerivative || plan->dev.N - k - 1 <= 0) return false;
    if (!(p->soft_limit[c] > 0.0)) return false;
  }
  return true;
}

int mtg_free_cost(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                  const double* free_vals, const double* times, const mtg_time_params* params,
                  int mode, double* cost, double* grad, int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || !params || B < 0 || B > 0x7fffffff || !times || mode < 0 || mode > 1)
    return MTG_ERR_INVALID_ARG;
  if ((plan->dev.nf > 0 && !fixed_vals) || (plan->dev.np > 0 && !free_vals))
    return MTG_ERR_INVALID_ARG;
  if (!valid_soft(plan, params)) return MTG_ERR_INVALID_ARG;
  if (mtg::free_lds_bytes(plan->dev.N, plan->dev.S, plan->dev.D, plan->dev.np,
                          params->n_soft > 0) > static_cast<size_t>(mtg::kMaxLdsBytes))
    return MTG_ERR_UNSUPPORTED;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_free_cost(plan->dev, B, fixed_vals, free_vals, times, *params,
                                        mode, cost, mode == 0 ? grad : nullptr, status,
                                        static_cast<hipStream_t>(stream)));
}

int mtg_time_free_optimize_ex(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                              double* free_io, double* times_io, const mtg_time_params* params,
                              int max_evals, double* cost, int32_t* evals, int32_t* result,
                              int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || !params || B < 0 || B > 0x7fffffff || !times_io || max_evals < 1)
    return MTG_ERR_INVALID_ARG;
  if ((plan->dev.nf > 0 && !fixed_vals) || plan->dev.np < 1 || !free_io)
    return MTG_ERR_INVALID_ARG;
  if (params->optimizer != 0 && params->optimizer != 1) return MTG_ERR_INVALID_ARG;
  if (params->optimizer == 0 && !(params->increment > 0)) return MTG_ERR_INVALID_ARG;
  if (!valid_soft(plan, params)) return MTG_ERR_INVALID_ARG;
  const bool soft = params->n_soft > 0;
  const PlanDev& pl = plan->dev;
  const size_t lds = params->optimizer == 1
                         ? mtg::free_sbplx_lds_bytes(pl.N, pl.S, pl.D, pl.np, soft)
                         : mtg::free_lds_bytes(pl.N, pl.S, pl.D, pl.np, soft);
  if (lds > static_cast<size_t>(mtg::kMaxLdsBytes)) return MTG_ERR_UNSUPPORTED;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_time_free_optimize(pl, B, fixed_vals, free_io, times_io, *params,
                                                 max_evals, cost, evals, result, status,
                                                 static_cast<hipStream_t>(stream)));
}

int mtg_time_free_optimize(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                           double* free_io, double* times_io, const mtg_time_params* params,
                           int max_evals, double* cost, int32_t* evals, int32_t* status,
                           void* stream) {
  return mtg_time_free_optimize_ex(plan, B, fixed_vals, free_io, times_io, params, max_evals,
                                   cost, evals, nullptr, status, stream);
}

int mtg_free_optimize(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                      double* free_io, const double* times, const double* lower,
                      const double* upper, const mtg_time_params* params, int max_evals,
                      double* cost, int32_t* evals, int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || !params || B < 0 || B > 0x7fffffff || !times || max_evals < 1)
    return MTG_ERR_INVALID_ARG;
  if ((plan->dev.nf > 0 && !fixed_vals) || plan->dev.np < 1 || !free_io)
    return MTG_ERR_INVALID_ARG;
  if (!valid_soft(plan, params)) return MTG_ERR_INVALID_ARG;
  if (mtg::free_lds_bytes(plan->dev.N, plan->dev.S, plan->dev.D, plan->dev.np,
                          params->n_soft > 0) > static_cast<size_t>(mtg::kMaxLdsBytes))
    return MTG_ERR_UNSUPPORTED;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_free_optimize(plan->dev, B, fixed_vals, free_io, times, lower,
                                            upper, *params, max_evals, cost, evals, status,
                                            static_cast<hipStream_t>(stream)));
}

int mtg_time_cost(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                  const double* times, const mtg_time_params* params, double* cost,
                  double* grad, int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || !params || B < 0 || B > 0x7fffffff || !times) return MTG_ERR_INVALID_ARG;
  if (params->grad_mode < 0 || params->grad_mode > 2) return MTG_ERR_INVALID_ARG;
  if (params->grad_mode && !(params->increment > 0)) return MTG_ERR_INVALID_ARG;
  if (!valid_soft(plan, params, true)) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_time_cost(plan->dev, B, fixed_vals, times, *params, cost, grad,
                                        status, static_cast<hipStream_t>(stream)));
}

int mtg_time_optimize_ex(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                         double* times_io, const mtg_time_params* params, int max_evals,
                         double* cost, int32_t* evals, int32_t* solves, int32_t* result,
                         int32_t* status, void* stream) {
  clear_stale_error();
  if (!plan || !params || B < 0 || B > 0x7fffffff || !times_io || max_evals < 1)
    return MTG_ERR_INVALID_ARG;
  if (!(params->increment > 0)) return MTG_ERR_INVALID_ARG;
  if (!valid_soft(plan, params, true)) return MTG_ERR_INVALID_ARG;
  if (params->optimizer != 0 && params->optimizer != 1) return MTG_ERR_INVALID_ARG;
  // LN_SBPLX takes no inequality constraints (NLopt rejects them)
  if (params->optimizer == 1 && params->hard_constraints && params->n_soft > 0)
    return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_time_optimize(plan->dev, B, fixed_vals, times_io, *params,
                                            max_evals, cost, evals, solves, result, status,
                                            static_cast<hipStream_t>(stream)));
}

int mtg_time_optimize(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                      double* times_io, const mtg_time_params* params, int max_evals,
                      double* cost, int32_t* evals, int32_t* solves, int32_t* status,
                      void* stream) {
  return mtg_time_optimize_ex(plan, B, fixed_vals, times_io, params, max_evals, cost, evals,
                              solves, nullptr, status, stream);
}

int mtg_tube_num_constraints(int N, int S) {
  if (!valid_N(N) || S < 1) return MTG_ERR_INVALID_ARG;
  return (S - 1) + S * (N - 2) + 2 * S * (N - 2);
}

// One 64-lane workgroup per QCQP problem: the launch must stay below 2^32
// work-items (and 2^32 workgroups), and the B x P x S point arrays below
// 2^31 entries.
static bool tube_grid_ok(int S, int64_t problems) {
  return problems >= 0 && problems < (int64_t(1) << 26) &&
         problems * static_cast<int64_t>(S) < (int64_t(1) << 31);
}

static int tube_args(mtg_ctx* ctx, int N, int r, int S, int64_t B, const double* positions,
                     const double* fixed_vals, const double* times_cp, const double* times,
                     const double* radii, mtg::TubeArgs* a) {
  if (!ctx || !valid_N(N) || r < 0 || r > N / 2 - 1 || S < 2 || !tube_grid_ok(S, B))
    return MTG_ERR_INVALID_ARG;
  if (B && (!positions || !fixed_vals || !times_cp || !times || !radii))
    return MTG_ERR_INVALID_ARG;
  if (mtg::tube_lds_bytes(N, S) > static_cast<size_t>(mtg::kMaxLdsBytes))
    return MTG_ERR_UNSUPPORTED;
  const double* tab = nullptr;
  int rc = get_tables(ctx, N, r, &tab);
  if (rc) return rc;
  *a = mtg::TubeArgs{N, r, S, B, tab, positions, fixed_vals, times_cp, times, radii};
  return MTG_OK;
}

int mtg_tube_residuals(mtg_ctx* ctx, int N, int r, int S, int64_t B, const double* positions,
                       const double* fixed_vals, const double* times_cp, const double* times,
                       const double* radii, const double* x, double* resid, void* stream) {
  clear_stale_error();
  mtg::TubeArgs a;
  int rc = tube_args(ctx, N, r, S, B, positions, fixed_vals, times_cp, times, radii, &a);
  if (rc) return rc;
  if (B && (!x || !resid)) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_tube_residuals(a, x, resid, static_cast<hipStream_t>(stream)));
}

int mtg_tube_solve(mtg_ctx* ctx, int N, int r, int S, int64_t B, const double* positions,
                   const double* fixed_vals, const double* times_cp, const double* times,
                   const double* radii, double tol, int max_iter, double* x, double* coeffs,
                   double* cost, int32_t* iters, int32_t* status, void* stream) {
  clear_stale_error();
  mtg::TubeArgs a;
  int rc = tube_args(ctx, N, r, S, B, positions, fixed_vals, times_cp, times, radii, &a);
  if (rc) return rc;
  if (B && !coeffs) return MTG_ERR_INVALID_ARG;
  if (!(tol > 0) || max_iter < 1) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  return from_hip(mtg::launch_tube_solve(a, tol, max_iter, x, coeffs, cost, iters, status,
                                         static_cast<hipStream_t>(stream)));
}

static bool valid_tube_time_params(int N, int S, const mtg_time_params* p) {
  if (!p || p->n_soft < 0 || p->n_soft > mtg::kMaxSoftConstraints) return false;
  if (p->hard_constraints != 0) return false;
  if (p->n_soft > 0 && S > 256) return false;
  for (int c = 0; c < p->n_soft; ++c) {
    const int k = p->soft_derivative[c];
    if (k < 0 || k > mtg::kMaxExtremaDerivative || N - k - 1 <= 0) return false;
    if (!(p->soft_limit[c] > 0.0)) return false;
  }
  return p->increment > 0.0;
}

int64_t mtg_tube_time_workspace_bytes(int N, int S, int64_t B, const mtg_time_params* params,
                                      int optimize) {
  if (!valid_N(N) || S < 2 || B < 0 || !valid_tube_time_params(N, S, params))
    return MTG_ERR_INVALID_ARG;
  if (!tube_grid_ok(S, mtg::tube_time_problems(S, B, *params, optimize != 0)))
    return MTG_ERR_INVALID_ARG;
  return static_cast<int64_t>(mtg::tube_time_workspace_bytes(N, S, B, *params, optimize != 0));
}

int mtg_tube_time_cost(mtg_ctx* ctx, int N, int r, int S, int64_t B, const double* positions,
                       const double* fixed_vals, const double* times_cp, const double* times,
                       const double* radii, double tol, int max_iter,
                       const mtg_time_params* params, double* cost, double* grad,
                       int32_t* status, void* workspace, size_t workspace_bytes,
                       void* stream) {
  clear_stale_error();
  mtg::TubeArgs a;
  int rc = tube_args(ctx, N, r, S, B, positions, fixed_vals, times_cp, times, radii, &a);
  if (rc) return rc;
  if (!valid_tube_time_params(N, S, params) || !(tol > 0) || max_iter < 1)
    return MTG_ERR_INVALID_ARG;
  if (params->grad_mode == 1) return MTG_ERR_UNSUPPORTED;
  if (params->grad_mode != 0 && params->grad_mode != 2) return MTG_ERR_INVALID_ARG;
  if (params->grad_mode == 2 && B && !grad) return MTG_ERR_INVALID_ARG;
  if (B && !cost) return MTG_ERR_INVALID_ARG;
  if (!tube_grid_ok(S, mtg::tube_time_problems(S, B, *params, false)))
    return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!workspace) return MTG_ERR_INVALID_ARG;
  return mtg::tube_time_cost(a, tol, max_iter, *params, cost, grad, status, workspace,
                             workspace_bytes, static_cast<hipStream_t>(stream));
}

int mtg_tube_time_optimize_ex(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                              const double* positions, const double* fixed_vals,
                              const double* radii, double* times_io, double tol, int max_iter,
                              const mtg_time_params* params, int max_evals, double* cost,
                              int32_t* evals, int32_t* result, int32_t* status, void* workspace,
                              size_t workspace_bytes, void* stream) {
  clear_stale_error();
  // optimizer 0: the projected descent; 1: LN_SBPLX (the reference's default)
  if (params && params->optimizer != 0 && params->optimizer != 1) return MTG_ERR_INVALID_ARG;
  mtg::TubeArgs a;
  // times_cp = the initial times (read before the first write of times_io).
  int rc = tube_args(ctx, N, r, S, B, positions, fixed_vals, times_io, times_io, radii, &a);
  if (rc) return rc;
  if (!valid_tube_time_params(N, S, params) || !(tol > 0) || max_iter < 1 || max_evals < 1)
    return MTG_ERR_INVALID_ARG;
  if (!tube_grid_ok(S, mtg::tube_time_problems(S, B, *params, true))) return MTG_ERR_INVALID_ARG;
  if (B == 0) return MTG_OK;
  if (!workspace) return MTG_ERR_INVALID_ARG;
  return mtg::tube_time_optimize(a, times_io, tol, max_iter, *params, max_evals, cost, evals,
                                 result, status, workspace, workspace_bytes,
                                 static_cast<hipStream_t>(stream));
}

int mtg_tube_time_optimize(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                           const double* positions, const double* fixed_vals,
                           const double* radii, double* times_io, double tol, int max_iter,
                           const mtg_time_params* params, int max_evals, double* cost,
                           int32_t* evals, int32_t* status, void* workspace,
                           size_t workspace_bytes, void* stream) {
  return mtg_tube_time_optimize_ex(ctx, N, r, S, B, positions, fixed_vals, radii, times_io, tol,
                                   max_iter, params, max_evals, cost, evals, nullptr, status,
                                   workspace, workspace_bytes, stream);
}

int mtg_generate_random_problems(int N, int D, int S, int64_t B, uint64_t seed0,
                                 double pos_bound, double v_max, double a_max,
                                 uint8_t* fixed_mask, double* fixed_vals, double* times,
                                 double* positions) {
  using namespace mav_trajectory_generation;
  if (!valid_N(N) || D < 1 || S < 1 || B < 0 || !(pos_bound > 0) || !(v_max > 0) ||
      !(a_max > 0))
    return MTG_ERR_INVALID_ARG;
  const int M = N / 2;
  // Standard pattern: start/end fixed to order M-1, intermediates position.
  std::vector<uint8_t> mask((S + 1) * M, 0);
  for (int v = 0; v <= S; ++v)
    for (int k = 0; k < M; ++k) mask[v * M + k] = (v == 0 || v == S || k == 0) ? 1 : 0;
  if (fixed_mask) std::memcpy(fixed_mask, mask.data(), mask.size());
  const int nf = 2 * M + (S - 1);
  const VectorXd lo = VectorXd::Constant(D, -pos_bound), hi = VectorXd::Constant(D, pos_bound);
  for (int64_t b = 0; b < B; ++b) {
    Vertex::Vector vs = createRandomVertices(M - 1, S, lo, hi, seed0 + b);
    std::vector<double> t = estimateSegmentTimes(vs, v_max, a_max);
    if (times)
      for (int s = 0; s < S; ++s) times[b * S + s] = t[s];
    if (positions)
      for (int v = 0; v <= S; ++v) {
        VectorXd p;
        vs[v].getConstraint(derivative_order::POSITION, &p);
        for (int d = 0; d < D; ++d) positions[(b * (S + 1) + v) * D + d] = p[d];
      }
    if (fixed_vals) {
      int f = 0;
      for (int v = 0; v <= S; ++v)
        for (int k = 0; k < M; ++k) {
          if (!mask[v * M + k]) continue;
          VectorXd c;
          vs[v].getConstraint(k, &c);
          for (int d = 0; d < D; ++d) fixed_vals[(b * D + d) * nf + f] = c[d];
          ++f;
        }
    }
  }
  return MTG_OK;
}

}  // extern "C"
