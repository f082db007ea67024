// Cost of finishing a batch-wide argmin inside the solve kernel instead of in
// a second launch: 1024 (or 8192) one-wave workgroups each write one cost,
// then
//   kind 0  nothing more (the solve kernel alone),
//   kind 1  + a separate one-workgroup reduction launch (today's selection),
//   kind 2  + relaxed device-scope atomicAdd on one counter; the last
//           arriver reduces all costs (loads that bypass the non-coherent
//           L2) and resets the counter,
//   kind 3  as 2, with the cost stored through to memory and the store
//           waited for before the atomic (no L2 writeback fence),
//   kind 4  as 2, with __threadfence() (release, L2 writeback) before it,
//   kind 5  only a same-address 64-bit atomicMin per workgroup.
// Per-launch times over K launches captured in one HIP graph.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/last_arriver tools/ubench/last_arriver.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kK = 50;

__device__ inline double work(int b) {
  // A little FP64 so the waves do not all finish in the same cycle.
  double x = 1.0 + b * 1e-6;
#pragma unroll 1
  for (int i = 0; i < 200 + (b & 63); ++i) x = fma(x, 0.999999, 1e-7);
  return x;
}

__device__ inline double ld_nc(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_nc(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The last arriver's reduction: wave 0 of that workgroup reads all n costs.
__device__ void reduce_all(const double* cost, int n, double* out) {
  double best = HUGE_VAL;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += 64) {
    const double c = ld_nc(cost + i);
    if (c < best || (c == best && i < bi)) {
      best = c;
      bi = i;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double c2 = __shfl_xor(best, off, 64);
    const int i2 = __shfl_xor(bi, off, 64);
    if (c2 < best || (c2 == best && i2 < bi)) {
      best = c2;
      bi = i2;
    }
  }
  if (threadIdx.x == 0) {
    out[0] = best;
    out[1] = bi;
  }
}

template <int KIND>
__global__ __launch_bounds__(64) void solve_like(double* cost, unsigned* counter, double* out) {
  const int b = blockIdx.x, n = gridDim.x;
  const double c = work(b);
  if (KIND == 0 || KIND == 1 || KIND == 2 || KIND == 4) {
    if (threadIdx.x == 0) cost[b] = c;
  } else {
    if (threadIdx.x == 0) st_nc(cost + b, c);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (KIND < 2) return;
  if (KIND == 4) __threadfence();
  unsigned last = 0;
  if (KIND == 5) {
    // Only a same-address 64-bit atomicMin per workgroup (its throughput).
    if (threadIdx.x == 0)
      __hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(counter + 64),
                             static_cast<unsigned long long>(__double_as_longlong(c)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  } else if (threadIdx.x == 0) {
    const unsigned t =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == static_cast<unsigned>(n - 1);
  }
  last = __shfl(last, 0, 64);
  if (!last) return;
  reduce_all(cost, n, out);
  if (threadIdx.x == 0) {
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(64) void reduce_kernel(const double* cost, int n, double* out) {
  reduce_all(cost, n, out);
}

#define CHECK(x)                                                 \
  do {                                                           \
    hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                      \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                                  \
    }                                                            \
  } while (0)

template <int KIND>
void launch(int n, double* cost, unsigned* counter, double* out, hipStream_t st) {
  hipLaunchKernelGGL(solve_like<KIND>, dim3(n), dim3(64), 0, st, cost, counter, out);
  if (KIND == 1) hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(64), 0, st, cost, n, out);
}

int main() {
  double *cost, *out;
  unsigned* counter;
  CHECK(hipMalloc(&cost, sizeof(double) * 8192));
  CHECK(hipMalloc(&out, sizeof(double) * 2));
  CHECK(hipMalloc(&counter, sizeof(unsigned) * 256));
  CHECK(hipMemset(counter, 0, sizeof(unsigned) * 256));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  for (int n : {1024, 8192}) {
    for (int kind = 0; kind < 6; ++kind) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int k = 0; k < kK; ++k) {
        switch (kind) {
          case 0: launch<0>(n, cost, counter, out, st); break;
          case 1: launch<1>(n, cost, counter, out, st); break;
          case 2: launch<2>(n, cost, counter, out, st); break;
          case 3: launch<3>(n, cost, counter, out, st); break;
          case 4: launch<4>(n, cost, counter, out, st); break;
          default: launch<5>(n, cost, counter, out, st); break;
        }
      }
      CHECK(hipStreamEndCapture(st, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      for (int w = 0; w < 3; ++w) CHECK(hipGraphLaunch(ge, st));
      CHECK(hipEventRecord(e0, st));
      for (int r = 0; r < 5; ++r) CHECK(hipGraphLaunch(ge, st));
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      double h[2];
      CHECK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
      unsigned cnt;
      CHECK(hipMemcpy(&cnt, counter, sizeof(cnt), hipMemcpyDeviceToHost));
      std::printf("n=%d kind=%d: %.3f us per step  (argmin %.0f, counter %u)\n", n, kind,
                  1000.0 * ms / (5 * kK), h[1], cnt);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
      CHECK(hipMemset(out, 0, sizeof(double) * 2));
    }
  }
  return 0;
}
