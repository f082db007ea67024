// What a launch's output stores cost at C2's shape: 1024 one-wave
// workgroups each store W doubles (W = 0, 64, 300, 1200: 0, 0.5, 2.4, 9.6 MB
// per launch) with plain, non-temporal (`__builtin_nontemporal_store`) or
// write-through (agent-scope atomic store) 16-byte stores, after the same
// few microseconds of FP64 work.  K = 200 launches in one graph; per-launch
// time.  Tells whether the end-of-kernel writeback of dirty L2 lines is part
// of the C2 launch time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/store_tail tools/ubench/store_tail.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(64) void store_kernel(double* __restrict__ out, int W) {
  double x = 1.0 + threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < 600; ++i) x = fma(x, 0.9999999, 1e-9);
  double2* o = reinterpret_cast<double2*>(out + static_cast<size_t>(blockIdx.x) * W);
  for (int i = threadIdx.x; i < W / 2; i += 64) {
    const double2 v = make_double2(x + i, x - i);
    if constexpr (MODE == 0) {
      o[i] = v;
    } else if constexpr (MODE == 1) {
      __builtin_nontemporal_store(v.x, &o[i].x);
      __builtin_nontemporal_store(v.y, &o[i].y);
    } else {
      __hip_atomic_store(&o[i].x, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&o[i].y, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

#define CHECK(x)                                                 \
  do {                                                           \
    hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                      \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                                  \
    }                                                            \
  } while (0)

int main() {
  const int K = 200, G = 1024;
  double* out;
  CHECK(hipMalloc(&out, sizeof(double) * 1200 * G));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  for (int mode = 0; mode < 3; ++mode) {
    for (int W : {0, 64, 300, 1200}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int k = 0; k < K; ++k) {
        if (mode == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(G), dim3(64), 0, st, out, W);
        if (mode == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(G), dim3(64), 0, st, out, W);
        if (mode == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(G), dim3(64), 0, st, out, W);
      }
      CHECK(hipStreamEndCapture(st, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      for (int w = 0; w < 2; ++w) CHECK(hipGraphLaunch(ge, st));
      float best = 1e9f;
      for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0, st));
        CHECK(hipGraphLaunch(ge, st));
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      std::printf("%-13s W=%5d (%6.2f MB/launch): %.3f us per launch\n",
                  mode == 0 ? "plain" : (mode == 1 ? "nontemporal" : "write-through"), W,
                  8.0 * W * G / 1e6, 1000.0 * best / K);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
  }
  return 0;
}
