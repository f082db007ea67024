// Fixed cost of one graph replay (the bench's timing method): K launches of
// a one-wave-per-workgroup kernel (1024 workgroups, ~2 us of work each)
// captured in one graph, timed by events around hipGraphLaunch, for K = 20
// and 200, with and without hipGraphUpload before the timed launch, and with
// a 50 us busy kernel queued just before the start event (so the graph's
// submission overlaps it); round 5: with the timing events created with
// hipEventDisableSystemFence / hipEventReleaseToDevice (no system-scope
// cache writeback and invalidation when an event is recorded), and the K
// launches eager (not captured) behind the busy kernel.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/graph_fixed tools/ubench/graph_fixed.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void work_kernel(double* out) {
  double x = 1.0 + threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < 400; ++i) x = fma(x, 0.9999999, 1e-9);
  if (x == 0.0) out[blockIdx.x] = x;  // never: keeps the loop
}

__global__ void busy_kernel(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
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
  double* out;
  CHECK(hipMalloc(&out, 8192 * 8));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  for (int K : {20, 200}) {
    for (int mode = 0; mode < 6; ++mode) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(work_kernel, dim3(1024), dim3(64), 0, st, out);
      CHECK(hipStreamEndCapture(st, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      if (mode == 1) CHECK(hipGraphUpload(ge, st));
      hipEvent_t e0, e1;
      const unsigned ef = mode == 3 ? hipEventDisableSystemFence
                          : mode == 4 ? hipEventReleaseToDevice : hipEventDefault;
      CHECK(hipEventCreateWithFlags(&e0, ef));
      CHECK(hipEventCreateWithFlags(&e1, ef));
      for (int w = 0; w < 3; ++w) CHECK(hipGraphLaunch(ge, st));
      CHECK(hipStreamSynchronize(st));
      float best = 1e9f, sum = 0.0f;
      for (int r = 0; r < 10; ++r) {
        if (mode == 2 || mode == 5)
          hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, st, (mode == 5 ? 400LL : 50LL) * 2400);
        CHECK(hipEventRecord(e0, st));
        if (mode == 5) {
          for (int k = 0; k < K; ++k)
            hipLaunchKernelGGL(work_kernel, dim3(1024), dim3(64), 0, st, out);
        } else {
          CHECK(hipGraphLaunch(ge, st));
        }
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
      }
      std::printf("K=%3d mode=%s: best %.3f us/launch, mean %.3f us/launch\n", K,
                  mode == 0   ? "plain "
                  : mode == 1 ? "upload"
                  : mode == 2 ? "busy  "
                  : mode == 3 ? "nofence"
                  : mode == 4 ? "reldev"
                              : "eager ",
                  1000.0 * best / K,
                  1000.0 * sum / 10 / K);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
  }
  return 0;
}
