// Launch floor of back-to-back kernels in one HIP graph (the bench's timing
// method): per-launch time of an empty kernel and of a one-load-one-store
// kernel over 1024 / 8192 one-wave workgroups, and the empty kernel with
// the same waves in four-wave workgroups.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_floor tools/ubench/launch_floor.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void empty_kernel() {}
__global__ void copy_kernel(const double* __restrict__ a, double* __restrict__ b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  b[i] = a[i] + 1.0;
}

#define CHECK(x)                                                           \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const int K = 50;
  double *a, *b;
  CHECK(hipMalloc(&a, sizeof(double) * 8192 * 64));
  CHECK(hipMalloc(&b, sizeof(double) * 8192 * 64));
  CHECK(hipMemset(a, 0, sizeof(double) * 8192 * 64));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  // kind 2: the 1024 one-wave workgroups as 256 workgroups of four waves.
  for (int kind = 0; kind < 3; ++kind) {
    for (int blocks : {1024, 8192}) {
      const int wg = kind == 2 ? 256 : 64;
      const int nb = kind == 2 ? blocks / 4 : blocks;
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int k = 0; k < K; ++k) {
        if (kind == 1)
          hipLaunchKernelGGL(copy_kernel, dim3(nb), dim3(wg), 0, st, a, b);
        else
          hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(wg), 0, st);
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
      std::printf("%s waves=%d (%d x %d): %.3f us per launch\n",
                  kind == 1 ? "copy " : "empty", blocks, nb, wg, 1000.0 * ms / (5 * K));
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
  }
  return 0;
}
