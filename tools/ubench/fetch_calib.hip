// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths
// this library's kernels use (MI355X_MICROARCH.md: only 16-byte-per-lane
// streaming reads and stores are calibrated; other widths are not).  Each
// kernel moves exactly 64 MiB (past the 32 MiB of L2): reads of 4, 8 and 16
// bytes per lane (results summed into one store per workgroup), and stores
// of 8 and 16 bytes per lane.  Run under separate --pmc FETCH_SIZE and
// WRITE_SIZE passes (tools/gpu_r04_prof.sh); the per-kernel counter over
// 65536 KiB is the factor to apply.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/fetch_calib tools/ubench/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = 64ull << 20;

template <typename T>
__global__ __launch_bounds__(256) void read_kernel(const T* __restrict__ a, double* __restrict__ out,
                                                   size_t n) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const T v = a[i];
    if constexpr (sizeof(T) == 4) s += static_cast<double>(v);
    if constexpr (sizeof(T) == 8) s += v;
    if constexpr (sizeof(T) == 16) s += v.x + v.y;
  }
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < 256; ++k) t += red[k];
    out[blockIdx.x] = t;  // 8 B per workgroup (2 KiB in all)
  }
}

template <typename T>
__global__ __launch_bounds__(256) void write_kernel(T* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    T v;
    if constexpr (sizeof(T) == 8) v = static_cast<double>(i);
    if constexpr (sizeof(T) == 16) v = make_double2(static_cast<double>(i), 1.0);
    a[i] = v;
  }
}

int main() {
  void* buf;
  double* out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 256 * 8) != hipSuccess) return 1;
  hipMemset(buf, 0, kBytes);
  const dim3 grid(256 * 8), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read_kernel<float>, grid, block, 0, 0, static_cast<const float*>(buf),
                       out, kBytes / 4);
    hipLaunchKernelGGL(read_kernel<double>, grid, block, 0, 0, static_cast<const double*>(buf),
                       out, kBytes / 8);
    hipLaunchKernelGGL(read_kernel<double2>, grid, block, 0, 0,
                       static_cast<const double2*>(buf), out, kBytes / 16);
    hipLaunchKernelGGL(write_kernel<double>, grid, block, 0, 0, static_cast<double*>(buf),
                       kBytes / 8);
    hipLaunchKernelGGL(write_kernel<double2>, grid, block, 0, 0, static_cast<double2*>(buf),
                       kBytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("moved %zu KiB per kernel\n", kBytes >> 10);
  return 0;
}
