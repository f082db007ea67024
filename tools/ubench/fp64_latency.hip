// Microbenchmark (diagnostic, not product): FP64 VALU issue cost and
// dependent latency on gfx950, one wave per SIMD, measured with s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ inline unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int KIND>
__global__ void bench(double* out, unsigned long long* cyc, double seed) {
  double a = seed + threadIdx.x, b = 1.0000001, c = 1e-9;
  double x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3, x4 = a + 4, x5 = a + 5, x6 = a + 6, x7 = a + 7;
  __shared__ double lds[1024];
  lds[threadIdx.x] = a;
  __syncthreads();
  int idx = threadIdx.x;
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t0 = now();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 256; ++i) {
    if (KIND == 0) {  // dependent fma chain
      x0 = fma(x0, b, c);
    } else if (KIND == 1) {  // 8 independent chains
      x0 = fma(x0, b, c); x1 = fma(x1, b, c); x2 = fma(x2, b, c); x3 = fma(x3, b, c);
      x4 = fma(x4, b, c); x5 = fma(x5, b, c); x6 = fma(x6, b, c); x7 = fma(x7, b, c);
    } else if (KIND == 2) {  // dependent rcp
      x0 = __builtin_amdgcn_rcp(x0);
    } else if (KIND == 3) {  // 8 independent rcp
      x0 = __builtin_amdgcn_rcp(x0); x1 = __builtin_amdgcn_rcp(x1); x2 = __builtin_amdgcn_rcp(x2); x3 = __builtin_amdgcn_rcp(x3);
      x4 = __builtin_amdgcn_rcp(x4); x5 = __builtin_amdgcn_rcp(x5); x6 = __builtin_amdgcn_rcp(x6); x7 = __builtin_amdgcn_rcp(x7);
    } else if (KIND == 4) {  // dependent LDS read chain (address depends on data)
      double v = lds[idx & 1023];
      idx = (int)v & 1023;
      x0 += v;
    } else if (KIND == 5) {  // dependent DPP row_shr through fma
      long long u = __builtin_bit_cast(long long, x0);
      int lo = __builtin_amdgcn_update_dpp(0, (int)u, 0x111, 0xf, 0xf, false);
      int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x111, 0xf, 0xf, false);
      x0 = fma(__builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo), b, c);
    } else if (KIND == 6) {  // dependent mul chain
      x0 = x0 * b;
    } else if (KIND == 8) {  // back-substitution step: 4 quad broadcasts (mov_dpp) + 4-FMA chain
      long long u = __builtin_bit_cast(long long, x0);
      double xb[4];
#define QB(J) xb[J] = __builtin_bit_cast(double, ((long long)__builtin_amdgcn_mov_dpp((int)(u >> 32), J * 0x55, 0xf, 0xf, false) << 32) | \
                      (unsigned)__builtin_amdgcn_mov_dpp((int)u, J * 0x55, 0xf, 0xf, false))
      QB(0); QB(1); QB(2); QB(3);
#undef QB
      double s2 = x1;
      s2 = fma(-x2, xb[0], s2); s2 = fma(-x3, xb[1], s2); s2 = fma(-x4, xb[2], s2); s2 = fma(-x5, xb[3], s2);
      x0 = s2 * 1e-3;
    } else if (KIND == 7) {  // dependent readlane broadcast through fma
      x0 = fma(__builtin_bit_cast(double, (long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(long long, x0)), 3) |
                  ((long long)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(long long, x0) >> 32), 3) << 32)), b, c);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t1 = now();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 4096);
  const char* names[] = {"fma_f64 dep", "fma_f64 8-indep", "rcp_f64 dep", "rcp_f64 8-indep", "ds_read_b64 dep", "dpp+fma dep", "mul_f64 dep", "readlane+fma dep", "backsub step"};
  const int ops[] = {256, 2048, 256, 2048, 256, 256, 256, 256, 256};
  for (int rep = 0; rep < 2; ++rep) {
    for (int k = 0; k < 9; ++k) {
      switch (k) {
        case 0: bench<0><<<1, 64>>>(out, cyc, 1.0); break;
        case 1: bench<1><<<1, 64>>>(out, cyc, 1.0); break;
        case 2: bench<2><<<1, 64>>>(out, cyc, 1.0); break;
        case 3: bench<3><<<1, 64>>>(out, cyc, 1.0); break;
        case 4: bench<4><<<1, 64>>>(out, cyc, 1.0); break;
        case 5: bench<5><<<1, 64>>>(out, cyc, 1.0); break;
        case 6: bench<6><<<1, 64>>>(out, cyc, 1.0); break;
        case 7: bench<7><<<1, 64>>>(out, cyc, 1.0); break;
        case 8: bench<8><<<1, 64>>>(out, cyc, 1.0); break;
      }
      unsigned long long h;
      hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-20s %8llu cyc / %d ops = %.2f cyc/op\n", names[k], h, ops[k], (double)h / ops[k]);
    }
  }
  return 0;
}
