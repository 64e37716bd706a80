// prim_probe.hip — gfx950 probe for the resolver's f64 primitives.
//   1. accuracy of v_rcp_f64 / v_rsq_f64 (max relative error over random normal inputs)
//   2. dependent-chain latency (cycles per op, one wave) of the f64 ops on the carry chain
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/prim_probe.hip -o build/prim_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// relative errors in units of 2^-60 (as integers for atomicMax)
__global__ void k_acc(int iters, unsigned long long* out) {
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  double erc = 0.0, ers = 0.0;
  for (int i = 0; i < iters; ++i) {
    const uint64_t h = mix(tid * 7919ull + (uint64_t)i * 0x9e3779b97f4a7c15ull);
    // mantissa random, exponent in [-60, 60]
    const int e = (int)(h >> 52) % 121 - 60;
    const double m = 1.0 + (double)(h & ((1ull << 52) - 1)) * 0x1p-52;
    const double x = ldexp(m, e);
    const double r = __builtin_amdgcn_rcp(x);
    // exact residual 1 - x*r (fma is exact enough: |x*r - 1| small)
    const double res = __builtin_fma(-x, r, 1.0);
    erc = fmax(erc, fabs(res));
    const double y = __builtin_amdgcn_rsq(x);
    const double ref = 1.0 / sqrt(x);   // within ~2^-52 of 1/sqrt(x)
    ers = fmax(ers, fabs(y - ref) / ref);
  }
  atomicMax(&out[0], (unsigned long long)(erc * 0x1p60));
  atomicMax(&out[1], (unsigned long long)(ers * 0x1p60));
}

template <int OP>
__device__ __forceinline__ double op(double a, double b) {
  if constexpr (OP == 0) return __builtin_fma(a, b, 1e-300);
  if constexpr (OP == 1) return a * b;
  if constexpr (OP == 2) return a + b;
  if constexpr (OP == 3) return __builtin_amdgcn_rcp(a) * 0.0 + a;   // rcp + dependent fma
  if constexpr (OP == 4) return __builtin_amdgcn_rsq(a) * 0.0 + a;
  if constexpr (OP == 5) return a / b;
  if constexpr (OP == 6) return (double)(float)(a * b);   // mul + 2 cvt                  // cvt f32 <- f64 -> f64
  if constexpr (OP == 7) return sqrt(a) * 0.0 + a;
  if constexpr (OP == 8) {   // f32 fma chain (for reference), via cvt at the ends only
    float f = (float)a;
    return (double)__builtin_fmaf(f, (float)b, 1e-30f);
  }
  return a;
}

template <int OP>
__global__ void k_lat(double seed, double b, int n, unsigned long long* cyc, double* sink) {
  double a = seed + threadIdx.x * 1e-9;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 32; ++k) a = op<OP>(a, b);
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[OP] = t1 - t0;
  sink[threadIdx.x] = a;
}

// issue cost: 8 independent chains interleaved (one wave)
template <int OP>
__global__ void k_thr(double seed, double b, int n, unsigned long long* cyc, double* sink) {
  double a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = seed + threadIdx.x * 1e-9 + j * 1e-7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = op<OP>(a[j], b);
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[16 + OP] = t1 - t0;
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j];
  sink[threadIdx.x] = s;
}

int main() {
  unsigned long long* d;
  double* sink;
  hipMalloc(&d, 64 * sizeof(unsigned long long));
  hipMalloc(&sink, 64 * sizeof(double));
  hipMemset(d, 0, 64 * sizeof(unsigned long long));
  k_acc<<<4096, 256>>>(256, d);
  unsigned long long h[64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("rcp_f64 max rel err 2^%.2f   rsq_f64 max rel err 2^%.2f  (%.3g random inputs)\n",
         log2((double)h[0]) - 60, log2((double)h[1]) - 60, 4096.0 * 256 * 256);
  hipMemset(d, 0, 64 * sizeof(unsigned long long));
  const int n = 256;
  const char* names[] = {"fma_f64", "mul_f64", "add_f64", "rcp_f64+fma", "rsq_f64+fma",
                         "div_f64", "mul+cvt f64->f32->f64", "sqrt_f64 (compiler)+fma", "fma_f32"};
  k_lat<0><<<1, 64>>>(1.0, 0.999999, n, d, sink);
  k_lat<1><<<1, 64>>>(1.0, 0.999999, n, d, sink);
  k_lat<2><<<1, 64>>>(1.0, 1e-20, n, d, sink);
  k_lat<3><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_lat<4><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_lat<5><<<1, 64>>>(1.5, 1.0000001, n, d, sink);
  k_lat<6><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_lat<7><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_lat<8><<<1, 64>>>(1.5, 0.9999, n, d, sink);
  k_thr<0><<<1, 64>>>(1.0, 0.999999, n, d, sink);
  k_thr<1><<<1, 64>>>(1.0, 0.999999, n, d, sink);
  k_thr<2><<<1, 64>>>(1.0, 1e-20, n, d, sink);
  k_thr<3><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_thr<4><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_thr<5><<<1, 64>>>(1.5, 1.0000001, n, d, sink);
  k_thr<6><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_thr<7><<<1, 64>>>(1.5, 1.0, n, d, sink);
  k_thr<8><<<1, 64>>>(1.5, 0.9999, n, d, sink);
  hipDeviceSynchronize();
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int i = 0; i < 9; ++i)
    printf("%-26s %6.1f cycles per dependent op, %6.1f per independent op (one wave)\n", names[i],
           (double)h[i] / (n * 32.0), (double)h[16 + i] / (n * 64.0));
  return 0;
}
