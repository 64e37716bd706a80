// mask_rate_probe.hip — measurement tooling: does a CU-masked stream run a many-workgroup,
// VALU-bound kernel (phase A's shape: 65 536 workgroups of 256 threads, a few us each) at its
// CU share of the device's rate?  Times the same kernel on an unmasked stream and on masked
// streams of 64 / 128 / 192 CUs, as a one-tile-per-workgroup grid and as a persistent grid
// (8 workgroups per CU of the mask, striding over the same tiles).
//   hipcc --offload-arch=gfx950 -O3 scripts/mask_rate_probe.hip -o /tmp/mask_rate_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ __forceinline__ float work(float x, int iters) {
  float a = x, b = x * 0.5f, c = x * 0.25f, d = x * 0.125f;
  for (int i = 0; i < iters; ++i) {
    a = a * 1.0000001f + 0.5f;
    b = b * 0.9999999f + 0.25f;
    c = c * 1.0000002f + 0.125f;
    d = d * 0.9999998f + 0.0625f;
  }
  return a + b + c + d;
}

__global__ void __launch_bounds__(256) tiles(float* out, int iters) {
  const int t = blockIdx.x;
  out[(size_t)t * 256 + threadIdx.x] = work((float)threadIdx.x, iters);
}

__global__ void __launch_bounds__(256) persistent(float* out, int ntiles, int iters) {
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x)
    out[(size_t)t * 256 + threadIdx.x] = work((float)threadIdx.x, iters);
}

int main(int argc, char** argv) {
  const int ntiles = 65536, iters = argc > 1 ? atoi(argv[1]) : 400;
  float* d;
  if (hipMalloc(&d, (size_t)ntiles * 256 * 4) != hipSuccess) return 1;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](hipStream_t s, bool pers, int ncu) {
    float best = 1e30f;
    for (int r = 0; r < 4; ++r) {
      hipEventRecord(e0, s);
      if (pers)
        hipLaunchKernelGGL(persistent, dim3(ncu * 8), dim3(256), 0, s, d, ntiles, iters);
      else
        hipLaunchKernelGGL(tiles, dim3(ntiles), dim3(256), 0, s, d, iters);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms = 0.0f;
      hipEventElapsedTime(&ms, e0, e1);
      if (r > 0 && ms < best) best = ms;
    }
    return best;
  };
  hipStream_t s0;
  hipStreamCreate(&s0);
  const float full = time(s0, false, cus), fullp = time(s0, true, cus);
  std::printf("unmasked %d CUs: tiles %.3f ms, persistent %.3f ms\n", cus, full, fullp);
  const int words = (cus + 31) / 32;
  for (int n : {64, 128, 192}) {
    for (int hi = 0; hi < 2; ++hi) {
      std::vector<uint32_t> m(words, 0);
      for (int i = 0; i < cus; ++i) {
        const bool in = hi ? i >= cus - n : i < n;
        if (in) m[i / 32] |= 1u << (i % 32);
      }
      hipStream_t s;
      if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, m.data()) != hipSuccess) return 1;
      const float a = time(s, false, n), b = time(s, true, n);
      std::printf("mask %s %3d CUs: tiles %.3f ms (%.2fx the CU share), persistent %.3f ms (%.2fx)\n",
                  hi ? "high" : "low ", n, a, a / (full * cus / n), b, b / (fullp * cus / n));
      hipStreamDestroy(s);
    }
  }
  return 0;
}
