// Does a one-workgroup kernel on a second stream start beside a long kernel already running on
// another stream?  (The early leader's question, profiles/r06i_early_leader.txt: it ran behind
// phase A because their streams shared an in-order hardware queue.)  A long kernel A fills CUs
// 1..255 (a CU-masked stream) for ~2 ms; right after it, kernel L (one workgroup) goes to a
// second stream of the kind under test.  Both record their start on the 100 MHz clock.
// Streams created before the pair (`pre`) shift the runtime's round-robin queue assignment.
//   hipcc --offload-arch=gfx950 -O2 scripts/queue_probe.hip -o scripts/bin/queue_probe
//   scripts/bin/queue_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);             \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

__global__ void k_long(unsigned long long* t, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) t[0] = t0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void k_one(unsigned long long* t) {
  if (threadIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> rest(words, 0), one(words, 0);
  for (int i = 1; i < cus; ++i) rest[i / 32] |= 1u << (i % 32);
  one[0] = 1u;
  unsigned long long* t = nullptr;
  CK(hipMalloc(&t, 64));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  const char* kinds[] = {"plain", "cu-masked (1 CU)", "high priority"};
  for (int pre = 0; pre <= 6; pre += 2) {
    for (int kind = 0; kind < 3; ++kind) {
      std::vector<hipStream_t> extra(pre);
      for (auto& s : extra) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      hipStream_t sa, sl;
      CK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)words, rest.data()));
      if (kind == 0) CK(hipStreamCreateWithFlags(&sl, hipStreamNonBlocking));
      if (kind == 1) CK(hipExtStreamCreateWithCUMask(&sl, (uint32_t)words, one.data()));
      if (kind == 2) CK(hipStreamCreateWithPriority(&sl, hipStreamNonBlocking, hi));
      double worst = 0, best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemset(t, 0, 64));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_long, dim3(cus * 8), dim3(256), 0, sa, t, 200000ull);   // 2 ms
        hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, sl, t);
        CK(hipDeviceSynchronize());
        unsigned long long h[2];
        CK(hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost));
        const double us = ((double)h[1] - (double)h[0]) / 100.0;
        worst = us > worst ? us : worst;
        best = us < best ? us : best;
      }
      std::printf("streams before: %d  second stream: %-18s  L starts %8.1f .. %8.1f us after A\n",
                  pre, kinds[kind], best, worst);
      CK(hipStreamDestroy(sa));
      CK(hipStreamDestroy(sl));
      for (auto& s : extra) CK(hipStreamDestroy(s));
    }
  }
  return 0;
}
