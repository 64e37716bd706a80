// Probe: do CU-masked streams partition the CUs, and how do mask bits map to XCC/SE/CU?
// Each workgroup records (xcc, se, cu) from the hardware id registers and spins ~50 us so
// the grid spreads over every CU the mask allows.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_ID (gfx9)
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
    out[blockIdx.x] = (xcc & 0xf) << 24 | (hw & 0xffffff);
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 5000) {}
  }
}

static void run(const char* name, hipStream_t s, unsigned* d, int nblk) {
  hipLaunchKernelGGL(probe, dim3(nblk), dim3(64), 0, s, d);
  if (hipStreamSynchronize(s) != hipSuccess) { printf("%s: sync failed\n", name); exit(1); }
  std::vector<unsigned> h(nblk);
  hipMemcpy(h.data(), d, nblk * 4, hipMemcpyDeviceToHost);
  std::set<unsigned> cus, xccs;
  for (unsigned v : h) {
    unsigned xcc = v >> 24, se = (v >> 13) & 7, cu = (v >> 8) & 15, sa = (v >> 12) & 1;  // gfx9 HW_ID fields
    cus.insert(xcc << 16 | se << 8 | sa << 4 | cu);
    xccs.insert(xcc);
  }
  printf("%s: %zu distinct CUs over %zu XCCs:", name, cus.size(), xccs.size());
  unsigned last = ~0u; int cnt = 0;
  for (unsigned c : cus) { if ((c >> 16) != last) { if (cnt) printf(" %d", cnt); printf(" [x%u]", c >> 16); last = c >> 16; cnt = 0; } cnt++; }
  printf(" %d\n", cnt);
}

int main() {
  unsigned* d;
  const int nblk = 8192;
  hipMalloc(&d, nblk * 4);
  hipStream_t s0;
  hipStreamCreate(&s0);
  run("nomask", s0, d, nblk);
  int tests[] = {32, 64, 96, 160, 192};
  for (int n : tests) {
    uint32_t m[8] = {0};
    for (int i = 0; i < n; ++i) m[i / 32] |= 1u << (i % 32);
    hipStream_t s;
    hipError_t e = hipExtStreamCreateWithCUMask(&s, 8, m);
    if (e != hipSuccess) { printf("mask %d: create failed %s\n", n, hipGetErrorString(e)); continue; }
    char nm[64]; snprintf(nm, sizeof nm, "low %d bits", n);
    run(nm, s, d, nblk);
    uint32_t mi[8];
    for (int i = 0; i < 8; ++i) mi[i] = ~m[i];
    hipStream_t s2;
    if (hipExtStreamCreateWithCUMask(&s2, 8, mi) == hipSuccess) {
      snprintf(nm, sizeof nm, "complement of %d", n);
      run(nm, s2, d, nblk);
      hipStreamDestroy(s2);
    }
    hipStreamDestroy(s);
  }
  // every 8th bit pattern
  {
    uint32_t m[8] = {0};
    for (int i = 0; i < 256; i += 8) m[i / 32] |= 1u << (i % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, 8, m) == hipSuccess) { run("every 8th bit", s, d, nblk); hipStreamDestroy(s); }
  }
  return 0;
}
