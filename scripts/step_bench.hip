// step_bench.hip — measurement tooling (not a test, not the product): the resolver's
// cooperative evaluator (rc_device.hpp carry_path_spec) alone on the GPU, over the DEP entries
// scripts/dump_entries.c wrote from the CPU oracle (records, exact carry-ins and carry-outs).
// Every evaluation is checked bit for bit against the oracle's carry-out and hit flag; the
// timing is s_memtime cycles per evaluation on lone waves (one wave per SIMD), as the team
// leader's and the helpers' block steps run it.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero
//     -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Iraytracing-programs_amd/csrc
//     scripts/step_bench.hip -o /tmp/step_bench
//   /tmp/step_bench entries.bin [batches per wave] [waves per block] [blocks]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rc_device.hpp"
#include "spec_exp.hpp"

using namespace rc;

struct Entry {
  DepRec r;
  float cin[3], cout[3];
  int steps, hit;
};
static_assert(sizeof(Entry) == 80, "dump_entries.c layout");

#ifndef SB_GT
#define SB_GT 8
#endif
#ifndef SB_Q
#define SB_Q 1   // the resolver's specialisation (RC_X0_RESOLVE 0: quadrics with cross terms)
#endif

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
k_bench(Scene sc, const Entry* __restrict__ ent, int nent, int batches,
        unsigned long long* __restrict__ acc, int* __restrict__ bad) {
  __shared__ rc_shape s_shapes[16];
  const int words = (int)(sizeof(rc_shape) / 4) * (sc.n + 1);
  for (int i = threadIdx.x; i < words; i += blockDim.x)
    ((unsigned*)s_shapes)[i] = ((const unsigned*)sc.shapes)[i];
  __syncthreads();
  sc.shapes = s_shapes;
  sc.lshapes = s_shapes;
  constexpr int G = SB_GT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  const int kself = lane % G, half = (lane / G) & 1, e = lane / (2 * G);
  constexpr int E = 64 / (2 * G);
  LaneShape ls;
  ls.has = kself < sc.n;
  ls.s = sc.shapes[ls.has ? kself : sc.n];   // (the extra lanes: a defined record, never used)
  unsigned long long cyc = 0, steps = 0;
  int nb = 0, mism = 0;
  const int wid = blockIdx.x * waves + wave, nw = gridDim.x * waves;
  for (int b = wid; b < batches && (b + 1) * E <= nent; b += nw) {
    const Entry& q = ent[b * E + e];
    const DepRec ri = q.r;
    const V3 c = v3(q.cin[0], q.cin[1], q.cin[2]);
    int zero = 0;
    bool hg = false;
    int mx = q.steps;
    for (int off = 2 * G; off < 64; off <<= 1) mx = max(mx, __shfl_xor(mx, off, 64));
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#ifdef SB_VAR
    const V3 o = carry_path_x<G, SB_Q, SB_VAR>(sc, ls, kself, G, half, ri, 7, c, zero, hg);
#else
    const V3 o = carry_path_spec<G, SB_Q>(sc, ls, kself, G, half, ri, 7, c, zero, hg);
#endif
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    cyc += t1 - t0;
    steps += mx;
    ++nb;
    const bool ok = __float_as_uint(o.x) == __float_as_uint(q.cout[0]) &&
                    __float_as_uint(o.y) == __float_as_uint(q.cout[1]) &&
                    __float_as_uint(o.z) == __float_as_uint(q.cout[2]) && (hg == (q.hit != 0));
    mism += ((lane % (2 * G)) == 0 && !ok) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) mism += __shfl_xor(mism, off, 64);
  if (lane == 0) {
    atomicAdd(&acc[0], cyc);
    atomicAdd(&acc[1], steps);
    atomicAdd(&acc[2], (unsigned long long)nb);
    atomicAdd(bad, mism);
  }
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  int hdr[4];
  if (std::fread(hdr, sizeof hdr, 1, f) != 1 || hdr[0] != 0x45444352) return 1;
  const int n = hdr[1], maxrec = hdr[2], sbytes = hdr[3];
  std::vector<char> img(sbytes);
  std::vector<Entry> ent(n);
  if (std::fread(img.data(), sbytes, 1, f) != 1 ||
      std::fread(ent.data(), sizeof(Entry), n, f) != (size_t)n)
    return 1;
  std::fclose(f);
  if (maxrec != 7) return 1;
  if (((const rc_packed_header*)img.data())->n > 15) return 1;   // s_shapes[16]
  const rc_packed_header* h = (const rc_packed_header*)img.data();
  const int per_wave = argc > 2 ? std::atoi(argv[2]) : 256;
  const int waves = argc > 3 ? std::atoi(argv[3]) : 4;
  const int blocks = argc > 4 ? std::atoi(argv[4]) : 1;
  char* d_img;
  Entry* d_ent;
  unsigned long long* d_acc;
  int* d_bad;
  CK(hipMalloc(&d_img, sbytes));
  CK(hipMalloc(&d_ent, sizeof(Entry) * (size_t)n));
  CK(hipMalloc(&d_acc, 64));
  CK(hipMalloc(&d_bad, 4));
  CK(hipMemcpy(d_img, img.data(), sbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ent, ent.data(), sizeof(Entry) * (size_t)n, hipMemcpyHostToDevice));
  Scene sc{};
  sc.shapes = (const rc_shape*)(d_img + h->off_shapes);
  sc.lights = (const rc_light*)(d_img + h->off_lights);
  sc.pairs = (const rc_shade_pair*)(d_img + h->off_pairs);
  sc.lshapes = sc.shapes;
  sc.lpairs = sc.pairs;
  sc.n = h->n;
  sc.m = h->m;
  const rc_shape* hs = (const rc_shape*)(img.data() + h->off_shapes);
  for (int k = 0; k < h->n && k < 64; ++k)
    if (hs[k].refl > 0.0f) sc.refl_mask |= 1ull << k;
  sc.has_quadric = 0;
  for (int k = 0; k < h->n; ++k) sc.has_quadric |= hs[k].type == RC_SHAPE_QUADRIC;
  sc.o0_ok = 0;
  sc.dep_fast = 1;
  const int E = 64 / (2 * SB_GT);
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(d_acc, 0, 64));
    CK(hipMemset(d_bad, 0, 4));
    const long long want = (long long)blocks * waves * per_wave;
    const int batches = (int)(want < n / E ? want : n / E);
    hipLaunchKernelGGL(k_bench, dim3(blocks), dim3(64 * waves), 0, 0, sc, d_ent, n, batches,
                       d_acc, d_bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long acc[3];
    int bad;
    CK(hipMemcpy(acc, d_acc, sizeof acc, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
    std::printf("%s: %llu evaluations of %d entries per wave (%d waves x %d blocks): %.0f cycles "
                "each, %.3f steps each, %.0f cycles per step; mismatches %d of %llu entries\n",
                argv[1], acc[2], E, waves, blocks, (double)acc[0] / acc[2],
                (double)acc[1] / acc[2], (double)acc[0] / acc[1], bad, acc[2] * E);
  }
  return 0;
}
