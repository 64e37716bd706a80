// block_bench.hip — measurement tooling (not a test, not the product): the team leader's block
// step (rc_kernels.hip block_window, cooperative steps of 16 entries at one carry) alone on one
// workgroup, over windows of the long carry segment that scripts/dump_entries.c wrote from the
// CPU oracle.  Each window starts at one of the segment's changers with its exact carry-in and
// runs in cooperative steps to its end (K = 64: no LANE passes); every carry-in it publishes is
// checked bit for bit against the oracle's.  Cycles per cooperative step = what one changer
// costs the team leader, evaluator and step overhead together.
//
//   hipcc <the product flags> -Iinclude -Iraytracing-programs_amd/csrc scripts/block_bench.hip
//   /tmp/block_bench entries.bin [windows] [variant: 0 product step, 2 split by shape class]
#include "../raytracing-programs_amd/csrc/rc_kernels.hip"
#include "split_step.hpp"

#include <cstdio>
#include <cstring>
#include <vector>

namespace rc {

struct BEntry {
  DepRec r;
  float cin[3], cout[3];
  int steps, hit;
};
static_assert(sizeof(BEntry) == 80, "dump_entries.c layout");

__global__ void __launch_bounds__(kResolveBlock) k_bb(Scene sc, const BEntry* __restrict__ ent,
                                                      const int* __restrict__ wstart, int nwin,
                                                      int n, CinG* __restrict__ cin, unsigned tag,
                                                      unsigned long long* __restrict__ acc,
                                                      int variant) {
  __shared__ rc_shape s_shapes[16];
  const int words = (int)(sizeof(rc_shape) / 4) * (sc.n + 1);
  for (int i = threadIdx.x; i < words; i += blockDim.x)
    ((unsigned*)s_shapes)[i] = ((const unsigned*)sc.shapes)[i];
  __syncthreads();
  sc.shapes = s_shapes;
  sc.lshapes = s_shapes;
  constexpr int G = 8;
  const int lane = threadIdx.x & 63;
  LaneShape ls;
  const int kself = lane % G;
  ls.has = kself < sc.n;
  ls.s = sc.shapes[ls.has ? kself : sc.n];
  __shared__ BlockWinShared bw;
  __shared__ SplitX sxs[2];                                       // variant 2: the split step
  const SplitLane sl = split_lane(sc, threadIdx.x >> 6, lane);
  unsigned long long cyc = 0, steps = 0, chg = 0;
  for (int wi = 0; wi < nwin; ++wi) {
    const int j = wstart[wi];
    const int nv = n - j < kResolveBlock ? n - j : kResolveBlock;
    const int t = threadIdx.x;
    if (t < nv) bw.rec[t] = ent[j + t].r;
    V3 c = v3(ent[j].cin[0], ent[j].cin[1], ent[j].cin[2]);
    __syncthreads();
    WinStats ws = {0, 0, 0};
    bool dense = true, changed = false;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    (void)variant;
#ifdef BB_LEAN
    if (variant == 1)
      block_window_lean(sc, 7, bw, j, nv, c, ls, G, dense, changed, 64, cin, tag, ws);
    else
#endif
      if (variant == 2)
        split_block_window(sc, 7, bw, sxs, sl, j, nv, c, cin, tag, ws);
      else
        block_window(sc, 7, bw, j, nv, c, ls, G, dense, changed, 64, cin, tag, ws, nullptr, false);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    cyc += t1 - t0;
    steps += ws.coop + ws.lane;
    chg += ws.changers;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    acc[0] = cyc;
    acc[1] = steps;
    acc[2] = chg;
  }
}

}  // namespace rc

using namespace rc;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                   __LINE__);                                                          \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  int hdr[4];
  if (std::fread(hdr, sizeof hdr, 1, f) != 1 || hdr[0] != 0x45444352) return 1;
  const int n = hdr[1], sbytes = hdr[3];
  std::vector<char> img(sbytes);
  std::vector<BEntry> ent(n);
  if (std::fread(img.data(), sbytes, 1, f) != 1 ||
      std::fread(ent.data(), sizeof(BEntry), n, f) != (size_t)n)
    return 1;
  std::fclose(f);
  const rc_packed_header* h = (const rc_packed_header*)img.data();
  if (hdr[2] != 7 || h->n > 15) return 1;
  const int want = argc > 2 ? std::atoi(argv[2]) : 64;
  const int variant = argc > 3 ? std::atoi(argv[3]) : 0;
  // windows: start at changers, at least one window apart
  std::vector<int> ws;
  for (int i = 0; i < n && (int)ws.size() < want; ++i) {
    const bool ch = std::memcmp(ent[i].cin, ent[i].cout, 12) != 0;
    if (ch && (ws.empty() || i >= ws.back() + kResolveBlock) && i + kResolveBlock <= n)
      ws.push_back(i);
  }
  char* d_img;
  BEntry* d_ent;
  int* d_ws;
  CinG* d_cin;
  unsigned long long* d_acc;
  CK(hipMalloc(&d_img, sbytes));
  CK(hipMalloc(&d_ent, sizeof(BEntry) * (size_t)n));
  CK(hipMalloc(&d_ws, sizeof(int) * ws.size()));
  CK(hipMalloc(&d_cin, sizeof(CinG) * (size_t)n));
  CK(hipMalloc(&d_acc, 64));
  CK(hipMemcpy(d_img, img.data(), sbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ent, ent.data(), sizeof(BEntry) * (size_t)n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ws, ws.data(), sizeof(int) * ws.size(), hipMemcpyHostToDevice));
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
  for (int k = 0; k < h->n; ++k) sc.has_quadric |= hs[k].type == RC_SHAPE_QUADRIC;
  sc.dep_fast = 1;
  for (int rep = 0; rep < 3; ++rep) {
    const unsigned tag = 100 + rep;
    CK(hipMemset(d_cin, 0, sizeof(CinG) * (size_t)n));
    hipLaunchKernelGGL(k_bb, dim3(1), dim3(kResolveBlock), 0, 0, sc, d_ent, d_ws, (int)ws.size(),
                       n, d_cin, tag, d_acc, variant);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long acc[3];
    CK(hipMemcpy(acc, d_acc, sizeof acc, hipMemcpyDeviceToHost));
    std::vector<CinG> cin(n);
    CK(hipMemcpy(cin.data(), d_cin, sizeof(CinG) * (size_t)n, hipMemcpyDeviceToHost));
    long long bad = 0, checked = 0;
    for (int w : ws)
      for (int i = w; i < w + kResolveBlock && i < n; ++i) {
        ++checked;
        for (int q = 0; q < 3; ++q) {
          unsigned v, tg;
          std::memcpy(&v, &ent[i].cin[q], 4);
          const unsigned long long g = cin[i].g[q];
          tg = (unsigned)(g >> 32);
          if ((unsigned)g != v || (tg & 0x7fffffffu) != tag ||
              ((tg >> 31) != 0) != (ent[i].hit != 0))
            ++bad;
        }
      }
    std::printf("%s variant %d: %zu windows, %llu steps, %llu changers: %.0f cycles per step "
                "(%.0f per changer); carry-ins checked %lld, wrong granules %lld\n",
                argv[1], variant, ws.size(), acc[1], acc[2], (double)acc[0] / acc[1],
                (double)acc[0] / acc[2], checked, bad);
  }
  return 0;
}
