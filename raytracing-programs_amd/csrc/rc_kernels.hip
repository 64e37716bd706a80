// rc_kernels.hip — HIP kernels of the MI355X raycaster (gfx950).
//
//   k_render      one lane per pixel, 16x16-pixel workgroups (four 8x8 wave tiles for ray
//                 coherence), full iterative_shoot + quantisation, RGB store.  Fast mode, and
//                 parity mode at depth 0 (no bounce loop => no carry).
//   k_phase_a     parity phase A: same as k_render but a pixel whose first reflection misses
//                 (a DEP pixel, it reads the scan-order carry) stops and records its state;
//                 every other pixel is final.  Writers record their carry-out.
//   k_row_stats / k_row_scan / k_row_compact
//                 scan-order compaction of the DEP pixels, each tagged with the last writer
//                 before it (its segment key); segment starts appended to a work list.
//   k_resolve     parity phase B: exact carry chain.  One workgroup per segment (dequeued
//                 from a counter): evaluate a window of DEP pixels at the current carry in
//                 parallel, the first pixel that changes the carry ends the step.
//   k_phase_c     parity phase C: shade every DEP pixel with its resolved carry-in.
#include <hip/hip_runtime.h>

#include "rc_device.hpp"
#include "rc_kernels.h"

namespace rc {

constexpr int kTile = 16;        // 16x16 pixels per workgroup, 256 lanes
constexpr int kBlock = kTile * kTile;

__device__ __forceinline__ void tile_pixel(int& lx, int& ly) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  lx = (wave & 1) * 8 + (lane & 7);
  ly = (wave >> 1) * 8 + (lane >> 3);
}

__device__ __forceinline__ void store_rgb(uint8_t* __restrict__ p, V3 c) {
  p[0] = quant(c.x);
  p[1] = quant(c.y);
  p[2] = quant(c.z);
}

__device__ __forceinline__ void flush_events(int zero_events, unsigned long long* counter) {
  if (zero_events) atomicAdd(counter, (unsigned long long)zero_events);
}

// ------------------------------------------------------------------ fast / depth 0 --
__global__ void __launch_bounds__(kBlock) k_render(Scene sc, Cam cam, int W, int H, int row0,
                                                   int row_step, int nrows, int maxrec,
                                                   uint8_t* __restrict__ out,
                                                   unsigned long long* __restrict__ zcount) {
  int lx, ly;
  tile_pixel(lx, ly);
  const int x = blockIdx.x * kTile + lx;
  const int r = blockIdx.y * kTile + ly;           // local (shard) row
  if (x >= W || r >= nrows) return;
  const int y = row0 + r * row_step;
  int zero = 0;
  const V3 d = primary_dir(cam, x, y, zero);
  PixelOut po;
  shoot<kModeFast>(sc, d, maxrec, v3(0.0f, 0.0f, 0.0f), po, zero);
  store_rgb(out + ((size_t)r * W + x) * 3, po.rgb);
  flush_events(zero, zcount);
}

// ------------------------------------------------------------------ parity phase A --
__global__ void __launch_bounds__(kBlock) k_phase_a(Scene sc, Cam cam, int W, int H, int maxrec,
                                                    uint8_t* __restrict__ out,
                                                    uint8_t* __restrict__ cls,
                                                    float4* __restrict__ wcarry,
                                                    DepRec* __restrict__ deprec,
                                                    unsigned long long* __restrict__ zcount) {
  int lx, ly;
  tile_pixel(lx, ly);
  const int x = blockIdx.x * kTile + lx;
  const int y = blockIdx.y * kTile + ly;
  if (x >= W || y >= H) return;
  const size_t p = (size_t)y * W + x;
  int zero = 0;
  const V3 d = primary_dir(cam, x, y, zero);
  PixelOut po;
  shoot<kModeParityA>(sc, d, maxrec, v3(0.0f, 0.0f, 0.0f), po, zero);
  cls[p] = po.cls;
  if (po.cls == kClsDep) {
    deprec[p] = po.dep;     // phase C recomputes the whole pixel (and counts its events)
    return;
  }
  if (po.cls == kClsWriter) wcarry[p] = make_float4(po.carry.x, po.carry.y, po.carry.z, 0.0f);
  store_rgb(out + p * 3, po.rgb);
  flush_events(zero, zcount);
}

// ------------------------------------------------------- scan-order DEP compaction --
// Per row: number of DEP pixels, last writer index, last DEP index (global pixel ids).
constexpr int kScanBlock = 256;

__device__ __forceinline__ int block_sum(int v, int* sh) {
  // 256 threads = 4 waves
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  int tot = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tot += sh[i];
  return tot;
}
__device__ __forceinline__ long long block_max64(long long v, long long* sh) {
  for (int o = 32; o > 0; o >>= 1) {
    long long u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  long long m = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = sh[i] > m ? sh[i] : m;
  return m;
}

__global__ void __launch_bounds__(kScanBlock) k_row_stats(const uint8_t* __restrict__ cls, int W,
                                                          int* __restrict__ row_ndep,
                                                          long long* __restrict__ row_lastw,
                                                          long long* __restrict__ row_lastdep) {
  __shared__ int shi[16];
  __shared__ long long shl[16];
  const int y = blockIdx.x;
  const long long base = (long long)y * W;
  int nd = 0;
  long long lw = -1, ld = -1;
  for (int x = threadIdx.x; x < W; x += blockDim.x) {
    const uint8_t c = cls[base + x];
    if (c == kClsDep) {
      nd++;
      ld = base + x;
    } else if (c == kClsWriter) {
      lw = base + x;
    }
  }
  nd = block_sum(nd, shi);
  lw = block_max64(lw, shl);
  ld = block_max64(ld, shl);
  if (threadIdx.x == 0) {
    row_ndep[y] = nd;
    row_lastw[y] = lw;
    row_lastdep[y] = ld;
  }
}

// Single workgroup: exclusive scans over rows (sum of DEP counts, max of writer/DEP ids).
__global__ void __launch_bounds__(1024) k_row_scan(int H, const int* __restrict__ row_ndep,
                                                   const long long* __restrict__ row_lastw,
                                                   const long long* __restrict__ row_lastdep,
                                                   int* __restrict__ row_off,
                                                   long long* __restrict__ row_prevw,
                                                   long long* __restrict__ row_prevdep,
                                                   int* __restrict__ ndep_total) {
  __shared__ int s_cnt[1024];
  __shared__ long long s_w[1024], s_d[1024];
  // carried across chunks of 1024 rows
  __shared__ int carry_cnt;
  __shared__ long long carry_w, carry_d;
  if (threadIdx.x == 0) {
    carry_cnt = 0;
    carry_w = -1;
    carry_d = -1;
  }
  __syncthreads();
  for (int base = 0; base < H; base += 1024) {
    const int y = base + threadIdx.x;
    s_cnt[threadIdx.x] = y < H ? row_ndep[y] : 0;
    s_w[threadIdx.x] = y < H ? row_lastw[y] : -1;
    s_d[threadIdx.x] = y < H ? row_lastdep[y] : -1;
    __syncthreads();
    // Hillis-Steele inclusive scan (1024 elements, 10 steps)
    for (int o = 1; o < 1024; o <<= 1) {
      int c = 0;
      long long w = -1, d = -1;
      if ((int)threadIdx.x >= o) {
        c = s_cnt[threadIdx.x - o];
        w = s_w[threadIdx.x - o];
        d = s_d[threadIdx.x - o];
      }
      __syncthreads();
      s_cnt[threadIdx.x] += c;
      if (w > s_w[threadIdx.x]) s_w[threadIdx.x] = w;
      if (d > s_d[threadIdx.x]) s_d[threadIdx.x] = d;
      __syncthreads();
    }
    if (y < H) {
      const int exc = (threadIdx.x ? s_cnt[threadIdx.x - 1] : 0);
      const long long pw = threadIdx.x ? s_w[threadIdx.x - 1] : -1;
      const long long pd = threadIdx.x ? s_d[threadIdx.x - 1] : -1;
      row_off[y] = carry_cnt + exc;
      row_prevw[y] = pw > carry_w ? pw : carry_w;
      row_prevdep[y] = pd > carry_d ? pd : carry_d;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      carry_cnt += s_cnt[1023];
      if (s_w[1023] > carry_w) carry_w = s_w[1023];
      if (s_d[1023] > carry_d) carry_d = s_d[1023];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *ndep_total = carry_cnt;
}

// Per row: write the DEP pixels in scan order with their segment key (last writer before
// the pixel, -1 = none: carry (0,0,0)) and append segment starts to the work list.
__global__ void __launch_bounds__(kScanBlock) k_row_compact(
    const uint8_t* __restrict__ cls, int W, const int* __restrict__ row_off,
    const long long* __restrict__ row_prevw, const long long* __restrict__ row_prevdep,
    long long* __restrict__ dep_pix, long long* __restrict__ dep_key,
    int* __restrict__ seg_start, int* __restrict__ nseg) {
  __shared__ int s_cnt[kScanBlock];
  __shared__ long long s_w[kScanBlock], s_d[kScanBlock];
  __shared__ int c_cnt;
  __shared__ long long c_w, c_d;
  const int y = blockIdx.x;
  const long long base = (long long)y * W;
  if (threadIdx.x == 0) {
    c_cnt = row_off[y];
    c_w = row_prevw[y];
    c_d = row_prevdep[y];
  }
  __syncthreads();
  for (int x0 = 0; x0 < W; x0 += kScanBlock) {
    const int x = x0 + threadIdx.x;
    const uint8_t c = x < W ? cls[base + x] : kClsIdent;
    const long long pix = base + x;
    s_cnt[threadIdx.x] = (c == kClsDep);
    s_w[threadIdx.x] = (c == kClsWriter) ? pix : -1;
    s_d[threadIdx.x] = (c == kClsDep) ? pix : -1;
    __syncthreads();
    for (int o = 1; o < kScanBlock; o <<= 1) {
      int cc = 0;
      long long w = -1, d = -1;
      if ((int)threadIdx.x >= o) {
        cc = s_cnt[threadIdx.x - o];
        w = s_w[threadIdx.x - o];
        d = s_d[threadIdx.x - o];
      }
      __syncthreads();
      s_cnt[threadIdx.x] += cc;
      if (w > s_w[threadIdx.x]) s_w[threadIdx.x] = w;
      if (d > s_d[threadIdx.x]) s_d[threadIdx.x] = d;
      __syncthreads();
    }
    if (c == kClsDep) {
      const int idx = c_cnt + s_cnt[threadIdx.x] - 1;
      // writers strictly before this pixel: inclusive scan includes none at this position
      // (a DEP pixel is not a writer), so the inclusive max is the exclusive one.
      long long key = s_w[threadIdx.x];
      if (c_w > key) key = c_w;
      long long prevd = threadIdx.x ? s_d[threadIdx.x - 1] : -1;
      if (c_d > prevd) prevd = c_d;
      dep_pix[idx] = pix;
      dep_key[idx] = key;
      if (prevd < 0 || key > prevd) seg_start[atomicAdd(nseg, 1)] = idx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      c_cnt += s_cnt[kScanBlock - 1];
      if (s_w[kScanBlock - 1] > c_w) c_w = s_w[kScanBlock - 1];
      if (s_d[kScanBlock - 1] > c_d) c_d = s_d[kScanBlock - 1];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ parity phase B: carry --
constexpr int kResolveBlock = 256;

__device__ __forceinline__ bool same_bits(V3 a, V3 b) {
  return __float_as_uint(a.x) == __float_as_uint(b.x) &&
         __float_as_uint(a.y) == __float_as_uint(b.y) &&
         __float_as_uint(a.z) == __float_as_uint(b.z);
}

__global__ void __launch_bounds__(kResolveBlock) k_resolve(
    Scene sc, int maxrec, const long long* __restrict__ dep_pix,
    const long long* __restrict__ dep_key, const DepRec* __restrict__ deprec,
    const float4* __restrict__ wcarry, const int* __restrict__ seg_start,
    const int* __restrict__ nseg_p, const int* __restrict__ ndep_p, int* __restrict__ head,
    float4* __restrict__ cin) {
  __shared__ int s_seg, s_first, s_nvalid;
  __shared__ float s_c[3];
  const int nseg = *nseg_p;
  const int ndep = *ndep_p;
  for (;;) {
    if (threadIdx.x == 0) s_seg = atomicAdd(head, 1);
    __syncthreads();
    const int seg = s_seg;
    __syncthreads();
    if (seg >= nseg) break;
    int j = seg_start[seg];
    const long long key = dep_key[j];
    V3 carry = v3(0.0f, 0.0f, 0.0f);
    if (key >= 0) {
      const float4 k4 = wcarry[key];
      carry = v3(k4.x, k4.y, k4.z);
    }
    for (;;) {
      if (threadIdx.x == 0) {
        s_first = kResolveBlock;
        s_nvalid = kResolveBlock;
      }
      __syncthreads();
      const int jj = j + (int)threadIdx.x;
      const bool valid = jj < ndep && dep_key[jj] == key;
      V3 o = carry;
      bool changed = false;
      if (valid) {
        int zero = 0;
        o = carry_path(sc, deprec[dep_pix[jj]], maxrec, carry, zero);
        changed = !same_bits(o, carry);
      } else {
        atomicMin(&s_nvalid, (int)threadIdx.x);
      }
      if (changed) atomicMin(&s_first, (int)threadIdx.x);
      __syncthreads();
      const int first = s_first, nvalid = s_nvalid;
      const int lim = first < kResolveBlock ? first + 1 : nvalid;
      if ((int)threadIdx.x < lim) cin[jj] = make_float4(carry.x, carry.y, carry.z, 0.0f);
      if ((int)threadIdx.x == first) {
        s_c[0] = o.x;
        s_c[1] = o.y;
        s_c[2] = o.z;
      }
      __syncthreads();
      if (first < kResolveBlock) {
        carry = v3(s_c[0], s_c[1], s_c[2]);
        j += first + 1;
        __syncthreads();
        continue;
      }
      if (nvalid == kResolveBlock) {
        j += kResolveBlock;
        continue;
      }
      break;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ parity phase C --
__global__ void __launch_bounds__(kBlock) k_phase_c(Scene sc, Cam cam, int W, int maxrec,
                                                    const long long* __restrict__ dep_pix,
                                                    const float4* __restrict__ cin,
                                                    const int* __restrict__ ndep_p,
                                                    uint8_t* __restrict__ out,
                                                    unsigned long long* __restrict__ zcount) {
  const int ndep = *ndep_p;
  int zero = 0;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < ndep; j += gridDim.x * blockDim.x) {
    const long long p = dep_pix[j];
    const int y = (int)(p / W), x = (int)(p % W);
    const V3 d = primary_dir(cam, x, y, zero);
    const float4 c4 = cin[j];
    PixelOut po;
    shoot<kModeParityC>(sc, d, maxrec, v3(c4.x, c4.y, c4.z), po, zero);
    store_rgb(out + (size_t)p * 3, po.rgb);
  }
  flush_events(zero, zcount);
}

// ---------------------------------------------------------------------- launchers --
static Scene make_scene(const LaunchScene& s) {
  Scene sc;
  sc.shapes = s.shapes;
  sc.lights = s.lights;
  sc.pairs = s.pairs;
  sc.n = s.n;
  sc.m = s.m;
  return sc;
}
static Cam make_cam(const LaunchScene& s, int W, int H) {
  Cam c;
  c.hx = 0.0 - (double)s.cam_w / 2.0;
  c.hy = 0.0 + (double)s.cam_h / 2.0;
  c.pw = s.cam_w / (float)W;
  c.ph = s.cam_h / (float)H;
  return c;
}

hipError_t launch_render(const LaunchScene& s, int W, int H, int row0, int row_step, int nrows,
                         int maxrec, uint8_t* out, unsigned long long* zcount,
                         hipStream_t stream) {
  dim3 grid((W + kTile - 1) / kTile, (nrows + kTile - 1) / kTile);
  hipLaunchKernelGGL(k_render, grid, dim3(kBlock), 0, stream, make_scene(s), make_cam(s, W, H),
                     W, H, row0, row_step, nrows, maxrec, out, zcount);
  return hipGetLastError();
}

hipError_t launch_parity(const LaunchScene& s, int W, int H, int maxrec, uint8_t* out,
                         const ParityWork& w, unsigned long long* zcount, hipStream_t stream,
                         hipEvent_t ev_a, hipEvent_t ev_b, hipEvent_t ev_c) {
  const Scene sc = make_scene(s);
  const Cam cam = make_cam(s, W, H);
  dim3 grid((W + kTile - 1) / kTile, (H + kTile - 1) / kTile);
  hipLaunchKernelGGL(k_phase_a, grid, dim3(kBlock), 0, stream, sc, cam, W, H, maxrec, out,
                     w.cls, w.wcarry, (DepRec*)w.deprec, zcount);
  if (ev_a) (void)hipEventRecord(ev_a, stream);
  (void)hipMemsetAsync(w.counters, 0, 4 * sizeof(int), stream);   // nseg, head, ndep, pad
  hipLaunchKernelGGL(k_row_stats, dim3(H), dim3(kScanBlock), 0, stream, w.cls, W, w.row_ndep,
                     w.row_lastw, w.row_lastdep);
  hipLaunchKernelGGL(k_row_scan, dim3(1), dim3(1024), 0, stream, H, w.row_ndep, w.row_lastw,
                     w.row_lastdep, w.row_off, w.row_prevw, w.row_prevdep, w.counters + 2);
  hipLaunchKernelGGL(k_row_compact, dim3(H), dim3(kScanBlock), 0, stream, w.cls, W, w.row_off,
                     w.row_prevw, w.row_prevdep, w.dep_pix, w.dep_key, w.seg_start,
                     w.counters + 0);
  hipLaunchKernelGGL(k_resolve, dim3(w.resolve_blocks), dim3(kResolveBlock), 0, stream, sc,
                     maxrec, w.dep_pix, w.dep_key, (const DepRec*)w.deprec, w.wcarry,
                     w.seg_start, w.counters + 0, w.counters + 2, w.counters + 1, w.cin);
  if (ev_b) (void)hipEventRecord(ev_b, stream);
  hipLaunchKernelGGL(k_phase_c, dim3(w.phase_c_blocks), dim3(kBlock), 0, stream, sc, cam, W,
                     maxrec, w.dep_pix, w.cin, w.counters + 2, out, zcount);
  if (ev_c) (void)hipEventRecord(ev_c, stream);
  return hipGetLastError();
}

size_t deprec_bytes() { return sizeof(DepRec); }

}  // namespace rc
