// rc_kernels.hip — HIP kernels of the MI355X raycaster (gfx950).
//
//   k_render      one lane per pixel, 16x16-pixel workgroups (four 8x8 wave tiles for ray
//                 coherence), full iterative_shoot + quantisation, RGB store.  Fast mode, and
//                 parity mode at depth 0 (no bounce loop => no carry).
//   k_classify    parity phase A, carry part: per pixel the class (ident / writer / DEP: a
//                 pixel whose first reflection misses reads the scan-order carry), the DEP
//                 record and the writers' carry-out — no shading.
//   k_phase_a     the same plus the shading of every non-DEP pixel (used without the side
//                 stream); with it, that shading runs in k_side beside the resolver.
//   k_row_stats / k_row_scan / k_row_compact
//                 scan-order list of the DEP pixels and the segment table (start, writer key),
//                 one wave per row with ballot scans.
//   k_resolve     parity phase B: exact carry chain.  One workgroup per segment (dequeued
//                 from a counter): evaluate a window of DEP pixels at the current carry in
//                 parallel, the first pixel that changes the carry ends the step.
//   k_side        side stream, beside the resolver: shade the non-DEP pixels, then every DEP
//                 pixel with its resolved carry-in (parity phase C) as the carries appear.
//   k_finish      after the resolver: whatever k_side has not claimed.
//   k_render_cuda RC_MODE_CUDA: k_render's layout with the CUDA port's arithmetic
//                 (rc_cudasem.hpp).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "rc_cudasem.hpp"
#include "rc_device.hpp"
#include "rc_kernels.h"

// Which kernels use the cross-term-free quadric form (quad_x0: Scene::has_quadric == 2,
// rc_device.hpp quad_abc) when the scene allows it.  A kernel with 0 folds has_quadric to 0/1,
// so quad_x0 is a constant false there and the form and its branches are compiled out.
#ifndef RC_EXP_NODEPW
#define RC_EXP_NODEPW 0   // timing attribution build only (wrong images): phase A without its
                          // DEP record and primary-shade stores
#endif
#ifndef RC_X0_PIXEL
#define RC_X0_PIXEL 1     // k_render, k_phase_a, k_classify
#endif
#ifndef RC_X0_PHASE_C
#define RC_X0_PHASE_C 0   // k_dep_chunks, k_finish, k_side
#endif
#ifndef RC_X0_RESOLVE
#define RC_X0_RESOLVE 0   // k_resolve (its inlined phase C included)
#endif
#ifndef RC_PHASE_A_WAVES
#define RC_PHASE_A_WAVES 4   // waves per SIMD the render kernels are compiled for
#endif

namespace rc {

// Pixel kernels: a workgroup renders a 16x16-pixel tile of four 8x8 wave tiles (ray coherence
// inside a wave); each lane stores its own three framebuffer bytes.  The LDS-staged form
// (RC_TILE_STAGE=1, built as libraycast_hip_coalesced.so with 32x8 tiles) writes every tile row
// as one 96-byte run instead: rocprofv3 WRITE_SIZE of k_render at quadric 4096^2 50.6 MB (=
// the 50.3 MB framebuffer) against 64.0 MB for the lane stores, but k_render 0.74-0.76 ms
// against 0.69 ms and phase A 0.93-0.96 against 0.86 ms: these kernels are VALU-
// bound and their stores use < 1 % of HBM bandwidth, so the lane stores are the default.
#ifndef RC_TILE_W
#define RC_TILE_W 16
#endif
#ifndef RC_TILE_STAGE
#define RC_TILE_STAGE 0   // 1: tiles staged in LDS, written as whole rows (variant)
#endif
constexpr int kTileW = RC_TILE_W, kTileH = 256 / RC_TILE_W;
constexpr int kBlock = kTileW * kTileH;
static_assert(kTileW % 8 == 0 && kTileH % 8 == 0, "8x8 wave tiles");

// XCD-aware tile order (MI355X_MICROARCH.md: workgroups are dealt round-robin to the 8 XCDs,
// each with its own L2).  With the grid's own order, horizontally adjacent tiles run on
// different XCDs, so a 128-byte line of class bytes (8 tiles wide) or of framebuffer bytes
// (~3 tiles) is written piecewise from several L2s and reaches HBM as partial-line writes
// (rocprofv3 WRITE_SIZE of k_phase_a 1.26x its bytes).
//   RC_XCD_TILES 1: XCD k takes the k-th contiguous eighth of the tiles — measured: phase A
//                   0.745 -> 0.878 ms (the image's heavy bands land on a few XCDs);
//   RC_XCD_TILES 2: chunks of 8 horizontally adjacent tiles per XCD, chunks dealt round-robin
//                   (a line's tiles share one L2; the load stays interleaved).
#ifndef RC_XCD_TILES
#define RC_XCD_TILES 2   // measured: k_phase_a WRITE_SIZE 312 -> 269 MB in flight, time within noise
#endif
// order: RC_XCD_TILES for k_phase_a; k_render keeps the grid order (its only stores are the
// framebuffer's; fast mode 0.64 ms in round 3 against 0.65-0.66 ms with chunks, r04l)
template <int kOrder = RC_XCD_TILES>
__device__ __forceinline__ void xcd_tile(int& bx, int& by) {
  const int nx = gridDim.x, n = nx * (int)gridDim.y;
  const int lin = (int)blockIdx.y * nx + (int)blockIdx.x;
  int t = lin;
  if (kOrder == 1) {
    const int xcd = lin & 7, k = lin >> 3, q = n >> 3, r = n & 7;
    // XCDs below r take q + 1 tiles, the others q: a bijection of [0, n)
    t = xcd < r ? xcd * (q + 1) + k : r * (q + 1) + (xcd - r) * q + k;
  } else if (kOrder == 2 && lin < (n & ~63)) {
    // the XCD's k-th workgroup -> chunk (k / 8) * 8 + xcd, tile k % 8 of it (a bijection of
    // the first n & ~63 tiles; the rest keep the grid order)
    const int xcd = lin & 7, k = lin >> 3;
    t = ((k >> 3) * 8 + xcd) * 8 + (k & 7);
  }
  bx = t % nx;
  by = t / nx;
}

__device__ __forceinline__ void tile_pixel(int& lx, int& ly) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  lx = (wave % (kTileW / 8)) * 8 + (lane & 7);
  ly = (wave / (kTileW / 8)) * 8 + (lane >> 3);
}

// A tile's framebuffer bytes (and, for phase A, its class bytes) staged in LDS: every lane
// drops its 3 (1) bytes in, then the workgroup writes each row of the tile as one contiguous
// run — dword stores when the run is whole and 4-byte aligned (W % 4 == 0), bytes otherwise —
// instead of three byte stores per lane into 8-pixel row fragments (the store
// north_star names is the coalesced one; C/raycast.c:122-127 is the store replaced).
struct TileBytes {
  uint32_t rgb[kTileH][kTileW * 3 / 4];
  uint32_t cls[kTileH][kTileW / 4];
  int done;   // waves that have staged their pixels
};

// Zeroes the wave counter; the caller's next barrier publishes it.
__device__ __forceinline__ void tile_init(TileBytes& t) {
  if (threadIdx.x == 0) t.done = 0;
}

// No workgroup barrier before the row writes (waiting for the slowest wave of a tile held the
// others' slots: measured +7 % on k_render): each wave releases its staged bytes and counts
// itself in; the LAST wave of the tile writes every row and the others simply end.
__device__ __forceinline__ bool tile_last_wave(TileBytes& t) {
  if (!RC_TILE_STAGE) return false;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  int old = 0;
  if ((threadIdx.x & 63) == 0)
    old = __hip_atomic_fetch_add(&t.done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0, 64);
  if (old != kBlock / 64 - 1) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return true;
}

__device__ __forceinline__ void tile_put_rgb(TileBytes& t, int lx, int ly, uint8_t r, uint8_t g,
                                             uint8_t b, uint8_t* direct) {
  if (!RC_TILE_STAGE) {   // the default: the lane's own three byte stores
    direct[0] = r;
    direct[1] = g;
    direct[2] = b;
    return;
  }
  uint8_t* q = (uint8_t*)t.rgb[ly] + lx * 3;
  q[0] = r;
  q[1] = g;
  q[2] = b;
}

// Row ly of the tile goes to dst_row(ly) (nullptr: the row is outside the image), nbytes
// valid bytes per row.  The tile's last wave calls this (tile_last_wave).
template <int kWords, typename RowPtr>
__device__ __forceinline__ void tile_write_rows(const uint32_t (*src)[kWords], RowPtr dst_row,
                                                int nbytes) {
  const int t = threadIdx.x & 63;   // one wave writes the tile (tile_last_wave)
  for (int i = t; i < kTileH * kWords; i += 64) {
    const int ly = i / kWords, k = i % kWords;
    uint8_t* d = dst_row(ly);
    if (!d) continue;
    if (nbytes == kWords * 4 && ((uintptr_t)d & 3u) == 0u) {
      ((uint32_t*)d)[k] = src[ly][k];
    } else {
      const uint8_t* sb = (const uint8_t*)src[ly];
      for (int b = k * 4; b < k * 4 + 4 && b < nbytes; ++b) d[b] = sb[b];
    }
  }
}

__device__ __forceinline__ void store_rgb(uint8_t* __restrict__ p, V3 c) {
  p[0] = quant(c.x);
  p[1] = quant(c.y);
  p[2] = quant(c.z);
}

// Phase C's store of DEP entry j at pixel p: the framebuffer, and — when the host is copying
// the framebuffer out while the resolver runs (rc_render) — the entry's packed RGB in `patch`,
// which the host then scatters over the DEP pixels of its copy.  The top byte is the frame's
// mark (patch_mark of its epoch `tag`): one 4-byte store carries colour and mark together, so a
// host reading mapped memory during the frame scatters an entry as soon as it sees the mark.
__device__ __forceinline__ void store_dep(uint8_t* __restrict__ out, uint32_t* __restrict__ patch,
                                          unsigned tag, long long p, int j, V3 c) {
  const uint8_t r = quant(c.x), g = quant(c.y), b = quant(c.z);
  uint8_t* q = out + (size_t)p * 3;
  q[0] = r;
  q[1] = g;
  q[2] = b;
  if (patch) patch[j] = patch_mark(tag) | (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16);
}

__device__ __forceinline__ void flush_events(int zero_events, unsigned long long* counter) {
  if (zero_events) atomicAdd(counter, (unsigned long long)zero_events);
}

// The pixel kernels' divergent record reads (the winner's frame, shading record and colour
// pairs: Scene::lshapes / lpairs) come from an LDS copy of the scene when it is small
// enough: an LDS read instead of a vector-memory round trip per lane.  The
// uniform loops over shapes and lights keep their scalar loads.
constexpr int kStageShapes = 32;   // shape records, phantom included
constexpr int kStagePairs = 128;   // (shape, light) colour pairs
struct SceneStage {
  rc_shape shapes[kStageShapes];
  rc_shade_pair pairs[kStagePairs];
};
template <bool kStage>
struct StageBuf {
  SceneStage s;
};
template <>
struct StageBuf<false> {
  int unused;
};

// Every thread of the workgroup must call this (it has a barrier).
template <bool kStage>
__device__ __forceinline__ void stage_scene(Scene& sc, StageBuf<kStage>& buf) {
  if constexpr (kStage) {
    const int ws = (int)(sizeof(rc_shape) / 4) * (sc.n + 1);
    for (int i = threadIdx.x; i < ws; i += blockDim.x)
      ((unsigned*)buf.s.shapes)[i] = ((const unsigned*)sc.shapes)[i];
    const int wp = (int)(sizeof(rc_shade_pair) / 4) * (sc.n + 1) * sc.m;
    for (int i = threadIdx.x; i < wp; i += blockDim.x)
      ((unsigned*)buf.s.pairs)[i] = ((const unsigned*)sc.pairs)[i];
    __syncthreads();
    sc.lshapes = buf.s.shapes;
    sc.lpairs = buf.s.pairs;
  }
}

// ------------------------------------------------------------------ fast / depth 0 --
template <bool kStage>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RC_PHASE_A_WAVES))) k_render(Scene sc, Cam cam, int W, int H, int row0,
                                                   int row_step, int nrows, int maxrec,
                                                   uint8_t* __restrict__ out,
                                                   unsigned long long* __restrict__ zcount) {
  if (!RC_X0_PIXEL) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  __shared__ StageBuf<kStage> stage;
  __shared__ TileBytes tb;
  tile_init(tb);
  stage_scene<kStage>(sc, stage);
  if (!kStage) __syncthreads();
  int lx, ly;
  tile_pixel(lx, ly);
  int bx, by;
  xcd_tile<0>(bx, by);
  const int x0 = bx * kTileW, r0 = by * kTileH;
  const int x = x0 + lx;
  const int r = r0 + ly;           // local (shard) row
  if (x < W && r < nrows) {
    const int y = row0 + r * row_step;
    int zero = 0;
    const V3 d = primary_dir(cam, x, y, zero);
    PixelOut po;
    shoot<kModeFast>(sc, d, maxrec, v3(0.0f, 0.0f, 0.0f), po, zero);
    tile_put_rgb(tb, lx, ly, quant(po.rgb.x), quant(po.rgb.y), quant(po.rgb.z),
                 out + ((size_t)r * W + x) * 3);
    flush_events(zero, zcount);
  }
  if (!tile_last_wave(tb)) return;
  const int nx = W - x0 < kTileW ? W - x0 : kTileW;
  tile_write_rows<kTileW * 3 / 4>(tb.rgb, [&](int q) -> uint8_t* {
    return r0 + q < nrows ? out + ((size_t)(r0 + q) * W + x0) * 3 : nullptr;
  }, nx * 3);
}

// ------------------------------------------------------- CUDA-port semantics (f4) --
// One lane per pixel like k_render; up to maxrec - 1 bounces (MAX_ITER, CUDA/raycast.cu:13).
template <bool kStage>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RC_PHASE_A_WAVES))) k_render_cuda(
    Scene sc, Cam cam, int W, int row0, int row_step, int nrows, int maxrec,
    uint8_t* __restrict__ out) {
  __shared__ StageBuf<kStage> stage;
  stage_scene<kStage>(sc, stage);
  int lx, ly;
  tile_pixel(lx, ly);
  const int x = blockIdx.x * kTileW + lx;
  const int r = blockIdx.y * kTileH + ly;   // local (shard) row
  if (x >= W || r >= nrows) return;
  const V3 c = cusem::render_pixel(sc, cam, x, row0 + r * row_step, maxrec - 1);
  store_rgb(out + ((size_t)r * W + x) * 3, c);
}

// ------------------------------------------------------------------ parity phase A --
// A writer's carry-out is read only as a segment key: the last writer before a DEP pixel in
// scan order (seg_init_carry), and by the row shards the last writer before a DEP pixel in its
// row or the last writer of a row (k_shard_pack).  Inside the lane's 8-pixel row fragment of
// the wave tile (lane = 8 * row + x), a writer followed by another writer with no DEP pixel
// between them is neither, so phase A stores only the others: a writer with no later writer
// in its fragment, or with a DEP pixel before the next one.  At quadric 4096^2 that drops most
// of the 1.8 M sparse 16-byte stores (a few thousand keys are ever read).
#ifndef RC_WKEY
#define RC_WKEY 1   // 0: every writer stores its carry-out (round 3)
#endif
__device__ __forceinline__ bool writer_may_key(unsigned long long mw, unsigned long long md) {
  if (!RC_WKEY) return true;
  const int l = threadIdx.x & 63, fe = l | 7;
  const unsigned long long upto = fe == 63 ? ~0ull : ((1ull << (fe + 1)) - 1ull);
  const unsigned long long above = upto & ~((2ull << l) - 1ull);   // lanes l+1 .. fe (l = 63: none)
  const unsigned long long nwm = mw & above;
  if (!nwm) return true;
  const int nw = __ffsll((long long)nwm) - 1;
  return (md & above & ((1ull << nw) - 1ull)) != 0ull;
}

template <bool kStage>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RC_PHASE_A_WAVES))) k_phase_a(Scene sc, Cam cam, int W, int row0, int row_step, int nrows, int maxrec,
                                                    uint8_t* __restrict__ out,
                                                    uint8_t* __restrict__ cls,
                                                    float4* __restrict__ wcarry,
                                                    DepLine* __restrict__ deprec,
                                                    unsigned long long* __restrict__ zcount,
                                                    int rpitch) {
  if (!RC_X0_PIXEL) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  __shared__ StageBuf<kStage> stage;
  __shared__ TileBytes tb;
  tile_init(tb);
  stage_scene<kStage>(sc, stage);
  if (!kStage) __syncthreads();
  int lx, ly;
  tile_pixel(lx, ly);
  // local row y (a shard renders rows row0 + y * row_step of the image; the whole image:
  // 0, 1, H); every per-pixel buffer is indexed by the local pixel
  int bx, by;
  xcd_tile(bx, by);
  const int x0 = bx * kTileW, y0 = by * kTileH;
  const int x = x0 + lx;
  const int y = y0 + ly;
  if (x < W && y < nrows) {
    const size_t p = (size_t)y * W + x;
    int zero = 0;
    const V3 d = primary_dir(cam, x, row0 + y * row_step, zero);
    PixelOut po;
    shoot<kModeParityA>(sc, d, maxrec, v3(0.0f, 0.0f, 0.0f), po, zero);
    if (RC_TILE_STAGE) ((uint8_t*)tb.cls[ly])[lx] = po.cls;
    else cls[p] = po.cls;
    // DEP lines and writer carries at row pitch rpitch (W: the local pixel; a row shard's root
    // passes G * W with the buffers offset by row0 * W: the IMAGE pixel, i.e. straight into the
    // root resolver's lone-frame layout, k_shard_pack thin entries)
    const size_t pr = (size_t)y * rpitch + x;
    if (po.cls == kClsDep) {
      // one 64-byte line: the record and, under dep_fast, the primary shade for phase C; this
      // part's events are counted here (else phase C recomputes the whole pixel and counts its
      // events).  The pixel's framebuffer bytes are phase C's: the tile writes a placeholder.
      if (!RC_EXP_NODEPW) {
        deprec[pr].r = po.dep;
        if (sc.dep_fast)
          *(float4*)&deprec[pr].px = make_float4(po.pcol.x, po.pcol.y, po.pcol.z, 0.0f);
      }
      if (sc.dep_fast) flush_events(zero, zcount);
      if (RC_TILE_STAGE) tile_put_rgb(tb, lx, ly, 0, 0, 0, nullptr);
    } else {
      tile_put_rgb(tb, lx, ly, quant(po.rgb.x), quant(po.rgb.y), quant(po.rgb.z), out + p * 3);
      flush_events(zero, zcount);
    }
    const unsigned long long mw = __ballot(po.cls == kClsWriter);
    const unsigned long long md = __ballot(po.cls == kClsDep);
    if (po.cls == kClsWriter && writer_may_key(mw, md))
      wcarry[pr] = make_float4(po.carry.x, po.carry.y, po.carry.z, 0.0f);
  }
  if (!tile_last_wave(tb)) return;
  const int nx = W - x0 < kTileW ? W - x0 : kTileW;
  auto row_at = [&](uint8_t* base, int q, int bpp) -> uint8_t* {
    return y0 + q < nrows ? base + ((size_t)(y0 + q) * W + x0) * bpp : nullptr;
  };
  tile_write_rows<kTileW * 3 / 4>(tb.rgb, [&](int q) { return row_at(out, q, 3); }, nx * 3);
  tile_write_rows<kTileW / 4>(tb.cls, [&](int q) { return row_at(cls, q, 1); }, nx);
}

// Phase A's carry part only (no shading): k_side shades the non-DEP pixels off the critical path.
template <bool kStage>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RC_PHASE_A_WAVES))) k_classify(Scene sc, Cam cam, int W, int H, int maxrec,
                                                     uint8_t* __restrict__ cls,
                                                     float4* __restrict__ wcarry,
                                                     DepLine* __restrict__ deprec) {
  if (!RC_X0_PIXEL) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  __shared__ StageBuf<kStage> stage;
  stage_scene<kStage>(sc, stage);
  int lx, ly;
  tile_pixel(lx, ly);
  const int x = blockIdx.x * kTileW + lx;
  const int y = blockIdx.y * kTileH + ly;
  if (x >= W || y >= H) return;
  const size_t p = (size_t)y * W + x;
  int zero = 0;   // events are counted by the shading passes
  const V3 d = primary_dir(cam, x, y, zero);
  PixelOut po;
  shoot<kModeClassify>(sc, d, maxrec, v3(0.0f, 0.0f, 0.0f), po, zero);
  cls[p] = po.cls;
  if (po.cls == kClsDep) deprec[p].r = po.dep;
  else if (po.cls == kClsWriter) wcarry[p] = make_float4(po.carry.x, po.carry.y, po.carry.z, 0.0f);
}

// ------------------------------------------------------- scan-order DEP compaction --
// The DEP pixels in scan order (dep_pix, the resolver's and phase C's index), the segment
// table (seg_start: first DEP index of every segment, seg_key: the writer pixel before it,
// -1 = none) and the totals (counters[0] = segments, counters[2] = DEP pixels).  A segment
// starts at a DEP pixel with no DEP pixel before it, or with a writer between it and the
// previous DEP pixel.  One wave per row, ballot scans (no LDS, no barriers); the DEP records
// stay where phase A wrote them (pixel-indexed) and the resolver gathers them by dep_pix.
//   k_row_stats  per row: DEP count, segment starts decided inside the row, last writer,
//                last DEP, the writer before the row's first DEP
//   k_row_scan   one workgroup: exclusive scans over the rows (DEP offsets, last writer /
//                last DEP before each row), the first DEP's start decision, segment offsets
//   k_row_compact per row: dep_pix, seg_start, seg_key
constexpr int kRowWaves = 4;   // rows per 256-thread workgroup

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}
__device__ __forceinline__ int hi_bit(unsigned long long m) { return 63 - __clzll((long long)m); }

struct RowStats {
  int ndep, nstart;        // DEP pixels; segment starts other than the row's first DEP
  long long lastw, lastd;  // last writer / DEP pixel of the row (-1: none)
  long long wfirst;        // last writer before the row's first DEP pixel (-1: none)
};

// A row's class bytes reach LDS in 4 KiB chunks, 16 bytes per lane per load (a wave's 64
// one-byte loads per chunk of 64 pixels were a chain of dependent round trips: k_row_stats
// 39 us, k_row_compact 29 us at 4096^2); the ballot scans then read LDS.
constexpr int kRowChunk = 4096;
__device__ __forceinline__ void stage_row_chunk(const uint8_t* __restrict__ src, int n,
                                                uint8_t* __restrict__ buf, int lane) {
  if ((((size_t)src) & 15) == 0) {
    for (int o = lane * 16; o < n; o += 64 * 16) {
      if (o + 16 <= n) {
        *(uint4*)(buf + o) = *(const uint4*)(src + o);
      } else {
        for (int i = o; i < n; ++i) buf[i] = src[i];
      }
    }
  } else {
    for (int i = lane; i < n; i += 64) buf[i] = src[i];
  }
}

// The one-workgroup kernels of the compaction (k_row_scan, k_seg_order) run as
// kScanBlock threads.  With frames in flight they are dispatched beside the next frame's
// phase A, whose workgroups (4 waves of 128 VGPRs) refill every CU slot they free: a
// 1024-thread workgroup needs a whole CU's wave slots at once and waited 0.05-1.2 ms for one
// (k_row_scan 0.164 ms mean in flight against 13 us alone, profiles/r05_rocprof_headline_...),
// holding the frame's resolver back; 256 threads fit the slot one phase A workgroup frees.
// k_row_scan: chunks of kScanBlock * kScanRows rows, kScanRows consecutive rows per thread
// (their loads issued together), a thread-level pass, block scans of the thread totals + a
// chunk carry.  (One row per thread took four dependent load/scan/store rounds at 4096 rows:
// 16 us.)
#ifndef RC_SCAN_BLOCK
#define RC_SCAN_BLOCK 256
#endif
constexpr int kScanBlock = RC_SCAN_BLOCK;
constexpr int kScanRows = kScanBlock >= 1024 ? 4 : 8;
static_assert(kScanBlock % 64 == 0 && kScanBlock <= 1024, "whole waves, at most 16");

// block-wide exclusive scan of (sum, max, max) over the workgroup; returns the block
// totals in t_cnt / t_w / t_d
__device__ __forceinline__ void block_scan3(int& cnt, long long& lw, long long& ld, int* w_cnt,
                                            long long* w_w, long long* w_d, int& t_cnt,
                                            long long& t_w, long long& t_d) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  int c = cnt;
  long long a = lw, d = ld;
  for (int o = 1; o < 64; o <<= 1) {   // inclusive wave scans
    const int c2 = __shfl_up(c, o, 64);
    const long long a2 = __shfl_up(a, o, 64), d2 = __shfl_up(d, o, 64);
    if (lane >= o) {
      c += c2;
      a = a2 > a ? a2 : a;
      d = d2 > d ? d2 : d;
    }
  }
  if (lane == 63) {
    w_cnt[wave] = c;
    w_w[wave] = a;
    w_d[wave] = d;
  }
  __syncthreads();
  int pc = 0;
  long long pw = -1, pd = -1;
  for (int q = 0; q < wave; ++q) {
    pc += w_cnt[q];
    pw = w_w[q] > pw ? w_w[q] : pw;
    pd = w_d[q] > pd ? w_d[q] : pd;
  }
  t_cnt = 0;
  t_w = -1;
  t_d = -1;
  for (int q = 0; q < nw; ++q) {
    t_cnt += w_cnt[q];
    t_w = w_w[q] > t_w ? w_w[q] : t_w;
    t_d = w_d[q] > t_d ? w_d[q] : t_d;
  }
  // exclusive: the wave prefix combined with the lanes before this one
  int ec = __shfl_up(c, 1, 64);
  long long ea = __shfl_up(a, 1, 64), ed = __shfl_up(d, 1, 64);
  if (lane == 0) {
    ec = 0;
    ea = -1;
    ed = -1;
  }
  cnt = pc + ec;
  lw = ea > pw ? ea : pw;
  ld = ed > pd ? ed : pd;
  __syncthreads();   // the wave totals are rewritten by the next scan
}

// the scan over the rows by one workgroup (any multiple of 64 threads up to 1024)
__device__ __forceinline__ void row_scan_body(int H, const RowStats* __restrict__ rs,
                                              int* __restrict__ row_off,
                                              int* __restrict__ row_soff,
                                              long long* __restrict__ row_prevw,
                                              long long* __restrict__ row_prevd,
                                              int* __restrict__ counters) {
  __shared__ int w_cnt[16];
  __shared__ long long w_w[16], w_d[16];
  int c_cnt = 0, c_seg = 0;           // chunk carries (every thread holds the same values)
  long long c_w = -1, c_d = -1;
  for (int y0 = 0; y0 < H; y0 += (int)blockDim.x * kScanRows) {
    const int yb = y0 + threadIdx.x * kScanRows;
    RowStats r[kScanRows];
#pragma unroll
    for (int k = 0; k < kScanRows; ++k)
      r[k] = yb + k < H ? rs[yb + k] : RowStats{0, 0, -1, -1, -1};
    // thread totals over its rows
    int cnt = 0;
    long long lw = -1, ld = -1;
#pragma unroll
    for (int k = 0; k < kScanRows; ++k) {
      cnt += r[k].ndep;
      lw = r[k].lastw > lw ? r[k].lastw : lw;
      ld = r[k].lastd > ld ? r[k].lastd : ld;
    }
    int t_cnt;
    long long t_w, t_d;
    block_scan3(cnt, lw, ld, w_cnt, w_w, w_d, t_cnt, t_w, t_d);
    // this thread's exclusive prefix, with the chunk carry
    int pc = c_cnt + cnt;
    long long pw = lw > c_w ? lw : c_w, pdd = ld > c_d ? ld : c_d;
    // per row: exclusive values, the first DEP's start decision, segment counts
    int nseg[kScanRows];
    int segsum = 0;
#pragma unroll
    for (int k = 0; k < kScanRows; ++k) {
      nseg[k] = r[k].nstart;
      if (r[k].ndep > 0) {
        const long long key = r[k].wfirst > pw ? r[k].wfirst : pw;
        if (pdd < 0 || key > pdd) nseg[k] += 1;
      }
      if (yb + k < H) {
        row_off[yb + k] = pc;
        row_prevw[yb + k] = pw;
        row_prevd[yb + k] = pdd;
      }
      pc += r[k].ndep;
      pw = r[k].lastw > pw ? r[k].lastw : pw;
      pdd = r[k].lastd > pdd ? r[k].lastd : pdd;
      segsum += nseg[k];
    }
    // segment offsets: a second block scan (sum)
    int sc = segsum;
    long long dw = -1, dd = -1;
    int t_seg;
    long long u1, u2;
    block_scan3(sc, dw, dd, w_cnt, w_w, w_d, t_seg, u1, u2);
    int ps = c_seg + sc;
#pragma unroll
    for (int k = 0; k < kScanRows; ++k) {
      if (yb + k < H) row_soff[yb + k] = ps;
      ps += nseg[k];
    }
    c_cnt += t_cnt;
    c_seg += t_seg;
    c_w = t_w > c_w ? t_w : c_w;
    c_d = t_d > c_d ? t_d : c_d;
  }
  if (threadIdx.x == 0) {
    counters[0] = c_seg;
    counters[2] = c_cnt;
  }
}

__global__ void __launch_bounds__(kScanBlock) k_row_scan(int H, const RowStats* __restrict__ rs,
                                                   int* __restrict__ row_off,
                                                   int* __restrict__ row_soff,
                                                   long long* __restrict__ row_prevw,
                                                   long long* __restrict__ row_prevd,
                                                   int* __restrict__ counters) {
  row_scan_body(H, rs, row_off, row_soff, row_prevw, row_prevd, counters);
}

// zero (optional): the frame's counters and TeamState words, cleared here instead of by two
// fill launches before this kernel (every workgroup clears a slice)
__global__ void __launch_bounds__(256) k_row_stats(const uint8_t* __restrict__ cls, int W, int H,
                                                   RowStats* __restrict__ rs,
                                                   int* __restrict__ counters,
                                                   uint4* __restrict__ zero, int zero_words,
                                                   int* __restrict__ zero2, int zero2_ints) {
  __shared__ __attribute__((aligned(16))) uint8_t s_row[kRowWaves][kRowChunk];
  if (zero) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    for (int i = g; i < zero_words; i += gridDim.x * 256) zero[i] = make_uint4(0, 0, 0, 0);
    for (int i = g; i < zero2_ints; i += gridDim.x * 256) zero2[i] = 0;
    if (g < 16) counters[g] = 0;
  }
  const int wave = threadIdx.x >> 6;
  const int y = blockIdx.x * kRowWaves + wave;
  const bool on = y < H;
  const int lane = threadIdx.x & 63;
  const long long base = (long long)y * W;
  const unsigned long long lt = lanemask_lt();
  int nd = 0, ns = 0;
  long long lw = -1, ld = -1, wf = -1;
  for (int xc = 0; xc < W; xc += kRowChunk) {
    const int n = W - xc < kRowChunk ? W - xc : kRowChunk;
    if (on) stage_row_chunk(cls + base + xc, n, s_row[wave], lane);
    __syncthreads();
    // unrolled so that the next sub-chunks' LDS reads issue before this one's ballots
#pragma unroll 8
    for (int x0 = xc; x0 < (on ? xc + n : xc); x0 += 64) {
      const int x = x0 + lane;
      const uint8_t c = x < W ? s_row[wave][x - xc] : kClsIdent;
      const unsigned long long md = __ballot(c == kClsDep), mw = __ballot(c == kClsWriter);
      if (md) {   // (half the image's rows hold no DEP pixel: their chunks skip this part)
        // a DEP lane (not the row's first DEP) starts a segment when a writer lies between it
        // and the previous DEP: last writer before it > previous DEP before it
        const long long kw = (mw & lt) ? base + x0 + hi_bit(mw & lt) : lw;
        const long long pd = (md & lt) ? base + x0 + hi_bit(md & lt) : ld;
        const bool st = c == kClsDep && pd >= 0 && kw > pd;
        ns += __popcll(__ballot(st));
        if (wf < 0 && ld < 0) {   // first DEP of the row is in this chunk
          const int f = __ffsll((long long)md) - 1;
          const unsigned long long wb = mw & ((f ? (~0ull >> (64 - f)) : 0ull));
          wf = wb ? base + x0 + hi_bit(wb) : lw;
        }
        nd += __popcll(md);
        ld = base + x0 + hi_bit(md);
      }
      if (mw) lw = base + x0 + hi_bit(mw);
    }
    __syncthreads();   // the chunk buffer is refilled
  }
  if (on && lane == 0) rs[y] = RowStats{nd, ns, lw, ld, wf};
}

// the segment order by one workgroup (any size)
__device__ __forceinline__ void seg_order_body(const int* __restrict__ seg_start,
                                               int* __restrict__ counters,
                                               int* __restrict__ order,
                                               int* __restrict__ batch_state,
                                               int* __restrict__ batch_cnt,
                                               int* __restrict__ batch_rq,
                                               int block_min, int block_cap,
                                               int zero_batches) {
  const int nseg = counters[0], ndep = counters[2];
  // phase C's per-batch claim words (64 DEP entries per batch), completion counts and ready
  // queue are zeroed for this frame: by k_row_stats (launch_parity, batch_ints > 0), else here
  if (zero_batches) {
    for (int b = threadIdx.x; b < (ndep + 63) / 64; b += blockDim.x) {
      batch_state[b] = 0;
      batch_cnt[b] = 0;
      batch_rq[b] = 0;
    }
  }
  if (nseg > kSegOrderMax) {
    if (threadIdx.x == 0) {
      counters[3] = 0;
      counters[14] = 0;
      counters[15] = 0;
    }
    return;
  }
  __shared__ int hist[256];
  __shared__ int off[256];
  const int t = threadIdx.x;
  for (int i = t; i < 256; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  auto bucket = [&](int s) {
    const int len = (s + 1 < nseg ? seg_start[s + 1] : ndep) - seg_start[s];
    const int b = len >> 5;
    return 255 - (b < 255 ? b : 255);
  };
  // chunked so that the scatter below keeps segment order within a bucket
  const int per = (nseg + (int)blockDim.x - 1) / (int)blockDim.x;
  const int s0 = t * per, s1 = s0 + per < nseg ? s0 + per : nseg;
  for (int s = s0; s < s1; ++s) atomicAdd(&hist[bucket(s)], 1);
  __syncthreads();
  if (t == 0) {
    int acc = 0, nlong = 0;
    int bmin = (block_min + 31) >> 5;   // smallest length bucket taken by workgroups
    if (bmin > 255) bmin = 255;
    for (int b = 0; b < 256; ++b) {
      off[b] = acc;
      acc += hist[b];
      if (block_min > 0 && 255 - b >= bmin) nlong = acc;
    }
    // whole workgroups for the long regular segments only when the regular workgroups can
    // take them in at most two turns: a workgroup resolves a 3 856-entry segment in ~0.55x a
    // lone wave's time at worst and most of them much faster (quadric 4096^2: 154 such
    // segments on 120 workgroups, all done by 2.5 ms); with more the turns queue up and it
    // loses (8192^2 lone 12.9 -> 14.4 ms, frames in flight at 4096^2 5.5e9 vs 6.3e9 rays/s)
    if (nlong > 2 * block_cap) nlong = 0;
    counters[14] = nlong;
    counters[15] = nlong;
  }
  __syncthreads();
  for (int s = s0; s < s1; ++s) order[atomicAdd(&off[bucket(s)], 1)] = s;
  if (t == 0) counters[3] = 1;
}

__global__ void __launch_bounds__(256) k_row_compact(
    const uint8_t* __restrict__ cls, int W, int H, const int* __restrict__ row_off,
    const int* __restrict__ row_soff, const long long* __restrict__ row_prevw,
    const long long* __restrict__ row_prevd, long long* __restrict__ dep_pix,
    int* __restrict__ seg_start, long long* __restrict__ seg_key) {
  __shared__ __attribute__((aligned(16))) uint8_t s_row[kRowWaves][kRowChunk];
  const int wave = threadIdx.x >> 6;
  const int y = blockIdx.x * kRowWaves + wave;
  const bool on = y < H;
  const int lane = threadIdx.x & 63;
  const long long base = (long long)y * W;
  const unsigned long long lt = lanemask_lt();
  int idx0 = on ? row_off[y] : 0, s0 = on ? row_soff[y] : 0;
  long long lw = on ? row_prevw[y] : -1, ld = on ? row_prevd[y] : -1;
  for (int xc = 0; xc < W; xc += kRowChunk) {
    const int n = W - xc < kRowChunk ? W - xc : kRowChunk;
    if (on) stage_row_chunk(cls + base + xc, n, s_row[wave], lane);
    __syncthreads();
#pragma unroll 8
    for (int x0 = xc; x0 < (on ? xc + n : xc); x0 += 64) {
      const int x = x0 + lane;
      const uint8_t c = x < W ? s_row[wave][x - xc] : kClsIdent;
      const unsigned long long md = __ballot(c == kClsDep), mw = __ballot(c == kClsWriter);
      if (md) {
        const long long kw = (mw & lt) ? base + x0 + hi_bit(mw & lt) : lw;
        const long long pd = (md & lt) ? base + x0 + hi_bit(md & lt) : ld;
        const bool dep = c == kClsDep;
        const bool st = dep && (pd < 0 || kw > pd);
        const unsigned long long ms = __ballot(st);
        if (dep) {
          const int idx = idx0 + __popcll(md & lt);
          dep_pix[idx] = base + x;
          if (st) {
            const int si = s0 + __popcll(ms & lt);
            seg_start[si] = idx;
            seg_key[si] = kw;
          }
        }
        idx0 += __popcll(md);
        s0 += __popcll(ms);
        ld = base + x0 + hi_bit(md);
      }
      if (mw) lw = base + x0 + hi_bit(mw);
    }
    __syncthreads();   // the chunk buffer is refilled
  }
}

// ------------------------------------------------------------ parity phase B: carry --
// The carry chain of one segment (DEP entries [start, end), initial carry from the writer
// before it) is resolved exactly: evaluate the transfer function f_p (carry_path) of a window
// of entries at the current carry in parallel; the FIRST entry whose output differs bitwise
// from its input is the next place the carry changes.  A wave keeps its 64 records in
// registers and re-evaluates only the lanes after each changer (ballot + shuffle, no barrier),
// so a changer costs one f_p latency.  Segments longer than `long_len` entries (one or two per
// image, up to ~10^6 entries) are resolved by a TEAM of workgroups that evaluate a
// team_blocks*256-entry window per round and agree on the first changer through a counter
// barrier (all team blocks are co-resident: they are the first blocks of a grid sized to the
// device's resident capacity).
#ifndef RC_HANDOFF_DIAG
#define RC_HANDOFF_DIAG 0   // 1: experiment builds record block 0's publish times (TeamState)
#endif
#ifndef RC_DIAG
#define RC_DIAG 0   // 1: the diagnostic builds (make stamps / stamps2) write the resolver trace
#endif
#ifndef RC_TEAM_CSCAN
#define RC_TEAM_CSCAN 1   // 0 compiles the cooperative SCAN rounds out (rc_tuning.team_cscan)
#endif
#ifndef RC_RES_GLOBAL_SCAN
#define RC_RES_GLOBAL_SCAN 0   // measured: global (scalar) records in the LANE loops: lone resolver 4.15 -> 4.35 ms
#endif
constexpr int kResolveBlock = 256;
constexpr int kTeamMax = 256;
constexpr int kLdsShapes = kLdsShapesMax;

__device__ __forceinline__ bool same_bits(V3 a, V3 b) {
  return __float_as_uint(a.x) == __float_as_uint(b.x) &&
         __float_as_uint(a.y) == __float_as_uint(b.y) &&
         __float_as_uint(a.z) == __float_as_uint(b.z);
}

__device__ __forceinline__ V3 seg_init_carry(const long long* __restrict__ seg_key,
                                             const float4* __restrict__ wcarry, int s) {
  const long long key = seg_key[s];
  if (key < 0) return v3(0.0f, 0.0f, 0.0f);
  const float4 k4 = wcarry[key];
  return v3(k4.x, k4.y, k4.z);
}

// DEP entry j's record: phase A wrote it at the pixel (dep_pix[j]); gathered, never copied.
__device__ __forceinline__ DepRec rec_at(const DepLine* __restrict__ deprec,
                                         const long long* __restrict__ dep_pix, int j) {
  return deprec[dep_pix[j]].r;   // the first 48 bytes of the line (the shade is phase C's)
}

// Resolve the 64 entries [base, base+64) ∩ [.., end) of one wave at carry `c`, changers
// included.  On return: `mine` = this lane's carry-in, `c` = carry after the window; the
// result counts transfer-function evaluation steps.  The first pass evaluates the 64
// entries one per lane.  After a changer the rest of the window is dense-prone (the carry
// creeps one entry at a time in long runs), so it continues with the cooperative evaluator:
// 64/G entries per step, shapes spread over the G lanes of each group.
__device__ __forceinline__ DepRec shfl_rec(const DepRec& r, int src) {
  DepRec o;
  o.ax = __shfl(r.ax, src, 64);
  o.ay = __shfl(r.ay, src, 64);
  o.az = __shfl(r.az, src, 64);
  o.n0x = __shfl(r.n0x, src, 64);
  o.n0y = __shfl(r.n0y, src, 64);
  o.n0z = __shfl(r.n0z, src, 64);
  o.obj0 = __shfl(r.obj0, src, 64);
  o.pad = 0;
  o.bx = __shfl(r.bx, src, 64);
  o.by = __shfl(r.by, src, 64);
  o.bz = __shfl(r.bz, src, 64);
  o.pad2 = 0;
  return o;
}

// Window state machine.  LANE: one entry per lane at the current carry (64 entries for one
// evaluation's latency: right for clean stretches).  COOP: the cooperative evaluator, 64/GE
// entries per step at a lower latency (right inside dense runs, where every entry may move
// the carry).  A changer found by a LANE pass switches to COOP; two clean COOP steps in a row
// switch back.  `dense` carries the mode into the next window.  Returns the number of
// evaluation steps; *changed tells whether any entry of the window moved the carry.
struct WinStats {
  int lane, coop, changers;
#if RC_STAMPS   // diagnostic build: cycles inside the evaluations / whole steps / waiting at
                // the step's barrier (block_window)
  unsigned long long ce, cs, cw;
#endif
};

// Carry predictor for dense runs.  Inside a run of changers the carry creeps: at quadric
// 4096^2 the seven 1 377-entry all-changer segments move one component by a near-constant
// number of float ulps per entry (9-12, 143-156, -195..-209, ...) and keep the other two.
// The cooperative evaluator then spends its spare lane groups on entry pos+1 at guessed
// carry-ins bits(c) + mean delta of the last few changes (+-1, +-2.. ulps on the moving
// component); when entry pos's exact output equals a guess bit for bit, entry pos+1's
// evaluation at that guess IS its exact evaluation and two entries retire in one step.  The
// guesses only choose what to evaluate, never what is accepted.
struct CarryHist {
  V3 h[4];   // carries after the last changes, h[0] the latest
  int n;
  int run;   // changes in a row (a hand-off to a helper block starts a long run, k_resolve)
};
#ifndef RC_PREDICT
#define RC_PREDICT 1
#endif
constexpr bool kPredict = RC_PREDICT != 0;
// Helper blocks' predictive step: 0 = its 15 guesses all for entry pos+1; k = groups 1..k guess
// pos+1 and groups k+1..15 guess pos+2 (oracle simulation of the seven dense 1 377-entry
// segments at quadric 4096^2, scripts/pred_sim.py: 1.65-1.99 entries per step with 15/0,
// 1.54-2.95 with 7/8, 1.60-2.91 with 9/6)
#ifndef RC_PRED_SPLIT
#define RC_PRED_SPLIT 0
#endif
constexpr int kPredSplit = RC_PRED_SPLIT;
__device__ __forceinline__ void hist_push(CarryHist& hs, V3 c) {
  hs.run = hs.n == 0 ? 0 : hs.run + 1;
  hs.h[3] = hs.h[2];
  hs.h[2] = hs.h[1];
  hs.h[1] = hs.h[0];
  hs.h[0] = c;
  hs.n = hs.n < 4 ? hs.n + 1 : 4;
}
// guess q (1..) of the carry after c: the mean delta of the history, in float bits, with the
// moving component offset by 0, -1, +1, -2, +2, ...
__device__ __forceinline__ V3 hist_guess(const CarryHist& hs, V3 c, int q, int mult = 1) {
  // no run-time index into h[] (it would put the history in scratch memory, whose reload
  // waits for every store in flight — the carry-in publications) and no run-time divisor
  const int m = hs.n - 1;   // 1..3
  const V3 o = sel(m == 3, hs.h[3], sel(m == 2, hs.h[2], hs.h[1]));   // not a struct ?:
  auto md = [&](float a, float b) {
    const int d = (int)(__float_as_uint(a) - __float_as_uint(b));
    const int r = d >= 0 ? 1 : -1;   // m / 2 rounded away from zero, for m = 2, 3
    return m == 1 ? d : (m == 2 ? (d + r) / 2 : (d + r) / 3);
  };
  int dx = md(hs.h[0].x, o.x), dy = md(hs.h[0].y, o.y), dz = md(hs.h[0].z, o.z);
  if (mult != 1) dx *= mult, dy *= mult, dz *= mult;
  const int j = q - 1;
  const int off = (j & 1) ? -((j + 1) >> 1) : (j >> 1);   // q = 1, 2, 3, 4.. -> 0, -1, +1, -2..
  const int ax = abs(dx), ay = abs(dy), az = abs(dz);
  if (ax >= ay && ax >= az) dx += off;
  else if (ay >= az) dy += off;
  else dz += off;
  return v3(__uint_as_float(__float_as_uint(c.x) + (unsigned)dx),
            __uint_as_float(__float_as_uint(c.y) + (unsigned)dy),
            __uint_as_float(__float_as_uint(c.z) + (unsigned)dz));
}

__device__ __forceinline__ int wave_window(const Scene& sc, int maxrec,
                                           const DepLine* __restrict__ deprec,
                                           const long long* __restrict__ dep_pix, int base,
                                           int end, V3& c, V3& mine, bool& mhit,
                                           const LaneShape& ls,
                                           int G, bool& dense, bool& changed,
                                           WinStats& ws, int K, CarryHist& hs
#if RC_STAMPS
                                           , Stamps* st_
#endif
) {
  const int lane = threadIdx.x & 63;
  const int idx = base + lane;
  const int nvalid = end - base < 64 ? end - base : 64;
  const bool valid = lane < nvalid;
  DepRec r;
  if (valid) r = rec_at(deprec, dep_pix, idx);
  mine = c;
  mhit = false;
  changed = false;
  int zero = 0;
  int evals = 0;
  int pos = 0;                     // lanes < pos are resolved
  bool coop = dense && G > 0;
  int clean_run = 0;
  const bool spec = 2 * G <= 64;
  const int GE = G > 0 ? (spec ? 2 * G : G) : 64;
  const int E = 64 / GE;
  const int e = lane / GE, kself = G > 0 ? lane % G : 0, half = spec ? (lane / G) & 1 : 0;
  while (pos < nvalid) {
    ++evals;
    if (!coop) {
      ++ws.lane;
      const bool act = valid && lane >= pos;
      V3 o = c;
      bool h = false;
#if RC_STAMPS
      const unsigned long long tl0_ = stamp_now();
#endif
      if (act) o = carry_path(sc, r, maxrec, c, zero, h);
      const unsigned long long m = __ballot(act && !same_bits(o, c));
#if RC_STAMPS
      st_->acc[0] += stamp_now() - tl0_;
#endif
      if (m == 0) {
        if (act) {
          mine = c;
          mhit = h;
        }
        hs.n = 0;
        pos = nvalid;
        break;
      }
      const int k = __ffsll((long long)m) - 1;
      if (act && lane <= k) {
        mine = c;
        mhit = h;
      }
      if (k > 0 || hs.n == 0) hs.n = 0, hist_push(hs, c);   // the run starts at this change
      c = v3(__shfl(o.x, k, 64), __shfl(o.y, k, 64), __shfl(o.z, k, 64));
      hist_push(hs, c);
      pos = k + 1;
      changed = true;
      ++ws.changers;
      coop = G > 0;
      clean_run = 0;
      continue;
    }
    ++ws.coop;
#if RC_STAMPS == 2   // coarse: acc[1] = evaluations, acc[2] = whole cooperative steps
    const unsigned long long cs0_ = __builtin_amdgcn_s_memtime();
#endif
    // predictive step (CarryHist): group 0 takes entry pos at c, the others entry pos+1 at
    // guessed carry-ins; otherwise groups take entries pos, pos+1, .. all at c
    const bool predict = hs.n >= 2 && E >= 2 && pos + 1 < nvalid && kPredict;
    const int i = predict ? pos + (e > 0 ? 1 : 0) : pos + e;
    const V3 ce = sel(predict && e > 0 && e < E, hist_guess(hs, c, e), c);
    const bool act = e < E && i < nvalid;
    const DepRec ri = shfl_rec(r, i < 64 ? i : 63);
    V3 oc = ce;
    bool hg = false;
#if RC_STAMPS
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself, G, half, ri, maxrec, ce, zero, hg, st_)
#else
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself, G, half, ri, maxrec, ce, zero, hg)
#endif
#define RC_SPEC(GT) \
  (sc.has_quadric ? (quad_x0(sc) ? RC_SPEC1(GT, 2) : RC_SPEC1(GT, 1)) : RC_SPEC1(GT, 0))
    if (act) {
      if (G == 8) oc = RC_SPEC(8);
      else if (G == 4) oc = RC_SPEC(4);
      else if (G == 16) oc = RC_SPEC(16);
      else if (spec) oc = RC_SPEC(0);
      else oc = carry_path_coop(sc, ls, kself, G, ri, maxrec, ce, zero, hg);
    }
#undef RC_SPEC
#undef RC_SPEC1
#if RC_STAMPS == 2
    st_->acc[1] += __builtin_amdgcn_s_memtime() - cs0_;
    struct StepEnd_ {
      Stamps* s;
      unsigned long long t;
      __device__ ~StepEnd_() { s->acc[2] += __builtin_amdgcn_s_memtime() - t; }
    } step_end_{st_, cs0_};
#endif
    if (predict) {
      const V3 o0 = v3(__shfl(oc.x, 0, 64), __shfl(oc.y, 0, 64), __shfl(oc.z, 0, 64));
      const bool h0 = __shfl((int)hg, 0, 64) != 0;
      if (lane == pos) {
        mine = c;
        mhit = h0;
      }
      if (same_bits(o0, c)) {   // entry pos leaves the carry: the run is over
        hs.n = 0;
        pos += 1;
        if (++clean_run >= K) coop = false;
        continue;
      }
      changed = true;
      ++ws.changers;
      clean_run = 0;
      hist_push(hs, o0);
      const unsigned long long mm =
          __ballot(act && e > 0 && (lane % GE) == 0 && same_bits(ce, o0));
      if (mm == 0) {
        c = o0;
        pos += 1;
        continue;
      }
      const int gl = __ffsll((long long)mm) - 1;   // leader lane of the matching group
      const V3 o1 = v3(__shfl(oc.x, gl, 64), __shfl(oc.y, gl, 64), __shfl(oc.z, gl, 64));
      const bool h1 = __shfl((int)hg, gl, 64) != 0;
      if (lane == pos + 1) {
        mine = o0;
        mhit = h1;
      }
      pos += 2;
      if (same_bits(o1, o0)) {
        hs.n = 0;
        c = o0;
        if (++clean_run >= K) coop = false;
      } else {
        ++ws.changers;
        hist_push(hs, o1);
        c = o1;
      }
      continue;
    }
    const unsigned long long mc = __ballot(act && (lane % GE) == 0 && !same_bits(oc, c));
    // entry pos+q's hit flag sits in its group's first lane, q*GE
    const int q = lane - pos;
    const bool hq = __shfl((int)hg, (q >= 0 && q < E ? q : 0) * GE, 64) != 0;
    if (mc == 0) {
      hs.n = 0;
      const int lim = pos + E < nvalid ? pos + E : nvalid;
      if (lane >= pos && lane < lim) {
        mine = c;
        mhit = hq;
      }
      pos = lim;
      if (++clean_run >= K) coop = false;
      continue;
    }
    const int g = (__ffsll((long long)mc) - 1) / GE;
    if (lane >= pos && lane <= pos + g) {
      mine = c;
      mhit = hq;
    }
    if (g > 0 || hs.n == 0) hs.n = 0, hist_push(hs, c);
    c = v3(__shfl(oc.x, g * GE, 64), __shfl(oc.y, g * GE, 64), __shfl(oc.z, g * GE, 64));
    hist_push(hs, c);
    pos += g + 1;
    changed = true;
    ++ws.changers;
    clean_run = 0;
  }
  dense = coop;
  return evals;
}

__device__ __forceinline__ unsigned long long pack2(unsigned lo, unsigned hi) {
  return (unsigned long long)lo | ((unsigned long long)hi << 32);
}

// Carry-in hand-off (MI355X_MICROARCH.md / cdna_hip_programming.md Guideline 16, R2): each
// entry's carry-in is three naturally aligned 8-byte granules {value, tag}, each written by ONE
// agent-scope (sc1) store, tag = this frame's epoch.  The phase-C tail (other waves of the same
// launch, any XCD) reads them with sc1 loads and accepts an entry only when all three tags
// match, so no flag, fence or ordering is involved; a stale or torn entry is simply retried.
struct CinG {
  unsigned long long g[3];
};
// The tag's top bit carries the entry's hit flag (some bounce level hit at this carry-in:
// not clean, Scene::dep_fast); epochs stay below 2^31.
constexpr unsigned kCinHit = 0x80000000u;
__device__ __forceinline__ void cin_put(CinG* cin, int j, V3 c, unsigned tag, bool hit) {
  const unsigned tg = tag | (hit ? kCinHit : 0u);
  __hip_atomic_store(&cin[j].g[0], pack2(__float_as_uint(c.x), tg), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&cin[j].g[1], pack2(__float_as_uint(c.y), tg), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&cin[j].g[2], pack2(__float_as_uint(c.z), tg), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// A whole wave publishes the entries j0+lo .. j0+hi-1 (lanes lo..hi-1 of the wave's 64-entry
// slice) together: store instruction i writes granule 64*i + lane of the slice, so each
// instruction covers 512 contiguous bytes instead of 64 granules at a 24-byte stride (the
// agent-scope stores write through to memory: strided granules cost ~3x their bytes in HBM
// writes, rocprofv3 WRITE_SIZE).  Every granule is still one 8-byte atomic store with its own
// tag, so readers are unchanged.  The carry is either the wave's own per-lane value
// (cin_put_wave) or one carry for the whole range (cin_put_wave_uniform); hitmask bit e is
// entry lane e's hit flag.  Every lane of the wave must call these.
__device__ __forceinline__ void cin_put_granules(CinG* cin, int j0, int lo, int hi, V3 c_lane,
                                                 bool uniform, unsigned tag,
                                                 unsigned long long hitmask) {
  const int lane = threadIdx.x & 63;
  unsigned long long* g = &cin[j0].g[0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int q = 64 * i + lane;
    const int e = q / 3, comp = q - 3 * e;
    float x = c_lane.x, y = c_lane.y, z = c_lane.z;
    if (!uniform) {
      x = __shfl(x, e, 64);
      y = __shfl(y, e, 64);
      z = __shfl(z, e, 64);
    }
    const float v = comp == 0 ? x : (comp == 1 ? y : z);
    const unsigned tg = tag | (((hitmask >> e) & 1ull) ? kCinHit : 0u);
    if (e >= lo && e < hi)
      __hip_atomic_store(&g[q], pack2(__float_as_uint(v), tg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}
// Per-lane carries staged through the wave's own 768 bytes of LDS (entry-major x, y, z: float
// q of the stage is granule q's value) instead of cross-lane shuffles.
__device__ __forceinline__ void cin_put_wave(CinG* cin, int j0, int lo, int hi, V3 c_lane,
                                             unsigned tag, unsigned long long hitmask,
                                             float* stage) {
  const int lane = threadIdx.x & 63;
  stage[3 * lane] = c_lane.x;
  stage[3 * lane + 1] = c_lane.y;
  stage[3 * lane + 2] = c_lane.z;
  __builtin_amdgcn_wave_barrier();   // one wave's LDS accesses complete in order
  unsigned long long* g = &cin[j0].g[0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int q = 64 * i + lane;
    const int e = q / 3;
    const unsigned tg = tag | (((hitmask >> e) & 1ull) ? kCinHit : 0u);
    const float v = stage[q];
    if (e >= lo && e < hi)
      __hip_atomic_store(&g[q], pack2(__float_as_uint(v), tg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  __builtin_amdgcn_wave_barrier();   // the stage is rewritten by the next window
}
__device__ __forceinline__ void cin_put_wave_uniform(CinG* cin, int j0, int lo, int hi, V3 c,
                                                     unsigned tag, unsigned long long hitmask) {
  cin_put_granules(cin, j0, lo, hi, c, true, tag, hitmask);
}

__device__ __forceinline__ bool cin_get(CinG* cin, int j, unsigned tag, V3& c, bool& hit) {
  const unsigned long long a =
      __hip_atomic_load(&cin[j].g[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b =
      __hip_atomic_load(&cin[j].g[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long d =
      __hip_atomic_load(&cin[j].g[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  c = v3(__uint_as_float((unsigned)a), __uint_as_float((unsigned)b),
         __uint_as_float((unsigned)d));
  const unsigned ta = (unsigned)(a >> 32);
  hit = (ta & kCinHit) != 0u;
  return (ta & ~kCinHit) == tag && (unsigned)(b >> 32) == ta && (unsigned)(d >> 32) == ta;
}

// Resolver queue order: segments longest first (LPT), so the chains that take longest start
// at once instead of after the queue reaches them.  One block: a counting sort into 256
// length buckets of 32 entries (>= 8160 share the top bucket), stable within a bucket.
// Above kSegOrderMax segments the queue stays in segment order (counters[3] = 0).
// The order's first counters[14] segments have >= block_min entries (rounded up to the
// bucket width): k_resolve's workgroups take them from head A (counters[1]) while its waves
// start on the rest from head B (counters[15]).
__global__ void __launch_bounds__(kScanBlock) k_seg_order(const int* __restrict__ seg_start,
                                                     int* __restrict__ counters,
                                                     int* __restrict__ order,
                                                     int* __restrict__ batch_state,
                                                     int* __restrict__ batch_cnt,
                                                     int* __restrict__ batch_rq,
                                                     int block_min, int block_cap,
                                                     int zero_batches) {
  seg_order_body(seg_start, counters, order, batch_state, batch_cnt, batch_rq, block_min,
                 block_cap, zero_batches);
}

// Block-level window for the team's RESOLVE leader: the 4 waves of one block resolve up to
// 256 entries at the block-uniform carry c with the same LANE/COOP state machine as
// wave_window, at 4x the width — COOP steps take 4*E entries (E per wave) and LANE passes
// 256 — so clusters with short clean gaps cost one cooperative evaluation per changer.
// The window's records sit in LDS (`rec`, loaded by the caller); per-step results meet in
// double-buffered per-wave slots behind one barrier.  Entries are written to cin as they
// resolve.  Every thread of the block must call this.
struct BlockWinShared {
  DepRec rec[kResolveBlock];
  uint8_t hit[kResolveBlock];   // per entry: some level hit at the window's carry
  int wpos[2][4];
  float wout[2][4][3];
  // predictive steps (helper blocks): per group its output, hit flag and guess, double-
  // buffered by step parity like wpos / wout (one barrier per step)
  float pout[2][16][3];
  float pce[2][16][3];
  int phit[2][16];
};

// hp (helper blocks): carry predictor; the cooperative step then takes entry pos at c in
// group 0 and entry pos+1 at Eb-1 guessed carry-ins in the other groups (wave_window's
// predictive step with the whole block: 15 guesses instead of 3).
// stop (the team leader): instead of a LANE pass after K clean cooperative steps, return at
// once with the number of entries resolved so far (the team's cooperative SCAN takes the
// rest, k_resolve).  Returns -1 when the window was resolved to its end.
__device__ __forceinline__ int block_window(const Scene& sc, int maxrec, BlockWinShared& bw,
                                            int base, int nvalid, V3& c, const LaneShape& ls,
                                            int G, bool& dense, bool& changed, int K,
                                            CinG* __restrict__ cin, unsigned tag,
                                            WinStats& ws, CarryHist* hp = nullptr,
                                            bool stop = false) {
  int stopped = -1;
  constexpr int kNo = 0x7fffffff;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  changed = false;
  int zero = 0;
  int pos = 0;
  int par = 0;
  bool coop = dense && G > 0;
  int clean_run = 0;
  const bool spec = 2 * G <= 64;
  const int GE = G > 0 ? (spec ? 2 * G : G) : 64;
  const int E = 64 / GE;
  const int Eb = 4 * E;
  const int e = lane / GE, kself = G > 0 ? lane % G : 0, half = spec ? (lane / G) & 1 : 0;
#if RC_STAMPS
  unsigned long long top_ = 0;
#endif
  while (pos < nvalid) {
#if RC_STAMPS
    {
      const unsigned long long n_ = __builtin_amdgcn_s_memtime();
      if (top_) ws.cs += n_ - top_;
      top_ = n_;
    }
#endif
    int last;      // entries [pos, last] resolve with carry c
    V3 cn = c;
    bool hit;
    if (coop && hp && kPredict && hp->n >= 2 && pos + 1 < nvalid && Eb <= 16 && Eb >= 2) {
      ++ws.coop;
      const int gi = wave * E + e;
      // groups 1..k1 guess entry pos+1's carry-in; with RC_PRED_SPLIT the groups above k1 guess
      // entry pos+2's (twice the history's mean step: a hit retires three entries)
      const bool three = kPredSplit > 0 && kPredSplit < Eb - 1 && pos + 2 < nvalid;
      const int k1 = three ? kPredSplit : Eb - 1;
      const bool g2 = gi > k1;
      const int i = pos + (gi > 0 ? 1 : 0) + (g2 ? 1 : 0);
      const V3 ce = sel(gi > 0, hist_guess(*hp, c, g2 ? gi - k1 : gi, g2 ? 2 : 1), c);
      const DepRec ri = bw.rec[i < nvalid ? i : pos];
      V3 oc = ce;
      bool hg = false;
#if RC_STAMPS
      Stamps stp = {{0, 0, 0, 0}, 0};
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself, G, half, ri, maxrec, ce, zero, hg, &stp)
#else
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself, G, half, ri, maxrec, ce, zero, hg)
#endif
#define RC_SPEC(GT) \
  (sc.has_quadric ? (quad_x0(sc) ? RC_SPEC1(GT, 2) : RC_SPEC1(GT, 1)) : RC_SPEC1(GT, 0))
      if (G == 8) oc = RC_SPEC(8);
      else if (G == 4) oc = RC_SPEC(4);
      else if (G == 16) oc = RC_SPEC(16);
      else oc = RC_SPEC(0);
#undef RC_SPEC
#undef RC_SPEC1
#if RC_STAMPS
      ws.ce += __builtin_amdgcn_s_memtime() - top_;
#endif
      if ((lane % GE) == 0) {
        bw.pout[par][gi][0] = oc.x;
        bw.pout[par][gi][1] = oc.y;
        bw.pout[par][gi][2] = oc.z;
        bw.pce[par][gi][0] = ce.x;
        bw.pce[par][gi][1] = ce.y;
        bw.pce[par][gi][2] = ce.z;
        bw.phit[par][gi] = hg ? 1 : 0;
      }
      // one barrier per step: every wave finds the matching guess itself (the same ballot
      // over the same slots), and the slots are double-buffered by step parity — a wave
      // writes parity p again only after every wave has passed the barrier of the step
      // in between, i.e. has read these
#if RC_STAMPS
      const unsigned long long bw0_ = __builtin_amdgcn_s_memtime();
#endif
      __syncthreads();
#if RC_STAMPS
      ws.cw += __builtin_amdgcn_s_memtime() - bw0_;
#endif
      const V3 o0 = v3(bw.pout[par][0][0], bw.pout[par][0][1], bw.pout[par][0][2]);
      const V3 pl = v3(bw.pce[par][lane < Eb ? lane : 0][0], bw.pce[par][lane < Eb ? lane : 0][1],
                       bw.pce[par][lane < Eb ? lane : 0][2]);
      const bool mt = lane > 0 && lane <= k1 && same_bits(pl, o0);
      const unsigned long long mm = __ballot(mt);
      const int mi = mm ? __ffsll((long long)mm) - 1 : 0;
      if (t == pos) cin_put(cin, base + pos, c, tag, bw.phit[par][0] != 0);
      if (same_bits(o0, c)) {   // entry pos leaves the carry: the run is over
        hp->n = 0;
        pos += 1;
        if (++clean_run >= K) coop = false;
      } else {
        changed = true;
        ++ws.changers;
        clean_run = 0;
        hist_push(*hp, o0);
        if (mi > 0) {
          const V3 o1 = v3(bw.pout[par][mi][0], bw.pout[par][mi][1], bw.pout[par][mi][2]);
          if (t == pos + 1) cin_put(cin, base + pos + 1, o0, tag, bw.phit[par][mi] != 0);
          pos += 2;
          if (same_bits(o1, o0)) {
            hp->n = 0;
            c = o0;
          } else {
            ++ws.changers;
            hist_push(*hp, o1);
            c = o1;
            // entry pos+2 (now pos) evaluated at a guess equal to o1: its exact evaluation
            const unsigned long long m2 = three ? __ballot(lane > k1 && lane < Eb && same_bits(pl, o1)) : 0ull;
            if (m2) {
              const int mj = __ffsll((long long)m2) - 1;
              const V3 o2 = v3(bw.pout[par][mj][0], bw.pout[par][mj][1], bw.pout[par][mj][2]);
              if (t == pos) cin_put(cin, base + pos, o1, tag, bw.phit[par][mj] != 0);
              pos += 1;
              if (same_bits(o2, o1)) {
                hp->n = 0;
              } else {
                ++ws.changers;
                hist_push(*hp, o2);
                c = o2;
              }
            }
          }
        } else {
          c = o0;
          pos += 1;
        }
      }
      par ^= 1;
      continue;
    }
    if (!coop) {
      ++ws.lane;
      const bool act = t >= pos && t < nvalid;
      V3 o = c;
      bool h = false;
      if (act) o = carry_path(sc, bw.rec[t], maxrec, c, zero, h);
#if RC_STAMPS
      ws.ce += __builtin_amdgcn_s_memtime() - top_;
#endif
      bw.hit[t] = h ? 1 : 0;
      const unsigned long long m = __ballot(act && !same_bits(o, c));
      const int k = m ? __ffsll((long long)m) - 1 : -1;
      if (lane == 0) bw.wpos[par][wave] = k >= 0 ? wave * 64 + k : kNo;
      if (k >= 0 && lane == k) {
        bw.wout[par][wave][0] = o.x;
        bw.wout[par][wave][1] = o.y;
        bw.wout[par][wave][2] = o.z;
      }
    } else {
      ++ws.coop;
      const int i = pos + wave * E + e;
      const bool act = e < E && i < nvalid;
      const DepRec ri = bw.rec[i < nvalid ? i : pos];
      V3 oc = c;
      bool hg = false;
#if RC_STAMPS
      Stamps stq = {{0, 0, 0, 0}, 0};
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself, G, half, ri, maxrec, c, zero, hg, &stq)
#else
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself, G, half, ri, maxrec, c, zero, hg)
#endif
#define RC_SPEC(GT) \
  (sc.has_quadric ? (quad_x0(sc) ? RC_SPEC1(GT, 2) : RC_SPEC1(GT, 1)) : RC_SPEC1(GT, 0))
      if (act) {
        if (G == 8) oc = RC_SPEC(8);
        else if (G == 4) oc = RC_SPEC(4);
        else if (G == 16) oc = RC_SPEC(16);
        else if (spec) oc = RC_SPEC(0);
        else oc = carry_path_coop(sc, ls, kself, G, ri, maxrec, c, zero, hg);
      }
#undef RC_SPEC
#undef RC_SPEC1
#if RC_STAMPS
      ws.ce += __builtin_amdgcn_s_memtime() - top_;
#endif
      if (act && (lane % GE) == 0) bw.hit[i] = hg ? 1 : 0;
      const unsigned long long mc = __ballot(act && (lane % GE) == 0 && !same_bits(oc, c));
      const int g = mc ? (__ffsll((long long)mc) - 1) / GE : -1;
      if (lane == 0) bw.wpos[par][wave] = g >= 0 ? pos + wave * E + g : kNo;
      if (g >= 0 && lane == g * GE) {
        bw.wout[par][wave][0] = oc.x;
        bw.wout[par][wave][1] = oc.y;
        bw.wout[par][wave][2] = oc.z;
      }
    }
#if RC_STAMPS
    const unsigned long long bw1_ = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#if RC_STAMPS
    ws.cw += __builtin_amdgcn_s_memtime() - bw1_;
#endif
    int wb = 0;
    int best = bw.wpos[par][0];
    for (int q = 1; q < 4; ++q) {
      const int v = bw.wpos[par][q];
      if (v < best) {
        best = v;
        wb = q;
      }
    }
    hit = best != kNo;
    if (hit) {
      last = best;
      cn = v3(bw.wout[par][wb][0], bw.wout[par][wb][1], bw.wout[par][wb][2]);
    } else {
      last = coop ? (pos + Eb < nvalid ? pos + Eb : nvalid) - 1 : nvalid - 1;
    }
    {   // entries pos..last of this window read carry c: each wave publishes its 64-entry slice
      const int w0 = wave * 64;
      const int lo = pos - w0 > 0 ? pos - w0 : 0;
      const int hi = last + 1 - w0 < 64 ? last + 1 - w0 : 64;
      const unsigned long long hm = __ballot(bw.hit[t] != 0);
      if (lo < hi) cin_put_wave_uniform(cin, base + w0, lo, hi, c, tag, hm);
    }
    if (hp) {   // keep the predictor's history across the non-predictive steps
      if (!hit || last > pos) hp->n = 0;
      if (hit) {
        if (hp->n == 0) hist_push(*hp, c);
        hist_push(*hp, cn);
      }
    }
    pos = last + 1;
    c = cn;
    par ^= 1;
    if (hit) {
      changed = true;
      ++ws.changers;
      coop = G > 0;
      clean_run = 0;
    } else if (coop) {
      if (++clean_run >= K) {
        coop = false;
        if (stop) {   // the cluster is over: the team scans on from pos
          stopped = pos;
          break;
        }
      }
    }
  }
#if RC_STAMPS
  if (top_) ws.cs += __builtin_amdgcn_s_memtime() - top_;
#endif
  dense = coop;
  return stopped;
}

// Team hand-off by data-tagged 8-byte granules (MI355X_MICROARCH.md: granule hand-off, R2):
// each block publishes {first changer position, carry x, y, z} as four granules
// {payload:32, round:32} with agent-scope (sc1) stores; a reader spins on the granules
// themselves until every tag equals the round, so no counter, fence or drain sits on the
// path.  Slots rotate over kTeamBufs rounds.  A SCAN round is all-to-all (every block
// publishes, every block collects every slot), a RESOLVE round is one-to-all (block 0
// publishes, every block collects it), and RESOLVE rounds never follow each other.  So while
// a slow block still reads round r, the others can publish at most up to round r + 2: after
// a SCAN round r, a RESOLVE round r + 1 waits for nobody but block 0, and the SCAN round r + 2
// cannot be collected without the slow block's own publish.  With round parity (two buffers)
// a hand-off spun out its 5 s limit in 1 frame of ~200-300 with split shading, whose k_side
// work slows the team; rotating over four rounds brought that to ~1 in 5 000-14 000
// (profiles/r06o_team_slot_race.txt).  The residual failure is not an overwrite: every other
// block waits for block 0's RESOLVE round r while block 0's slot holds r and r + 1 when the
// frame ends (profiles/r06zz_split_shade_residual.txt; open, split shading only).
constexpr int kTeamBufs = 4;
struct alignas(32) TeamSlot {
  unsigned long long g[4];
};

// Dense-run hand-off (k_resolve helper blocks): a regular wave deep in a run of changers
// hands the rest of its segment (position, carry, predictor history) to a helper block — but
// only to one that is idle: a helper announces itself (idle += 1) before it claims the next
// item, and a wave hands off only after taking one such announcement (idle -= 1), so every
// item has a helper already waiting for it and nothing queues behind a busy helper (a queued
// run would sit on the critical path; quadric 8192^2 has more dense runs than helpers).  At
// most `helpers` items are outstanding, so item k lives in ring slot k % kDenseQ, tagged k+1.
constexpr int kDenseQ = kDenseSlots;   // ring slots (>= helpers, checked by the host)
constexpr int kHandMin = 256;    // entries left in the segment
struct DenseItem {
  int s, j, hn, ready;           // ready = item index + 1 once published
  float c[3];
  float h[4][3];
};
struct DenseQueue {
  int prod, claim, finished, idle;   // hand-offs, helper claims, regular-loop waves done,
  int pad[28];                       // idle helper announcements not yet taken
  DenseItem item[kDenseQ];
};
struct TeamState {
  // First bounded spin that timed out (first writer wins, rc_spin_error): code (1 team
  // granule, 2 phase-C carry-in, 3 helper queue), the workgroup and a site detail.  Once it is
  // set every other spin gives up at its next check instead of waiting out its own limit.
  int error;
  int err_block;
  int err_info;
  int err_info2;
  // phase C's ready queue (lone frames with k_side): batches pushed as they complete, taken
  // by k_side's waves in that order (ready_range, phase_c_ready)
  int rq_prod, rq_cons;
  int helpers_out;   // helper workgroups past their hand-off loop (resolver_phase_c, mode 2)
  // Frame diagnostics, latched with the error word after the frame (FrameLog::Entry): the
  // team's SCAN (LANE), cooperative SCAN and RESOLVE rounds, and per spin site (kSpin*) the
  // longest bounded wait of the frame in 10 ns ticks (waits under 10 us are not noted)
  int n_scan, n_cscan, n_resolve;
  int spin_ticks[4];
  // the shader clock over the resolver's own run (workgroup 0: s_memtime cycles per 10 ns tick
  // of s_memrealtime, in MHz): a throttled box shows here instead of as an unexplained slow step
  int clock_mhz;
  // long carry segments of the frame (the host's schedule hint for the next frame of the same
  // scene and size, FrameLog::Entry): bits 0..29 = 1 + the last row any long segment reaches
  // (0: none), bit 30 = a long segment was resolved outside a team (the early team's band 0
  // missed it)
  int team_row;
  int pad[16];
  TeamSlot slot[kTeamBufs][kTeamMax];
  DenseQueue dq;
#if RC_HANDOFF_DIAG   // experiment builds: when the first spin failed, when block 0 published
  unsigned long long hd_err_t;
  unsigned long long hd_pub_t[kTeamBufs];
  int hd_pub_round[kTeamBufs];
  int hd_pad[2];
#endif
};

static_assert(sizeof(TeamState) % 16 == 0, "k_row_stats clears TeamState in 16-byte words");
// the host's per-frame record (rc_runtime.h FrameLog::Entry) is TeamState's first 64 bytes
static_assert(offsetof(TeamState, n_scan) == 28 && offsetof(TeamState, spin_ticks) == 40 &&
                  offsetof(TeamState, clock_mhz) == 56 && offsetof(TeamState, team_row) == 60,
              "FrameLog::Entry layout");

// spin sites (TeamState::spin_ticks)
constexpr int kSpinTeam = 0, kSpinCarry = 1, kSpinQueue = 2, kSpinHelper = 3;
constexpr unsigned long long kSpinLimit = 500000000ull;   // 5 s of the 100 MHz clock
constexpr unsigned long long kSpinPoll = 100000ull;       // check the error word after 1 ms

__device__ __forceinline__ void set_error(TeamState* ts, int code, int info, int info2) {
  int expect = 0;
  if (__hip_atomic_compare_exchange_strong(&ts->error, &expect, code, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
#if RC_HANDOFF_DIAG
    __hip_atomic_store(&ts->hd_err_t, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    __hip_atomic_store(&ts->err_block, (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ts->err_info, info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ts->err_info2, info2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// A bounded spin of `site` that started at t0 is over: note its wait when it was long (a
// frame's record of what it waited on; one atomic per long wait only).
__device__ __forceinline__ void spin_note(TeamState* ts, int site, unsigned long long t0) {
  const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
  if (dt > 1000)
    __hip_atomic_fetch_max(&ts->spin_ticks[site], (int)(dt < 0x7fffffffull ? dt : 0x7fffffffull),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A spin that started at t0 gives up: its own limit passed, or (after 1 ms) another spin
// already failed.
__device__ __forceinline__ bool spin_expired(TeamState* ts, unsigned long long t0) {
  const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
  if (dt > kSpinLimit) return true;
  return dt > kSpinPoll &&
         __hip_atomic_load(&ts->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// Phase C's ready queue.  Entries [j0, j1) of the DEP list have their carry-ins published:
// credit them to their 64-entry batches; a batch whose every entry is credited is pushed to
// the queue, so k_side shades batches in the order they complete instead of waiting on them
// in index order (the team's segment holds the first 844k entries at quadric 4096^2 and
// resolves last: index order left 70 % of phase C for after the resolver).  Ranges credited
// by the resolver partition the DEP list, so every batch is pushed exactly once.  A batch
// lying wholly inside the range needs no count.  One wave; every lane calls it.
__device__ __forceinline__ void ready_range(int* __restrict__ cnt, int* __restrict__ rq,
                                            TeamState* ts, int ndep, int j0, int j1) {
  if (!cnt || j0 >= j1) return;
  const int lane = threadIdx.x & 63;
  const int b0 = j0 >> 6, b1 = (j1 - 1) >> 6;
  // [j0, j1) is contiguous: only its first and last batch can be partial, so at most two
  // credit atomics (lanes 0 and 1, in flight together) and one queue reservation for every
  // completed batch — a team SCAN round completes ~512 batches, which took eight dependent
  // reservations when they were made per 64 batches
  int r = 1;
  if (lane < 2 && (lane == 0 || b1 != b0)) {
    const int b = lane == 0 ? b0 : b1;
    const int lo = j0 > b * 64 ? j0 : b * 64;
    const int hi = j1 < b * 64 + 64 ? j1 : b * 64 + 64;
    const int size = (ndep < b * 64 + 64 ? ndep : b * 64 + 64) - b * 64;
    const int add = hi - lo;
    r = (add == size || atomicAdd(&cnt[b], add) + add == size) ? 1 : 0;
  }
  const bool d0 = __shfl(r, 0, 64) != 0;
  const bool d1 = b1 != b0 ? __shfl(r, 1, 64) != 0 : d0;
  const int first = d0 ? b0 : b0 + 1;
  const int last = b1 != b0 ? (d1 ? b1 : b1 - 1) : (d0 ? b0 : b0 - 1);
  const int n = last - first + 1;
  if (n <= 0) return;
  int k0 = 0;
  if (lane == 0) k0 = atomicAdd(&ts->rq_prod, n);
  k0 = __shfl(k0, 0, 64);
  for (int i = lane; i < n; i += 64)
    __hip_atomic_store(&rq[k0 + i], first + i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void team_publish(TeamState* ts, int round, unsigned pos, V3 c) {
  TeamSlot* sl = &ts->slot[round & (kTeamBufs - 1)][blockIdx.x];
#if RC_HANDOFF_DIAG
  if (blockIdx.x == 0) {
    __hip_atomic_store(&ts->hd_pub_t[round & (kTeamBufs - 1)],
                       (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ts->hd_pub_round[round & (kTeamBufs - 1)], round, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
#endif
  const unsigned tag = (unsigned)round;
  __hip_atomic_store(&sl->g[0], pack2(pos, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&sl->g[1], pack2(__float_as_uint(c.x), tag), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&sl->g[2], pack2(__float_as_uint(c.y), tag), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&sl->g[3], pack2(__float_as_uint(c.z), tag), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Spin until block b's round-`round` slot is complete; returns false on timeout.
__device__ __forceinline__ bool team_collect(TeamState* ts, int round, int b, unsigned& pos,
                                             V3& c) {
  TeamSlot* sl = &ts->slot[round & (kTeamBufs - 1)][b];
  const unsigned tag = (unsigned)round;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const unsigned long long g0 = __hip_atomic_load(&sl->g[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long g1 = __hip_atomic_load(&sl->g[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long g2 = __hip_atomic_load(&sl->g[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long g3 = __hip_atomic_load(&sl->g[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(g0 >> 32) == tag && (unsigned)(g1 >> 32) == tag &&
        (unsigned)(g2 >> 32) == tag && (unsigned)(g3 >> 32) == tag) {
      spin_note(ts, kSpinTeam, t0);
      pos = (unsigned)g0;
      c = v3(__uint_as_float((unsigned)g1), __uint_as_float((unsigned)g2),
             __uint_as_float((unsigned)g3));
      return true;
    }
    if (spin_expired(ts, t0)) {
      set_error(ts, 1, round, b);
      return false;
    }
  }
}

// ------------------------------------------------------------------ parity phase C --
// Colours and phase C beside the resolver.  k_classify leaves every colour to be shaded: the
// non-DEP pixels (8x8 tiles, always ready) and the DEP pixels with their resolved carry-ins,
// in batches of 64 consecutive DEP entries (one per lane).  k_side runs them on a second
// stream while the resolver runs, on the CUs the resolver's workgroups have left (its LDS
// reservation cannot fit beside one: side_lds_bytes; sharing the SIMDs slows the chains and,
// above all, the team's rounds): tiles first, then phase C pass 1 (batches whose carry-ins
// are already published — tagged granules, CinG) and pass 2 (everything not yet claimed,
// waiting for it).  k_finish, after the resolver on the main stream, claims what is left.
// A batch is shaded exactly once: its claim word goes 0 -> 1 by an agent-scope CAS; tiles
// are claimed from one counter.
constexpr int kSideBlock = 256;

__device__ __forceinline__ bool batch_claim(int* state, int b) {
  int expect = 0;
  return __hip_atomic_compare_exchange_strong(&state[b], &expect, 1, __ATOMIC_RELAXED,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Loads batch b's carry-ins; false if `wait` is false and one is not published yet.
__device__ __forceinline__ bool batch_carries(CinG* cin, int ndep, int b, unsigned tag,
                                              bool wait, V3& c, bool& hit, TeamState* ts) {
  const int j = b * 64 + (int)(threadIdx.x & 63);
  // Only the lanes whose carry-in is still missing poll again (a lane keeps a complete entry),
  // and the poll interval grows: while the resolver runs, phase C's waiting waves would
  // otherwise re-read whole batches of agent-scope granules every microsecond and load the
  // memory fabric the resolver's own hand-offs go through (lone frame: resolver 4.65 ms
  // beside the waiting side kernel vs 4.48 ms alone).
  // The limit measures a lack of progress: it restarts whenever another of the
  // batch's carry-ins arrives or another regular resolver wave finishes, so a legitimately
  // long resolver (huge frames, scenes whose shapes are not staged in LDS) is not cut off.
  bool ok = j >= ndep;
  unsigned long long t0 = 0;
  int seen = -1;
  const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
  for (int poll = 0;; ++poll) {
    if (!ok) ok = cin_get(cin, j, tag, c, hit);
    if (__all(ok)) {
      if (poll > 0 && (threadIdx.x & 63) == 0) spin_note(ts, kSpinCarry, w0);
      return true;
    }
    if (!wait) return false;
    const int progress =
        __popcll(__ballot(ok)) +
        __hip_atomic_load(&ts->dq.finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (progress != seen) {
      seen = progress;
      t0 = __builtin_amdgcn_s_memrealtime();
    } else if (spin_expired(ts, t0)) {
      // the first entry of the batch that is still missing
      const unsigned long long miss = __ballot(!ok);
      if ((threadIdx.x & 63) == 0) set_error(ts, 2, b * 64 + (__ffsll((long long)miss) - 1), ndep);
      return true;
    }
    if (poll < 4) __builtin_amdgcn_s_sleep(32);
    else __builtin_amdgcn_s_sleep(127);
  }
}

// Phase C of one batch of 64 DEP entries.  Under dep_fast phase A left each entry's primary
// shade in its DEP line (deprec[p].px..pz) and counted the events of its primary part: a
// clean entry (no level hit at its carry-in) is exactly that shade (every level's shade is
// zero, C/raycast.c:366-378), the others resume at level 2 (shade_dep_cont).  Otherwise the
// pixel is recomputed.
__device__ __forceinline__ void shade_batch(const Scene& sc, const Cam& cam, int W, int maxrec,
                                            const long long* __restrict__ dep_pix,
                                            const DepLine* __restrict__ deprec, int ndep, int b,
                                            V3 c, bool hit, uint8_t* __restrict__ out,
                                            uint32_t* __restrict__ patch, unsigned tag,
                                            int& zero) {
  const int j = b * 64 + (int)(threadIdx.x & 63);
  if (j >= ndep) return;
  const long long p = dep_pix[j];
  if (sc.dep_fast) {
    V3 rgb;
    if (hit) {
      rgb = shade_dep_cont(sc, deprec + p, maxrec, c, zero);
    } else {
      rgb = dep_pcol(deprec + p);
    }
    store_dep(out, patch, tag, p, j, rgb);
    return;
  }
  const int y = (int)(p / W), x = (int)(p % W);
  const V3 d = primary_dir(cam, x, y, zero);
  PixelOut po;
  shoot<kModeParityC>(sc, d, maxrec, c, po, zero);
  store_dep(out, patch, tag, p, j, po.rgb);
}

__device__ __forceinline__ int wave_ticket(int* ctr) {
  int b = 0;
  if ((threadIdx.x & 63) == 0) b = atomicAdd(ctr, 1);
  return __shfl(b, 0, 64);
}

// Shading of one 8x8 tile's non-DEP pixels (phase A's colour part, events counted).
__device__ __forceinline__ void shade_tile(const Scene& sc, const Cam& cam, int W, int H,
                                           int maxrec, int t, const uint8_t* __restrict__ cls,
                                           uint8_t* __restrict__ out, int& zero) {
  const int tw = (W + 7) >> 3;
  const int lane = threadIdx.x & 63;
  const int x = (t % tw) * 8 + (lane & 7), y = (t / tw) * 8 + (lane >> 3);
  if (x >= W || y >= H) return;
  const size_t p = (size_t)y * W + x;
  if (cls[p] == kClsDep) return;
  const V3 d = primary_dir(cam, x, y, zero);
  PixelOut po;
  shoot<kModeParityA>(sc, d, maxrec, v3(0.0f, 0.0f, 0.0f), po, zero);
  store_rgb(out + p * 3, po.rgb);
}

// Phase C pass 1 (published batches) and pass 2 (everything unclaimed, waiting).
__device__ __forceinline__ void phase_c_passes(const Scene& sc, const Cam& cam, int W,
                                               int maxrec, const long long* __restrict__ dep_pix,
                                               const DepLine* __restrict__ deprec,
                                               CinG* __restrict__ cin, int* __restrict__ counters,
                                               int* __restrict__ batch_state,
                                               uint8_t* __restrict__ out,
                                               uint32_t* __restrict__ patch, TeamState* ts,
                                               unsigned tag, bool pass1, int& zero) {
  int* done_ctr = &counters[pass1 ? 9 : 11];
  const int ndep = counters[2];
  const int nb = (ndep + 63) / 64;
  while (pass1) {
    const int b = wave_ticket(&counters[4]);
    if (b >= nb) break;
    // one granule first: the batch's last entry (most batches are still unpublished in this
    // pass; probing all 192 granules of each would put ~1.5 KB of agent-scope loads per batch
    // on the fabric the resolver's hand-offs use)
    {
      const int jl = (b * 64 + 63 < ndep ? b * 64 + 63 : ndep - 1);
      const unsigned long long g0 =
          __hip_atomic_load(&cin[jl].g[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (((unsigned)(g0 >> 32) & ~kCinHit) != tag) continue;
    }
    V3 c = v3(0.0f, 0.0f, 0.0f);
    bool hit = true;
    if (!batch_carries(cin, ndep, b, tag, false, c, hit, ts)) continue;
    int mine = 0;
    if ((threadIdx.x & 63) == 0) mine = batch_claim(batch_state, b);
    if (!__shfl(mine, 0, 64)) continue;
    shade_batch(sc, cam, W, maxrec, dep_pix, deprec, ndep, b, c, hit, out, patch, tag, zero);
    if ((threadIdx.x & 63) == 0) atomicAdd(done_ctr, 1);
  }
  for (;;) {
    const int b = wave_ticket(&counters[6]);
    if (b >= nb) break;
    int mine = 0;
    if ((threadIdx.x & 63) == 0) mine = batch_claim(batch_state, b);
    if (!__shfl(mine, 0, 64)) continue;
    V3 c = v3(0.0f, 0.0f, 0.0f);
    bool hit = true;
    (void)batch_carries(cin, ndep, b, tag, true, c, hit, ts);
    shade_batch(sc, cam, W, maxrec, dep_pix, deprec, ndep, b, c, hit, out, patch, tag, zero);
    if ((threadIdx.x & 63) == 0) atomicAdd(done_ctr, 1);
  }
}

// Phase C beside the resolver: batches in the order they complete (the resolver's ready
// queue, ready_range).  Item k of the queue exists once k batches have completed; every
// batch completes by the resolver's end, so a wave waiting for item k < nb is waiting for
// resolver progress (bounded: a lack of progress for 5 s, or an error raised elsewhere).
// k_finish takes whatever these waves have not claimed.
__device__ __forceinline__ void phase_c_ready(const Scene& sc, const Cam& cam, int W,
                                              int maxrec, const long long* __restrict__ dep_pix,
                                              const DepLine* __restrict__ deprec,
                                              CinG* __restrict__ cin, int* __restrict__ counters,
                                              int* __restrict__ batch_state,
                                              const int* __restrict__ rq, uint8_t* __restrict__ out,
                                              uint32_t* __restrict__ patch, TeamState* ts,
                                              unsigned tag, int& zero,
                                              unsigned* __restrict__ trace,
                                              int stop_waves = 0, int stop_helpers = 0) {
  const int ndep = counters[2];
  const int nb = (ndep + 63) / 64;
  unsigned* tq = trace ? trace + 3 * (size_t)ndep + 5 * (size_t)counters[0] + 200000 : nullptr;
  for (;;) {
    // stop_waves > 0 (phase C inside the resolver, mode 2): take no new item once the resolver's
    // own work is over (every regular wave and helper done); k_finish shades the rest at full
    // occupancy.  An item ticketed here is always shaded or left unclaimed for k_finish.
    if (stop_waves > 0) {
      int over = 0;
      if ((threadIdx.x & 63) == 0)
        over = __hip_atomic_load(&ts->dq.finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                   stop_waves &&
               __hip_atomic_load(&ts->helpers_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                   stop_helpers;
      if (__shfl(over, 0, 64)) break;
    }
    const int k = wave_ticket(&ts->rq_cons);
    if (k >= nb) break;
    if (tq && (threadIdx.x & 63) == 0) tq[3 * k] = (unsigned)__builtin_amdgcn_s_memrealtime();
    int b = -1;
    if ((threadIdx.x & 63) == 0) {
      unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      const unsigned long long w0 = t0;
      int seen = -1;
      for (;;) {
        const int v = __hip_atomic_load(&rq[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v) {
          b = v - 1;
          spin_note(ts, kSpinQueue, w0);
          break;
        }
        const int prod = __hip_atomic_load(&ts->rq_prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prod != seen) {
          seen = prod;
          t0 = __builtin_amdgcn_s_memrealtime();
        } else if (spin_expired(ts, t0)) {   // the batch's carries are k_finish's to wait for
          break;
        }
        __builtin_amdgcn_s_sleep(32);
      }
    }
    b = __shfl(b, 0, 64);
    if (b < 0) break;
    int mine = 0;
    if ((threadIdx.x & 63) == 0) mine = batch_claim(batch_state, b);
    if (!__shfl(mine, 0, 64)) continue;
    V3 c = v3(0.0f, 0.0f, 0.0f);
    bool hit = true;
    if (tq && (threadIdx.x & 63) == 0) tq[3 * k + 1] = (unsigned)__builtin_amdgcn_s_memrealtime();
    (void)batch_carries(cin, ndep, b, tag, true, c, hit, ts);   // published: arrives at once
    shade_batch(sc, cam, W, maxrec, dep_pix, deprec, ndep, b, c, hit, out, patch, tag, zero);
    if ((threadIdx.x & 63) == 0) atomicAdd(&counters[9], 1);
    if (tq && (threadIdx.x & 63) == 0) tq[3 * k + 2] = (unsigned)__builtin_amdgcn_s_memrealtime();
  }
}

// Phase C inside the resolver (rc_tuning.side 3): a resolver wave whose own work is done (no
// segment left to take, no hand-off left for a helper) shades batches from the ready queue
// instead of leaving its SIMD idle; k_finish, after the resolver, finds the queue drained.
__device__ __forceinline__ void resolver_phase_c(const Scene& sc, const Cam& cam, int W, int maxrec,
                                              const long long* __restrict__ dep_pix,
                                              const DepLine* __restrict__ deprec,
                                              CinG* __restrict__ cin, int* __restrict__ counters,
                                              int* __restrict__ batch_state,
                                              const int* __restrict__ rq,
                                              uint8_t* __restrict__ out,
                                              uint32_t* __restrict__ patch,
                                              unsigned long long* __restrict__ zcount,
                                              TeamState* ts, unsigned tag, int mode,
                                              int helpers) {
  int zero = 0;
  const int waves = ((int)gridDim.x - helpers) * (kResolveBlock / 64);
  phase_c_ready(sc, cam, W, maxrec, dep_pix, deprec, cin, counters, batch_state, rq, out,
                patch, ts, tag, zero, nullptr, mode == 2 ? waves : 0, helpers);
  flush_events(zero, zcount);
}

// amdgpu_waves_per_eu(2): a pipeline lane places two resolver workgroups per CU (one wave per
// SIMD each), so the kernel must stay within 256 registers (VGPRs + AGPRs) per wave
template <bool kLds>
__global__ void __launch_bounds__(kResolveBlock) __attribute__((amdgpu_waves_per_eu(2))) k_resolve(
    Scene sc, int maxrec, const DepLine* __restrict__ deprec,
    const long long* __restrict__ dep_pix, const long long* __restrict__ seg_key,
    const float4* __restrict__ wcarry,
    const int* __restrict__ seg_start, const int* __restrict__ seg_order,
    int* __restrict__ counters, int* __restrict__ head,
    CinG* __restrict__ cin, int team_blocks, int long_len, TeamState* __restrict__ ts,
    unsigned* __restrict__ trace, int G, int wave_k, int resolve_k, int resolve_clean,
    int team_cscan, unsigned tag,
    int helpers, int hand_run, int inject, int block_min, int headb_first,
    int* __restrict__ rq_cnt,
    int* __restrict__ rq, Cam cam, int W, uint8_t* __restrict__ out, uint32_t* __restrict__ patch,
    unsigned long long* __restrict__ zcount, int* __restrict__ batch_state, int inres) {
  if (!RC_X0_RESOLVE) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  // the product build has no trace: its timestamps and counters then hold no registers
  if (!RC_DIAG) trace = nullptr;
  const unsigned long long clk_t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long clk_c0 = __builtin_amdgcn_s_memtime();
  // census for phase C's side kernel: it only proceeds once every resolver block is resident
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(&counters[5], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // test aid (rc_debug_inject_error): this frame's hand-off fails as a timed-out spin would
  // (first writer wins; every spin of the frame then gives up at its next check)
  if (inject && blockIdx.x == 0 && threadIdx.x == 0) set_error(ts, 4, 0, 0);
  const int nseg = counters[0];
  const int ndep = counters[2];
  const bool ordered = counters[3] != 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // The chain steps read the winner's record (hit_frame) and refl[obj] every bounce level:
  // stage the shape records (n <= kLdsShapes) in LDS so those reads cost an LDS access
  // instead of a vector-memory round trip.
  __shared__ rc_shape s_shapes[kLds ? kLdsShapes + 1 : 1];
  if (kLds) {   // host guarantees n <= kLdsShapes
    const int words = (int)(sizeof(rc_shape) / 4) * (sc.n + 1);
    for (int i = threadIdx.x; i < words; i += blockDim.x)
      ((unsigned*)s_shapes)[i] = ((const unsigned*)sc.shapes)[i];
    __syncthreads();
    // the divergent reads (the winner's record) go to the LDS copy; the wave-uniform shape
    // loops of the LANE evaluator keep the global records, which the compiler reads with
    // scalar loads into SGPRs (an LDS copy there costs a vector LDS round trip per field)
    if (!RC_RES_GLOBAL_SCAN) sc.shapes = s_shapes;
    sc.lshapes = s_shapes;
  }
#if RC_STAMPS
  Stamps stp = {{0, 0, 0, 0}, 0};
#endif
  LaneShape ls;
  ls.has = false;
  if (G > 0) {
    const int kself = lane % G;
    ls.has = kself < sc.n;
    if (ls.has) ls.s = sc.shapes[kself];
  }

  __shared__ BlockWinShared s_bw;   // the team leader's and the helpers' block windows
  if ((int)blockIdx.x < team_blocks) {
    // ------------------------------------------------------------------- team --
    // Changers inside long segments come in dense clusters separated by long clean runs
    // (4096^2 quadric: median gap 3 entries, but two runs of 707k and 112k).  The team
    // alternates two modes:
    //   SCAN     every team wave evaluates 64 entries, one per lane, at the current carry
    //            (a T*256-entry window per round); the team agrees on the first changer
    //            through tagged granules;
    //   RESOLVE  the leader wave (block 0, wave 0) resolves the cluster that starts there on
    //            its own (wave_window: per-lane pass + cooperative inner loop, no team sync)
    //            until a whole 64-entry window comes back clean, then hands (position, carry)
    //            back to the team.
    __shared__ int s_pos[4];
    __shared__ float s_o[4][3];
    __shared__ int s_gpos;
    __shared__ int s_cflag;
    __shared__ float s_nc[3];
    const int T = team_blocks;
    const int window = T * 4 * 64;
    // cooperative SCAN rounds (team_cscan): E entries per wave, 2G lanes each
    const int cGE = (G > 0 && 2 * G <= 64) ? 2 * G : 64;
    const int cE = 64 / cGE;
    const bool cscan_on = RC_TEAM_CSCAN && team_cscan && G > 0 && 2 * G <= 64;
    int round = 0;
    auto credit = [&](int j0, int j1) {   // the crediter wave (all its lanes)
      ready_range(rq_cnt, rq, ts, ndep, j0, j1);
    };
    // the long segments lead the length-ordered queue (k_seg_order): stop at the first
    // shorter one instead of walking the whole segment table with dependent loads (0.4 ms at
    // quadric 4096^2, 2 076 segments, after the team's one segment was done)
    for (int q = 0; q < nseg; ++q) {
      const int s = ordered ? seg_order[q] : q;
      const int start = seg_start[s];
      const int end = (s + 1 < nseg) ? seg_start[s + 1] : ndep;
      if (end - start < long_len) {
        // below the floor of long_len's length bucket (k_seg_order: 32-entry buckets, the
        // top one holds every length >= 8160 unsorted): no long segment follows
        if (ordered && (end - start) < (min(long_len >> 5, 255) << 5)) break;
        continue;
      }
      const unsigned long long t_seg = __builtin_amdgcn_s_memrealtime();
      const unsigned long long c_seg = __builtin_amdgcn_s_memtime();
      int rounds_here = 0;
      V3 c = seg_init_carry(seg_key, wcarry, s);
      int j = start;
      bool resolve = false;
      int n_scan_ = 0, n_cscan_ = 0, n_resolve_ = 0;   // this segment's rounds by kind
      // the next SCAN round is cooperative (after a RESOLVE round that handed back early)
      bool cscan = false;
      // SCAN width: sub-windows of `window` entries per round, doubled after every clean
      // round up to 4 (a clean stretch then costs one hand-off per 4 windows), back to 1 after
      // a changer; the same on every team block (it follows the agreed positions)
      int width = 1;
      // the previous round's entries, credited to phase C's ready queue by the team's last
      // block while it waits for the next round's hand-off (its latency then overlaps the
      // wait instead of delaying the block's own round)
      int pend0 = 0, pend1 = 0;
      const bool crediter = (int)blockIdx.x == T - 1 && wave == 0;
      while (j < end) {
        ++round;
        ++rounds_here;
        const unsigned long long c_round = __builtin_amdgcn_s_memtime();
        const int j_round = j;
        WinStats tws = {0, 0, 0};
        const bool was_resolve = resolve;
        const bool coop_scan = RC_TEAM_CSCAN && !resolve && cscan;
        n_resolve_ += resolve ? 1 : 0;
        n_cscan_ += coop_scan ? 1 : 0;
        n_scan_ += (!resolve && !coop_scan) ? 1 : 0;
        if (!resolve) {
          // ---------------------------------------------------------------- SCAN
          // LANE: sub-window q: entries j + q*window + (block*4 + wave)*64 + lane; a wave stops
          // at its first changer (everything after it in scan order is after it in the window).
          // COOP (right after a RESOLVE round, whose cluster may go on a few entries later):
          // one cooperative step of every team wave, E entries each at a cooperative
          // evaluation's latency — T*4*E entries (2 048 at G = 8) in ~1/4 of a LANE round.
          const int slice = ((int)blockIdx.x * 4 + wave) * 64;
          unsigned long long hmq[4] = {0, 0, 0, 0};
          int wpos = 0x7fffffff;
          V3 wo = c;
          const int ci = j + ((int)blockIdx.x * 4 + wave) * cE + lane / cGE;   // COOP: entry
          bool chit = false;   // COOP: the lane's entry hit some level (its group leader's flag)
          if (coop_scan) {
            const bool act = lane / cGE < cE && ci < end;
            DepRec ri;
            if (act) ri = rec_at(deprec, dep_pix, ci);
            V3 oc = c;
            bool hg = false;
            int zero = 0;
#if RC_STAMPS
            Stamps sts = {{0, 0, 0, 0}, 0};
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself_, G, half_, ri, maxrec, c, zero, hg, &sts)
#else
#define RC_SPEC1(GT, Q) carry_path_spec<GT, Q>(sc, ls, kself_, G, half_, ri, maxrec, c, zero, hg)
#endif
#define RC_SPEC(GT) \
  (sc.has_quadric ? (quad_x0(sc) ? RC_SPEC1(GT, 2) : RC_SPEC1(GT, 1)) : RC_SPEC1(GT, 0))
            const int kself_ = lane % G, half_ = (lane / G) & 1;
            if (act) {
              if (G == 8) oc = RC_SPEC(8);
              else if (G == 4) oc = RC_SPEC(4);
              else if (G == 16) oc = RC_SPEC(16);
              else oc = RC_SPEC(0);
            }
#undef RC_SPEC
#undef RC_SPEC1
            chit = hg;
            const unsigned long long m = __ballot(act && (lane % cGE) == 0 && !same_bits(oc, c));
            if (m) {
              const int gl = __ffsll((long long)m) - 1;
              wpos = j + ((int)blockIdx.x * 4 + wave) * cE + gl / cGE;
              wo = v3(__shfl(oc.x, gl, 64), __shfl(oc.y, gl, 64), __shfl(oc.z, gl, 64));
            }
          } else {
          // one record ahead (two live, not four: the lanes' two resolver workgroups per CU
          // need the kernel within 256 registers)
          DepRec cur;
          if (j + slice + lane < end) cur = rec_at(deprec, dep_pix, j + slice + lane);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < width && wpos == 0x7fffffff) {
              const int base = j + q * window + slice;
              const bool valid = base + lane < end;
              DepRec nx;
              const int nidx = base + window + lane;
              if (q + 1 < width && nidx < end) nx = rec_at(deprec, dep_pix, nidx);
              V3 o = c;
              bool h = false;
              if (valid) {
                int zero = 0;
                o = carry_path(sc, cur, maxrec, c, zero, h);
              }
              cur = nx;
              hmq[q] = __ballot(valid && h);
              const unsigned long long m = __ballot(valid && !same_bits(o, c));
              if (m) {
                const int k = __ffsll((long long)m) - 1;
                wpos = base + k;
                wo = v3(__shfl(o.x, k, 64), __shfl(o.y, k, 64), __shfl(o.z, k, 64));
              }
            }
          }
          }
          if (lane == 0) {
            s_pos[wave] = wpos;
            s_o[wave][0] = wo.x;
            s_o[wave][1] = wo.y;
            s_o[wave][2] = wo.z;
          }
          __syncthreads();
          if (threadIdx.x == 0) {
            int w = 0;
            for (int q = 1; q < 4; ++q)
              if (s_pos[q] < s_pos[w]) w = q;
            const bool hit = s_pos[w] != 0x7fffffff;
            team_publish(ts, round, (unsigned)s_pos[w],
                         hit ? v3(s_o[w][0], s_o[w][1], s_o[w][2]) : v3(0.0f, 0.0f, 0.0f));
          }
          if (crediter) {
            credit(pend0, pend1);
            pend0 = pend1 = 0;
          }
          // every thread t < T collects slot t; block-wide minimum position
          unsigned upos = 0x7fffffffu;
          V3 oc = v3(0.0f, 0.0f, 0.0f);
          bool ok = true;
          if ((int)threadIdx.x < T) ok = team_collect(ts, round, threadIdx.x, upos, oc);
          if (__syncthreads_or(!ok)) return;
          const int pos = (int)upos;
          int mp = pos;
          for (int off = 32; off > 0; off >>= 1) {
            const int u = __shfl_xor(mp, off, 64);
            mp = u < mp ? u : mp;
          }
          if (lane == 0) s_pos[wave] = mp;
          __syncthreads();
          const int gmin = min(min(s_pos[0], s_pos[1]), min(s_pos[2], s_pos[3]));
          if (threadIdx.x == 0) s_gpos = gmin;
          if (gmin != 0x7fffffff && pos == gmin && (int)threadIdx.x < T) {
            s_nc[0] = oc.x;
            s_nc[1] = oc.y;
            s_nc[2] = oc.z;
          }
          __syncthreads();
          const int gpos = s_gpos;
          // entries before the first changer, and the changer itself, read carry c (gpos =
          // 0x7fffffff: every entry of the round); a wave that stopped early has no entry
          // at or before gpos in its later sub-windows
          if (coop_scan) {
            if (ci < end && lane / cGE < cE && (lane % cGE) == 0 && ci <= gpos)
              cin_put(cin, ci, c, tag, chit);
          } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (q < width) {
              const int base = j + q * window + slice;
              const long long hi0 = end - base < 64 ? end - base : 64;
              const long long hi1 = (long long)gpos - base + 1;
              const int hi = (int)(hi1 < hi0 ? hi1 : hi0);
              if (hi > 0) cin_put_wave_uniform(cin, base, 0, hi, c, tag, hmq[q]);
            }
          }
          }
          if (gpos == 0x7fffffff) {
            if (coop_scan) {
              j += T * 4 * cE;   // no change nearby: LANE rounds from here
              width = 1;
            } else {
              j += width * window;
              width = width < 4 ? 2 * width : 4;
            }
            cscan = false;
          } else {
            j = gpos + 1;
            c = v3(s_nc[0], s_nc[1], s_nc[2]);
            resolve = true;
            width = 1;
          }
          __syncthreads();
        } else {
          // ------------------------------------------------------------- RESOLVE
          if (blockIdx.x == 0) {
            bool dense = true;   // the cluster starts right after a changer
            int clean = 0;       // clean windows in a row (resolve_clean of them end the round)
            // records of the first window; later windows are prefetched one ahead
            const int t = threadIdx.x;
            if (j + t < end) s_bw.rec[t] = rec_at(deprec, dep_pix, j + t);
            __syncthreads();
            while (j < end) {
              const int nv = end - j < kResolveBlock ? end - j : kResolveBlock;
              DepRec nxt;
              const int jn = j + nv;
              if (jn + t < end) nxt = rec_at(deprec, dep_pix, jn + t);
              bool changed;
              const int stop = block_window(sc, maxrec, s_bw, j, nv, c, ls, G, dense, changed,
                                            resolve_k, cin, tag, tws, nullptr, cscan_on);
              if (stop >= 0) {   // resolve_k clean cooperative steps: the team scans on
                j += stop;
                cscan = true;
                __syncthreads();
                break;
              }
              j = jn;
              __syncthreads();   // everyone is done reading this window's records
              // resolve_clean clean windows in a row: the cluster is over (the next one is
              // the team's to find; a short gap costs a LANE pass here instead of a SCAN round
              // and two hand-offs)
              clean = changed ? 0 : clean + 1;
              if (clean >= resolve_clean) break;
              if (j + t < end) s_bw.rec[t] = nxt;
              __syncthreads();
            }
            // bit 31: the next SCAN round is cooperative (the round ended early)
            if (threadIdx.x == 0)
              team_publish(ts, round, (unsigned)j | (cscan ? 0x80000000u : 0u), c);
          }
          if (crediter && T > 1) {
            credit(pend0, pend1);
            pend0 = pend1 = 0;
          }
          if (threadIdx.x == 0) {
            unsigned upos = 0;
            V3 oc;
            const bool ok = team_collect(ts, round, 0, upos, oc);
            s_gpos = ok ? (int)(upos & 0x7fffffffu) : -1;
            s_cflag = (int)(upos >> 31);
            s_nc[0] = oc.x;
            s_nc[1] = oc.y;
            s_nc[2] = oc.z;
          }
          __syncthreads();
          if (s_gpos < 0) return;
          j = s_gpos;
          c = v3(s_nc[0], s_nc[1], s_nc[2]);
          resolve = false;
          cscan = s_cflag != 0;
          __syncthreads();
        }
        // the round's entries [j_round, j) are published: credited during the next round's
        // wait (pend), or below when the segment ends
        if (crediter) {
          pend0 = j_round;
          pend1 = j < end ? j : end;
        }
        // debug trace: per-round team log after the per-segment records and stamps
        if (trace && blockIdx.x == 0 && wave == 0 && lane == 0 && round < 8192) {
          unsigned* tl = trace + 3 * (size_t)ndep + 4 * (size_t)nseg + 8 * (size_t)round;
          tl[0] = was_resolve ? 1u : (coop_scan ? 2u : 0u);
          tl[1] = (unsigned)j_round;
          tl[2] = (unsigned)j;
          tl[3] = (unsigned)(__builtin_amdgcn_s_memtime() - c_round);
          tl[4] = (unsigned)tws.lane;
          tl[5] = (unsigned)tws.coop;
          tl[6] = (unsigned)tws.changers;
          tl[7] = 0xA5A5A5A5u;
#if RC_STAMPS   // eval / step cycles of the round's block windows
          unsigned* te = trace + 3 * (size_t)ndep + 5 * (size_t)nseg + 8 * 8192 + 4096;
          te[2 * round] = (unsigned)tws.ce;
          te[2 * round + 1] = (unsigned)tws.cs;
          te[16384 + 8 * 64 + round] = (unsigned)tws.cw;
#endif
        }
      }
      if (crediter) credit(pend0, pend1);   // the last round's
      if (blockIdx.x == 0 && threadIdx.x == 0) {   // the frame's record (FrameLog)
        ts->n_scan += n_scan_;
        ts->n_cscan += n_cscan_;
        ts->n_resolve += n_resolve_;
        // diagnostic: the last row a long segment reaches (FrameLog)
        atomicMax(&ts->team_row, (int)(dep_pix[end - 1] / W) + 1);
      }
      if (trace && blockIdx.x == 0 && threadIdx.x == 0) {
        trace[3 * s] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t_seg);
        trace[3 * s + 1] = (unsigned)rounds_here | 0x80000000u;
        trace[3 * s + 2] = (unsigned)(__builtin_amdgcn_s_memtime() - c_seg);
        trace[3 * (size_t)ndep + 4 * (size_t)nseg + 8 * 8192 + s] = (unsigned)t_seg;
      }
    }
    // the team's segments are done: its waves join the regular queue (every wave from here
    // on is independent; a frame without long segments gets the whole grid)
  }

  // ------------------------------------------------------------- helper blocks --
  // Blocks [team_blocks, team_blocks + helpers) take the runs regular waves hand off (below)
  // and resolve the rest of each such segment with block windows and 15 carry guesses per
  // step.  They leave once every regular-loop wave is done and no hand-off is pending.
  if ((int)blockIdx.x >= team_blocks && (int)blockIdx.x < team_blocks + helpers) {
    __shared__ int s_item;
    __shared__ DenseItem s_it;
    const int total = ((int)gridDim.x - helpers) * (kResolveBlock / 64);
    const int t = threadIdx.x;
    for (;;) {
      if (t == 0) {
        __hip_atomic_fetch_add(&ts->dq.idle, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int k = atomicAdd(&ts->dq.claim, 1);
        DenseItem& slot = ts->dq.item[k % kDenseQ];
        int got = -1;
        // the limit measures a lack of progress: it restarts whenever a regular wave
        // finishes or hands a run off
        unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long w0 = t0;
        int seen = -1;
        for (;;) {
          if (__hip_atomic_load(&slot.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == k + 1) {
            got = k;
            spin_note(ts, kSpinHelper, w0);
            break;
          }
          // Acquire on `finished` (released by each wave after its last possible hand-off)
          // makes every item those waves produced visible: only then does prod <= k prove
          // that item k never comes.
          const int fin =
              __hip_atomic_load(&ts->dq.finished, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
          const int prod = __hip_atomic_load(&ts->dq.prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (fin >= total && prod <= k) break;   // every regular wave is done, no item k
          if (fin + prod != seen) {
            seen = fin + prod;
            t0 = __builtin_amdgcn_s_memrealtime();
          } else if (spin_expired(ts, t0)) {
            set_error(ts, 3, k, fin);
            break;
          }
          __builtin_amdgcn_s_sleep(8);
        }
        s_item = got;
        if (got >= 0) s_it = slot;   // after the acquire on `ready`
      }
      __syncthreads();
      const int k = s_item;
      if (k < 0) break;
      const DenseItem& it = s_it;
      const int sg = it.s;
      int j = it.j;
      V3 c = v3(it.c[0], it.c[1], it.c[2]);
      CarryHist hs;
      hs.n = it.hn;
      hs.run = hand_run;
      for (int q = 0; q < 4; ++q) hs.h[q] = v3(it.h[q][0], it.h[q][1], it.h[q][2]);
      const int end = (sg + 1 < nseg) ? seg_start[sg + 1] : ndep;
      bool dense = true;
      WinStats hws = {0, 0, 0};
      const int j_item = j;
      const unsigned long long t_item = __builtin_amdgcn_s_memrealtime();
      if (j + t < end) s_bw.rec[t] = rec_at(deprec, dep_pix, j + t);
      __syncthreads();
      while (j < end) {
        const int nv = end - j < kResolveBlock ? end - j : kResolveBlock;
        DepRec nxt;
        const int jn = j + nv;
        if (jn + t < end) nxt = rec_at(deprec, dep_pix, jn + t);
        bool changed;
        block_window(sc, maxrec, s_bw, j, nv, c, ls, G, dense, changed, resolve_k, cin, tag,
                     hws, &hs);
        j = jn;
        __syncthreads();   // everyone is done reading this window's records
        if (j + t < end) s_bw.rec[t] = nxt;
        __syncthreads();
      }
      if (wave == 0) ready_range(rq_cnt, rq, ts, ndep, j_item, end);
      if (trace && t == 0 && k < 64) {   // debug trace: the helper's items
        unsigned* ti = trace + 3 * (size_t)ndep + 5 * (size_t)nseg + 8 * 8192 + 4096 + 16384 + 8 * k;
        ti[0] = (unsigned)sg;
        ti[1] = (unsigned)(end - j_item);
        ti[2] = (unsigned)t_item;
        ti[3] = (unsigned)__builtin_amdgcn_s_memrealtime();
        ti[4] = (unsigned)hws.coop;
        ti[5] = (unsigned)hws.changers;
#if RC_STAMPS
        ti[6] = (unsigned)hws.ce;
        ti[7] = (unsigned)hws.cs;
        ti[1] = (unsigned)hws.cw;   // (the item's length is in the segment table)
#endif
      }
    }
    if (trace && lane == 0)   // debug trace: when each wave leaves
      trace[3 * (size_t)ndep + 5 * (size_t)nseg + 8 * 8192 + blockIdx.x * 4 + wave] =
          (unsigned)__builtin_amdgcn_s_memrealtime();
    if (inres) {
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(&ts->helpers_out, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      resolver_phase_c(sc, cam, W, maxrec, dep_pix, deprec, cin, counters, batch_state,
                       rq, out, patch, zcount, ts, tag, inres, helpers);
    }
    return;   // helpers take no regular segments
  }

  // ------------------------------------------------------- long regular segments --
  // Segments of >= block_min entries (the queue is longest first) are resolved by a whole
  // workgroup: block_window's cooperative steps take 4*E entries (16 at G = 8) where one wave
  // takes E, so a changer costs about one evaluation where a lone wave spends LANE passes
  // (~26k cycles each) looking for the next one.  Lone quadric 4096^2: the 3856-entry segments
  // took 4.3 ms on one wave (157 LANE passes and 505 cooperative steps for 377 changers).
  // Once the queue reaches a shorter segment, the block's wave 0 takes that one and every
  // wave goes on as a regular wave.
  // The queue's first nlong segments (k_seg_order) are taken from head A by workgroups; the
  // waves start at once on the rest (head B), so shorter segments that turn out dense are not
  // held back behind the long ones, and take what is left of head A at the end.
  const int nlong = counters[14];
  int* headb = counters + 15;
  // the first headb_first regular workgroups leave head A to the others and start on head B at
  // once: its front holds the shorter segments that can turn out to be dense runs (every entry
  // a changer), which a helper then takes after hand_run changes
  if (nlong > 0 && (int)blockIdx.x >= team_blocks + helpers + headb_first) {
    __shared__ int s_seg;
    const int t = threadIdx.x;
    for (;;) {
      if (t == 0) s_seg = atomicAdd(head, 1);
      __syncthreads();
      const int q = s_seg;
      __syncthreads();   // s_seg is rewritten by the next dequeue
      if (q >= nlong) break;
      const int sg = ordered ? seg_order[q] : q;
      const int start = seg_start[sg];
      const int end = (sg + 1 < nseg) ? seg_start[sg + 1] : ndep;
      if (end - start >= long_len && team_blocks > 0) continue;   // the team's
      const unsigned long long t_seg = __builtin_amdgcn_s_memrealtime();
      const unsigned long long c_seg = __builtin_amdgcn_s_memtime();
      V3 c = seg_init_carry(seg_key, wcarry, sg);
      bool dense = false;
      WinStats bws = {0, 0, 0};
      int j = start;
      if (j + t < end) s_bw.rec[t] = rec_at(deprec, dep_pix, j + t);
      __syncthreads();
      while (j < end) {
        const int nv = end - j < kResolveBlock ? end - j : kResolveBlock;
        DepRec nxt;
        const int jn = j + nv;
        if (jn + t < end) nxt = rec_at(deprec, dep_pix, jn + t);
        bool changed;
        // no carry predictor here: its steps take two entries, and a clean entry after a
        // change ends the cooperative mode (measured: 191 LANE passes on a 3856-entry segment)
        block_window(sc, maxrec, s_bw, j, nv, c, ls, G, dense, changed, wave_k, cin, tag,
                     bws, nullptr);
        j = jn;
        __syncthreads();   // everyone is done reading this window's records
        if (j + t < end) s_bw.rec[t] = nxt;
        __syncthreads();
      }
      if (wave == 0) ready_range(rq_cnt, rq, ts, ndep, start, end);
      if (trace && t == 0) {
        trace[3 * sg] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t_seg);
#if RC_STAMPS   // LANE passes << 16 | cooperative steps (block windows)
        trace[3 * sg + 1] = ((unsigned)bws.lane << 16) | ((unsigned)bws.coop & 0xffffu);
#else
        trace[3 * sg + 1] = (unsigned)(bws.lane + bws.coop);
#endif
        trace[3 * sg + 2] = (unsigned)(__builtin_amdgcn_s_memtime() - c_seg);
        trace[3 * (size_t)ndep + 4 * (size_t)nseg + 8 * 8192 + sg] = (unsigned)t_seg;
      }
    }
  }

  // ------------------------------------------------------------- regular waves --
  // A regular workgroup's waves take their first segments together: four consecutive ones
  // of the length-ordered queue.  The longest segments then sit in a few workgroups (lone
  // quadric 4096^2: ~100 segments of 2.5-4.2 ms land on ~25 workgroups instead of one wave in
  // each of ~100), and the others vacate their CUs as soon as the short segments are gone —
  // k_side shades phase C on vacated CUs only.
  __shared__ int s_first;
  int first = -1;
  if ((int)blockIdx.x >= team_blocks + helpers) {
    if (threadIdx.x == 0) s_first = atomicAdd(headb, kResolveBlock / 64);
    __syncthreads();
    first = s_first + wave;
  }
  for (;;) {
    int s = 0;
    if (lane == 0) {
      if (first >= 0 && first < nseg) {
        s = first;
      } else {
        s = atomicAdd(headb, 1);
        if (s >= nseg) {   // head B is done: any long segment no workgroup has taken yet
          s = atomicAdd(head, 1);
          if (s >= nlong) s = nseg;
        }
      }
    }
    first = -1;
    s = __shfl(s, 0, 64);
    if (s >= nseg) break;
    if (ordered) s = seg_order[s];
    const int start = seg_start[s];
    const int end = (s + 1 < nseg) ? seg_start[s + 1] : ndep;
    if (end - start >= long_len && team_blocks > 0) continue;   // the team's
    const unsigned long long t_seg = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_seg = __builtin_amdgcn_s_memtime();
    int iters = 0;
    V3 c = seg_init_carry(seg_key, wcarry, s);
    bool dense = false;
    WinStats ws = {0, 0, 0};
    CarryHist hs;
    hs.n = 0;
    hs.run = 0;
    for (int j = start; j < end; j += 64) {
      V3 mine;
      bool mhit, changed;
      iters += wave_window(sc, maxrec, deprec, dep_pix, j, end, c, mine, mhit, ls, G, dense,
                           changed, ws,
                           wave_k, hs
#if RC_STAMPS
                           , &stp
#endif
                           );
      {
        // the block-window LDS is free in the regular loop (team and helper work is over):
        // 768 bytes per wave stage the publication
        const unsigned long long hm = __ballot(j + lane < end && mhit);
        cin_put_wave(cin, j, 0, end - j < 64 ? end - j : 64, mine, tag, hm,
                     reinterpret_cast<float*>(&s_bw) + wave * 192);
        // phase C may shade these entries now (a window touches at most two batches)
        ready_range(rq_cnt, rq, ts, ndep, j, end - j < 64 ? end : j + 64);
      }
      // a long run of changers: hand the rest of the segment to a helper block (15 carry
      // guesses per step instead of this wave's 3)
      if (helpers > 0 && hs.run >= hand_run && hs.n >= 2 && end - (j + 64) >= kHandMin) {
        int k = -1;
        if (lane == 0 &&
            __hip_atomic_load(&ts->dq.idle, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0) {
          if (__hip_atomic_fetch_add(&ts->dq.idle, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0)
            k = atomicAdd(&ts->dq.prod, 1);
          else   // lost the race for the last idle helper: give the announcement back
            __hip_atomic_fetch_add(&ts->dq.idle, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        k = __shfl(k, 0, 64);
        if (k >= 0) {
          if (lane == 0) {
            DenseItem& it = ts->dq.item[k % kDenseQ];
            it.s = s;
            it.j = j + 64;
            it.hn = hs.n;
            it.c[0] = c.x;
            it.c[1] = c.y;
            it.c[2] = c.z;
            for (int q = 0; q < 4; ++q) {
              it.h[q][0] = hs.h[q].x;
              it.h[q][1] = hs.h[q].y;
              it.h[q][2] = hs.h[q].z;
            }
            __hip_atomic_store(&it.ready, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          }
          break;
        }
      }
    }
#if RC_STAMPS
    if (trace && lane == 0 && end - start > 1000) {
      for (int q = 0; q < 4; ++q) trace[3 * ndep + 4 * s + q] = (unsigned)stp.acc[q];
    }
    for (int q = 0; q < 4; ++q) stp.acc[q] = 0;
#endif
    if (trace && lane == 0) {
      trace[3 * s] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t_seg);
#if RC_STAMPS   // the diagnostic build splits the steps: LANE passes << 16 | COOP steps
      trace[3 * s + 1] = ((unsigned)ws.lane << 16) | ((unsigned)ws.coop & 0xffffu);
      (void)iters;
#else
      trace[3 * s + 1] = (unsigned)iters;
#endif
      trace[3 * s + 2] = (unsigned)(__builtin_amdgcn_s_memtime() - c_seg);
      // start time (low 32 bits of the 100 MHz clock) after the team log
      trace[3 * (size_t)ndep + 4 * (size_t)nseg + 8 * 8192 + s] = (unsigned)t_seg;
    }
  }
  // this wave hands nothing off any more (helper blocks wait for every such wave)
  if (lane == 0)
    __hip_atomic_fetch_add(&ts->dq.finished, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && threadIdx.x == 0) {   // the frame's record: shader clock of this run
    const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - clk_t0;
    const unsigned long long dc = __builtin_amdgcn_s_memtime() - clk_c0;
    if (dt > 0) ts->clock_mhz = (int)(dc * 100ull / dt);
  }
  if (trace && lane == 0)   // debug trace: when each wave leaves
    trace[3 * (size_t)ndep + 5 * (size_t)nseg + 8 * 8192 + blockIdx.x * 4 + wave] =
        (unsigned)__builtin_amdgcn_s_memrealtime();
  if (inres) resolver_phase_c(sc, cam, W, maxrec, dep_pix, deprec, cin, counters,
                              batch_state, rq, out, patch, zcount, ts, tag, inres, helpers);
}
template <bool kStage>
__global__ void __launch_bounds__(kSideBlock) k_side(
    Scene sc, Cam cam, int W, int H, int maxrec, const uint8_t* __restrict__ cls,
    const long long* __restrict__ dep_pix, const DepLine* __restrict__ deprec,
    CinG* __restrict__ cin, int* __restrict__ counters,
    int* __restrict__ batch_state, const int* __restrict__ rq, uint8_t* __restrict__ out,
    uint32_t* __restrict__ patch, unsigned long long* __restrict__ zcount,
    TeamState* __restrict__ ts, int resolve_blocks, unsigned tag, int tiles,
    unsigned* __restrict__ trace) {
  if (!RC_X0_PHASE_C) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  __shared__ int s_go;
  __shared__ StageBuf<kStage> stage;
  stage_scene<kStage>(sc, stage);
  // k_side's LDS reservation keeps it off CUs that hold a resolver workgroup
  // (side_lds_bytes), so a k_side workgroup dispatched BEFORE the resolver's last workgroups
  // holds a CU those need.  Each k_side workgroup therefore waits only briefly for the
  // resolver's census (every resolver workgroup resident): normally a few microseconds; if
  // the side stream won the dispatch race (seen on a process's first frame: the resolver then
  // took 24 ms behind a 20 ms wait) it gives up after 200 us, frees its CU and leaves its
  // batches to k_finish.
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int go = 1;
    while (__hip_atomic_load(&counters[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           resolve_blocks) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000ull) {   // 200 us of the 100 MHz clock
        go = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(64);
    }
    s_go = go;
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&counters[s_go ? 12 : 13], 1);
  if (!s_go) return;
  int zero = 0;
  const int ntiles = ((W + 7) >> 3) * ((H + 7) >> 3);
  while (tiles) {   // the non-DEP pixels' colours (split shading only): always ready
    const int t = wave_ticket(&counters[7]);
    if (t >= ntiles) break;
    shade_tile(sc, cam, W, H, maxrec, t, cls, out, zero);
    if ((threadIdx.x & 63) == 0) atomicAdd(&counters[8], 1);
  }
  phase_c_ready(sc, cam, W, maxrec, dep_pix, deprec, cin, counters, batch_state, rq, out,
                patch, ts, tag, zero, trace);
  flush_events(zero, zcount);
}

// After the resolver: the tiles (when `tiles`) and DEP batches k_side has not claimed.
#ifndef RC_FINISH_WAVES
#define RC_FINISH_WAVES 4   // phase C is throughput work: occupancy over a few spilled registers
#endif
template <bool kStage>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RC_FINISH_WAVES))) k_finish(
    Scene sc, Cam cam, int W, int H, int maxrec, const uint8_t* __restrict__ cls,
    const long long* __restrict__ dep_pix, const DepLine* __restrict__ deprec,
    CinG* __restrict__ cin, int* __restrict__ counters,
    int* __restrict__ batch_state, uint8_t* __restrict__ out, uint32_t* __restrict__ patch,
    unsigned long long* __restrict__ zcount, TeamState* __restrict__ ts, unsigned tag,
    int tiles, const int* __restrict__ rq) {
  if (!RC_X0_PHASE_C) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  // every batch already shaded through the ready queue (the usual case when the resolver's
  // own waves shade them): nothing to stage or claim
  if (rq && !tiles &&
      __hip_atomic_load(&counters[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
          (counters[2] + 63) / 64)
    return;
  __shared__ StageBuf<kStage> stage;
  stage_scene<kStage>(sc, stage);
  int zero = 0;
  const int ntiles = ((W + 7) >> 3) * ((H + 7) >> 3);
  while (tiles) {
    const int t = wave_ticket(&counters[7]);
    if (t >= ntiles) break;
    shade_tile(sc, cam, W, H, maxrec, t, cls, out, zero);
    if ((threadIdx.x & 63) == 0) atomicAdd(&counters[10], 1);
  }
  // with k_side: the ready queue's remaining items first (every batch has completed when this
  // kernel runs: the last ones are the resolver's final rounds, shaded here at full occupancy
  // instead of by k_side's one workgroup per CU), then anything still unclaimed
  if (rq)
    phase_c_ready(sc, cam, W, maxrec, dep_pix, deprec, cin, counters, batch_state, rq,
                  out, patch, ts, tag, zero, nullptr);
  phase_c_passes(sc, cam, W, maxrec, dep_pix, deprec, cin, counters, batch_state, out, patch, ts, tag, false,
                 zero);
  flush_events(zero, zcount);
}

// Phase C after the resolver has finished (stream order: every carry-in is published).  A
// workgroup takes a chunk of kChunk consecutive DEP entries: pass 1 (one lane per entry)
// stores every clean entry (dep_fast, no level hit at its carry-in: its primary shade) and
// compacts the others, with their carry-ins, into an LDS list; pass 2 shades that list in
// full waves (levels 2.. with shading, shade_dep_cont; the whole pixel again when the scene
// is not dep_fast).  Entries are independent once their carry-ins are known, so the list order
// is free; the point is full waves of heavy work (~35 % of the entries are clean at quadric
// 4096^2) without a second kernel or global atomics.
#ifndef RC_CHUNK
#define RC_CHUNK 1024
#endif
constexpr int kChunk = RC_CHUNK;

// kFast = Scene::dep_fast (host-known): each form compiles only its own shading path, which
// keeps the other's live state out of the register budget.
template <bool kStage, bool kFast>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RC_FINISH_WAVES))) k_dep_chunks(
    Scene sc, Cam cam, int W, int row0, int row_step, int maxrec,
    const long long* __restrict__ dep_pix,
    const DepLine* __restrict__ deprec, CinG* __restrict__ cin,
    const int* __restrict__ counters, uint8_t* __restrict__ out, uint32_t* __restrict__ patch,
    unsigned long long* __restrict__ zcount, TeamState* __restrict__ ts, unsigned tag,
    int limit) {
  if (!RC_X0_PHASE_C) sc.has_quadric = sc.has_quadric != 0;   // no cross-term-free form here (RC_X0_*)
  __shared__ StageBuf<kStage> stage;
  __shared__ int s_j[kChunk];
  __shared__ float s_c[kChunk][3];
  __shared__ int s_n;
  stage_scene<kStage>(sc, stage);
  // limit: a row shard's fixed-size exchange delivered carry-ins for its first `limit` entries
  // only (the frame is rendered again when the count exceeds it, rc_shard.hip)
  const int ndep = counters[2] < limit ? counters[2] : limit;
  const int nchunks = (ndep + kChunk - 1) / kChunk;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int zero = 0;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    for (int bb = wave; bb < kChunk / 64; bb += kBlock / 64) {
      const int b = ch * (kChunk / 64) + bb;
      if (b * 64 >= ndep) break;
      const int j = b * 64 + lane;
      V3 c = v3(0.0f, 0.0f, 0.0f);
      bool hit = true;
      (void)batch_carries(cin, ndep, b, tag, true, c, hit, ts);
      const bool in = j < ndep;
      const bool hv = in && (!kFast || hit);
      if (in && !hv) {
        const long long p = dep_pix[j];
        store_dep(out, patch, tag, p, j, dep_pcol(deprec + p));
      }
      const unsigned long long m = __ballot(hv);
      int base = 0;
      if (lane == 0 && m) base = atomicAdd(&s_n, __popcll(m));
      base = __shfl(base, 0, 64);
      if (hv) {
        const int q = base + __popcll(m & lanemask_lt());
        s_j[q] = j;
        s_c[q][0] = c.x;
        s_c[q][1] = c.y;
        s_c[q][2] = c.z;
      }
    }
    __syncthreads();
    const int n = s_n;
    for (int q = threadIdx.x; q < n; q += kBlock) {
      const int j = s_j[q];
      const V3 c = v3(s_c[q][0], s_c[q][1], s_c[q][2]);
      const long long p = dep_pix[j];
      V3 rgb;
      if constexpr (kFast) {
        rgb = shade_dep_cont(sc, deprec + p, maxrec, c, zero);
      } else {
        const int y = row0 + (int)(p / W) * row_step, x = (int)(p % W);   // p: local pixel
        const V3 d = primary_dir(cam, x, y, zero);
        PixelOut po;
        shoot<kModeParityC>(sc, d, maxrec, c, po, zero);
        rgb = po.rgb;
      }
      store_dep(out, patch, tag, p, j, rgb);
    }
    __syncthreads();   // the list is rebuilt for the next chunk
  }
  flush_events(zero, zcount);
}

// ------------------------------------------------------ row shards (rc_shard.hip) --
// A parity image split over G ranks by rows (row y -> rank y % G, local row y / G; SURVEY.md
// §8e).  Every rank runs phase A on its rows into rank-local buffers and packs its DEP entries
// (k_shard_pack); the root gathers them and the ranks' row blocks (every non-DEP pixel is final
// after phase A), rebuilds the image's scan order in a lone frame's layout (k_shard_rows,
// k_row_scan, k_shard_unpack) and runs a lone frame's resolver with phase C inside it, which
// shades every DEP entry into the root's image.  Entries travel in the rank's local scan order,
// which is the image's scan order restricted to the rank's rows.
//
// A DEP entry on the wire: its record (pad = image pixel, pad2 = the last writer pixel before
// it in the same row, -1 = none), that writer's carry-out and the entry's primary shade.  A row's summary: the RowStats
// fields in image pixel indices, the row's first entry in the rank's list and the carry-out of
// the row's last writer (the key of a segment that starts after this row).
struct ShardEntry {
  DepLine rec;   // with the entry's primary shade (phase A, Scene::dep_fast): phase C runs on the root
  float4 kc;     // carry-out of the last writer before the entry in its row
};
struct RowShard {
  int ndep, nstart, loff, pad;
  long long lastw, lastd, wfirst;
  float4 cw;
};
static_assert(sizeof(ShardEntry) == 80 && sizeof(RowShard) == 64, "wire records");

// One wave per local row: the rank's DEP list (local pixels, phase C's index), its wire
// entries (at the local DEP offsets of k_row_scan) and the row summary.
__global__ void __launch_bounds__(256) k_shard_pack(
    const uint8_t* __restrict__ cls, const float4* __restrict__ wcarry,
    const DepLine* __restrict__ deprec, int W, int row0, int row_step, int nrows,
    const int* __restrict__ row_off, long long* __restrict__ dep_pix,
    ShardEntry* __restrict__ ent, RowShard* __restrict__ rs, int thin) {
  const int y = blockIdx.x * kRowWaves + (int)(threadIdx.x >> 6);
  if (y >= nrows) return;
  const int lane = threadIdx.x & 63;
  const long long lbase = (long long)y * W;
  const long long gbase = (long long)(row0 + (long long)y * row_step) * W;
  // thin (the root): records and writer carries are already at their image pixels (k_phase_a
  // rec_img); an entry is only {image pixel, in-row writer before it} (8 B, read in place)
  const long long wbase = thin ? gbase : lbase;
  const unsigned long long lt = lanemask_lt();
  int l0 = row_off[y], nd = 0, ns = 0;
  int lw = -1, ld = -1, wf = -1;   // x of the row's last writer / last DEP / first DEP's writer
  bool first_seen = false;
  for (int x0 = 0; x0 < W; x0 += 64) {
    const int x = x0 + lane;
    const uint8_t c = x < W ? cls[lbase + x] : kClsIdent;
    const unsigned long long md = __ballot(c == kClsDep), mw = __ballot(c == kClsWriter);
    const int kw = (mw & lt) ? x0 + hi_bit(mw & lt) : lw;   // in-row writer before the lane
    const int pd = (md & lt) ? x0 + hi_bit(md & lt) : ld;   // in-row DEP before the lane
    const bool dep = c == kClsDep;
    ns += __popcll(__ballot(dep && pd >= 0 && kw > pd));
    if (!first_seen && md) {
      const int f = __ffsll((long long)md) - 1;
      const unsigned long long wb = mw & (f ? (~0ull >> (64 - f)) : 0ull);
      wf = wb ? x0 + hi_bit(wb) : lw;
      first_seen = true;
    }
    if (dep) {
      const int l = l0 + __popcll(md & lt);
      dep_pix[l] = lbase + x;
      if (thin) {
        ((int2*)ent)[l] = make_int2((int)(gbase + x), kw >= 0 ? (int)(gbase + kw) : -1);
      } else {
        ShardEntry e;
        e.rec = deprec[lbase + x];
        e.rec.r.pad = (int)(gbase + x);
        e.rec.r.pad2 = kw >= 0 ? (int)(gbase + kw) : -1;
        e.kc = kw >= 0 ? wcarry[lbase + kw] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        ent[l] = e;
      }
    }
    l0 += __popcll(md);
    nd += __popcll(md);
    if (mw) lw = x0 + hi_bit(mw);
    if (md) ld = x0 + hi_bit(md);
  }
  if (lane == 0) {
    RowShard r;
    r.ndep = nd;
    r.nstart = ns;
    r.loff = row_off[y];
    r.pad = 0;
    r.lastw = lw >= 0 ? gbase + lw : -1;
    r.lastd = ld >= 0 ? gbase + ld : -1;
    r.wfirst = wf >= 0 ? gbase + wf : -1;
    r.cw = lw >= 0 ? wcarry[wbase + lw] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    rs[y] = r;
  }
}

struct ShardOffs {
  long long off[kMaxShards];   // first entry of rank g in the gathered entry list
};

// Root: the image's RowStats from the gathered row summaries ([G][rmax], row y at [y%G][y/G]).
__global__ void __launch_bounds__(256) k_shard_rows(const RowShard* __restrict__ rsall, int G,
                                                    int rmax, int H, RowStats* __restrict__ rs) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= H) return;
  const RowShard r = rsall[(size_t)(y % G) * rmax + y / G];
  rs[y] = RowStats{r.ndep, r.nstart, r.lastw, r.lastd, r.wfirst};
}

// Root, one wave per image row: the row's entries in scan order -> the resolver's inputs, in a
// lone frame's layout (image pixel indices): the DEP line (record and primary shade) at
// deprec[pixel], dep_pix = the pixels in scan order and every segment's key =
// the image pixel of the writer before it, whose carry-out goes to wcarry[writer] (a DEP
// pixel and a writer are never the same pixel).  The resolver, phase C inside it and its
// framebuffer stores then run exactly as in a lone frame, into the root's image.  A segment
// start is decided exactly as in k_row_compact (writer after the previous DEP).
__global__ void __launch_bounds__(256) k_shard_unpack(
    const RowShard* __restrict__ rsall, const ShardEntry* __restrict__ ent,
    const ShardEntry* __restrict__ ent0, ShardOffs offs,
    int G, int rmax, int W, int H, const int* __restrict__ row_off,
    const int* __restrict__ row_soff, const long long* __restrict__ row_prevw,
    const long long* __restrict__ row_prevd, DepLine* __restrict__ deprec,
    long long* __restrict__ dep_pix, int* __restrict__ seg_start,
    long long* __restrict__ seg_key, float4* __restrict__ wcarry, int bound, int thin0) {
  const int y = blockIdx.x * kRowWaves + (int)(threadIdx.x >> 6);
  if (y >= H) return;
  const int lane = threadIdx.x & 63;
  const long long P = (long long)W * H;
  const int g = y % G;
  const RowShard r = rsall[(size_t)g * rmax + y / G];
  // rank 0's entries are the root's own list (never copied), the others' the gathered blocks;
  // thin0: the root's list is {image pixel, writer} pairs whose records and writer carries its
  // phase A already wrote at their image pixels (k_shard_pack thin)
  const bool th = g == 0 && ent0 && thin0;
  const ShardEntry* e = (g == 0 && ent0 ? ent0 : ent + offs.off[g]) + r.loff;
  const int2* et = (const int2*)ent0 + r.loff;
  const int n = r.ndep;
  const int idx0 = row_off[y];
  int s0 = row_soff[y];
  long long pd = row_prevd[y];
  const long long pw = row_prevw[y];
  float4 pwc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (pw >= 0) {   // the writer before the row is the last writer of its own row
    const int yw = (int)(pw / W);
    pwc = rsall[(size_t)(yw % G) * rmax + yw / G].cw;
  }
  const unsigned long long lt = lanemask_lt();
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const bool valid = i < n;
    ShardEntry q;
    if (valid && !th) q = e[i];
    if (valid && th) {
      const int2 tq = et[i];
      q.rec.r.pad = tq.x;
      q.rec.r.pad2 = tq.y;
    }
    // bound: the fixed-size exchange delivered each rank's first `bound` entries.  A longer
    // list (the frame is then rendered again, rc_shard.hip) reads the next rank's block: such
    // an entry becomes a harmless record (zero directions, shape 0) at the spare pixel P (the
    // root's buffers hold P + 1 pixels), continuing its segment — never an out-of-range shape
    // or pixel index for the resolver and phase C.  The root's own list is read in place: whole.
    const bool spare = valid && ((!th && r.loff + i >= bound) || q.rec.r.pad < 0 ||
                                 q.rec.r.pad >= P);
    if (spare) {
      q.rec = DepLine{DepRec{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0, -1, 0.0f, 0.0f, 0.0f, -1},
                      0.0f, 0.0f, 0.0f, 0};
      q.kc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    const long long pix = valid ? (spare ? P : (long long)q.rec.r.pad) : -1;
    const long long kin = valid && !spare && q.rec.r.pad2 >= 0 && q.rec.r.pad2 < P
                              ? (long long)q.rec.r.pad2 : -1;
    long long prev = __shfl_up(pix, 1, 64);
    if (lane == 0) prev = pd;
    const long long kw = kin >= 0 ? kin : pw;
    const bool st = valid && (prev < 0 || kw > prev);
    const unsigned long long ms = __ballot(st);
    if (valid) {
      const int idx = idx0 + i;
      if (!th || spare) deprec[pix] = q.rec;
      dep_pix[idx] = pix;
      if (st) {
        const int s = s0 + __popcll(ms & lt);
        seg_start[s] = idx;
        seg_key[s] = kw;
        // every entry keyed by kw writes the same carry-out; the root's own in-row writers'
        // carries are in place already
        if (kw >= 0 && !(th && kin >= 0)) wcarry[kw] = kin >= 0 ? q.kc : pwc;
      }
    }
    s0 += __popcll(ms);
    const int last = (n - i0 < 64 ? n - i0 : 64) - 1;
    pd = __shfl(pix, last, 64);
  }
}

// Root: image row y <- gathered[y % G][y / G] (the row-cyclic partition undone).
__global__ void __launch_bounds__(256) k_deinterleave(const uint8_t* __restrict__ gathered,
                                                      const uint8_t* __restrict__ block0,
                                                      int G, int rmax, int W, int H,
                                                      uint8_t* __restrict__ img) {
  const int y = blockIdx.x;
  const size_t rb = (size_t)W * 3;
  // rank 0's rows come from the root's own block (not copied into `gathered`)
  const uint8_t* src = (y % G == 0 && block0) ? block0 + (size_t)(y / G) * rb
                                              : gathered + ((size_t)(y % G) * rmax + y / G) * rb;
  uint8_t* dst = img + (size_t)y * rb;
  if ((rb & 3) == 0) {
    for (size_t i = threadIdx.x; i < rb / 4; i += blockDim.x)
      ((uint32_t*)dst)[i] = ((const uint32_t*)src)[i];
  } else {
    for (size_t i = threadIdx.x; i < rb; i += blockDim.x) dst[i] = src[i];
  }
}

// ---------------------------------------------------------------------- launchers --
static Scene make_scene(const LaunchScene& s) {
  Scene sc;
  sc.shapes = s.shapes;
  sc.lights = s.lights;
  sc.pairs = s.pairs;
  sc.lshapes = s.shapes;
  sc.lpairs = s.pairs;
  sc.n = s.n;
  sc.m = s.m;
  sc.refl_mask = s.refl_mask;
  sc.has_quadric = s.has_quadric;
  sc.o0_ok = s.o0_ok;
  sc.dep_fast = s.dep_fast;
  return sc;
}
static bool stage_fits(const LaunchScene& s) {
  return s.n + 1 <= kStageShapes && (s.n + 1) * s.m <= kStagePairs;
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
                         hipStream_t stream, bool cuda_sem) {
  dim3 grid((W + kTileW - 1) / kTileW, (nrows + kTileH - 1) / kTileH);
  if (cuda_sem) {
    hipLaunchKernelGGL(stage_fits(s) ? k_render_cuda<true> : k_render_cuda<false>, grid,
                       dim3(kBlock), 0, stream, make_scene(s), make_cam(s, W, H), W, row0,
                       row_step, nrows, maxrec, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(stage_fits(s) ? k_render<true> : k_render<false>, grid, dim3(kBlock), 0, stream, make_scene(s), make_cam(s, W, H),
                     W, H, row0, row_step, nrows, maxrec, out, zcount);
  return hipGetLastError();
}

static void enqueue_phase_c(const Scene& sc, const Cam& cam, bool st, int W, int H, int maxrec,
                            uint8_t* out, const ParityWork& w, unsigned long long* zcount,
                            hipStream_t stream);

hipError_t launch_parity(const LaunchScene& s, int W, int H, int maxrec, uint8_t* out,
                         const ParityWork& w, unsigned long long* zcount, hipStream_t stream,
                         const hipEvent_t* ev) {
  // ev (optional): [0] after phase A, [1] after compaction, [2] after the resolver,
  // [3] after phase C
  const Scene sc = make_scene(s);
  const Cam cam = make_cam(s, W, H);
  const bool st = stage_fits(s);
  dim3 grid((W + kTileW - 1) / kTileW, (H + kTileH - 1) / kTileH);
  auto kres = s.n <= kLdsShapes ? k_resolve<true> : k_resolve<false>;
  if (w.side && w.split_shade)   // carry part only; colours shaded beside the resolver (k_side)
    hipLaunchKernelGGL(st ? k_classify<true> : k_classify<false>, grid, dim3(kBlock), 0, stream, sc, cam, W, H, maxrec, w.cls,
                       w.wcarry, (DepLine*)w.deprec);
  else
    hipLaunchKernelGGL(st ? k_phase_a<true> : k_phase_a<false>, grid, dim3(kBlock), 0, stream, sc, cam, W, 0, 1, H, maxrec, out,
                       w.cls, w.wcarry, (DepLine*)w.deprec, zcount, W);
  if (ev) (void)hipEventRecord(ev[0], stream);
  if (w.adone) (void)hipEventRecord(w.adone, stream);
  // frames in flight: the compaction (small latency-bound kernels that gate this frame's
  // resolver) leaves the pixel partition, where its workgroups would queue behind the other
  // frames' phase A / phase C workgroups
  if (w.cstream && w.adone) {
    (void)hipStreamWaitEvent(w.cstream, w.adone, 0);
    stream = w.cstream;
  }
  // k_row_stats clears the counters (nseg, head, ndep, ...) and the TeamState (error word,
  // round tags, queues) before anything reads them
  const int row_blocks = (H + kRowWaves - 1) / kRowWaves;
  const int block_cap = w.resolve_blocks - w.team_blocks - w.helpers - w.headb_first;
  hipLaunchKernelGGL(k_row_stats, dim3(row_blocks), dim3(256), 0, stream, w.cls, W, H,
                     (RowStats*)w.row_stats, w.counters, (uint4*)w.team,
                     (int)(sizeof(TeamState) / sizeof(uint4)), w.batch_state, w.batch_ints);
  hipLaunchKernelGGL(k_row_scan, dim3(1), dim3(kScanBlock), 0, stream, H, (const RowStats*)w.row_stats,
                     w.row_off, w.row_soff, w.row_prevw, w.row_prevd, w.counters);
  hipLaunchKernelGGL(k_row_compact, dim3(row_blocks), dim3(256), 0, stream, w.cls, W, H,
                     w.row_off, w.row_soff, w.row_prevw, w.row_prevd, w.dep_pix, w.seg_start,
                     w.seg_key);
  hipLaunchKernelGGL(k_seg_order, dim3(1), dim3(kScanBlock), 0, stream, w.seg_start, w.counters,
                     w.seg_order, w.batch_state, w.batch_cnt, w.batch_rq, w.block_min,
                     block_cap, w.batch_ints > 0 ? 0 : 1);
  // resolve_lds > 80 KiB keeps one resolver block (4 waves, one per SIMD) per CU: the chain
  // steps are latency-bound, so a resolver wave should not share its SIMD
  if (ev) (void)hipEventRecord(ev[1], stream);
  if (w.side) (void)hipEventRecord(w.fork, stream);
  hipStream_t rs = stream;
  if (w.rstream) {   // pipelined: the resolver on its partition, in frame order
    rs = w.rstream;
    (void)hipEventRecord(w.rready, stream);
    (void)hipStreamWaitEvent(rs, w.rready, 0);
    if (w.rt0) (void)hipEventRecord(w.rt0, rs);
  }
  hipLaunchKernelGGL(kres, dim3(w.resolve_blocks), dim3(kResolveBlock), w.resolve_lds, rs, sc,
                     maxrec, (const DepLine*)w.deprec, w.dep_pix, w.seg_key, w.wcarry,
                     w.seg_start, w.seg_order, w.counters, w.counters + 1, (CinG*)w.cin, w.team_blocks,
                     w.long_len, (TeamState*)w.team, w.trace, w.coop_group, w.wave_k,
                     w.resolve_k, w.resolve_clean > 0 ? w.resolve_clean : 1, w.team_cscan, w.epoch, w.helpers, w.hand_run, w.inject, w.block_min,
                     w.headb_first, (w.side || w.inres) ? w.batch_cnt : nullptr, w.batch_rq, cam, W, out,
                     w.patch, zcount, w.batch_state, w.inres);
  if (w.rstream) {
    if (w.rt1) (void)hipEventRecord(w.rt1, rs);
    (void)hipEventRecord(w.rdone, rs);
    if (w.defer_c) return hipGetLastError();   // phase C: launch_phase_c, later
    if (w.pstream) stream = w.pstream;
    (void)hipStreamWaitEvent(stream, w.rdone, 0);
  }
  if (w.side) {   // colours and phase C beside the resolver
    (void)hipStreamWaitEvent(w.side, w.fork, 0);
    hipLaunchKernelGGL(st ? k_side<true> : k_side<false>, dim3(w.side_blocks), dim3(kSideBlock), w.side_lds, w.side, sc, cam,
                       W, H, maxrec, w.cls, w.dep_pix, (const DepLine*)w.deprec,
                       (CinG*)w.cin, w.counters,
                       w.batch_state, w.batch_rq,
                       out, w.patch, zcount, (TeamState*)w.team, w.resolve_blocks, w.epoch,
                       w.split_shade, w.trace);
    (void)hipEventRecord(w.join, w.side);
  }
  if (ev) (void)hipEventRecord(ev[2], stream);
  enqueue_phase_c(sc, cam, st, W, H, maxrec, out, w, zcount, stream);
  if (w.side) (void)hipStreamWaitEvent(stream, w.join, 0);
  if (ev) (void)hipEventRecord(ev[3], stream);
  return hipGetLastError();
}

hipError_t launch_phase_c(const LaunchScene& s, int W, int H, int maxrec, uint8_t* out,
                          const ParityWork& w, unsigned long long* zcount, hipStream_t stream) {
  (void)hipStreamWaitEvent(stream, w.rdone, 0);
  enqueue_phase_c(make_scene(s), make_cam(s, W, H), stage_fits(s), W, H, maxrec, out, w, zcount,
                  stream);
  return hipGetLastError();
}

static void enqueue_phase_c(const Scene& sc, const Cam& cam, bool st, int W, int H, int maxrec,
                            uint8_t* out, const ParityWork& w, unsigned long long* zcount,
                            hipStream_t stream) {
  if (w.side || w.inres || w.phase_c_finish) {   // what k_side / the resolver's waves left
    hipLaunchKernelGGL(st ? k_finish<true> : k_finish<false>, dim3(w.phase_c_blocks), dim3(kBlock), 0, stream, sc, cam, W, H,
                       maxrec, w.cls, w.dep_pix, (const DepLine*)w.deprec,
                       (CinG*)w.cin, w.counters, w.batch_state,
                       out, w.patch,
                       zcount, (TeamState*)w.team, w.epoch, (w.side && w.split_shade) ? 1 : 0,
                       (w.side || w.inres) ? w.batch_rq : nullptr);
  } else {   // all of phase C after the resolver: clean entries, then full waves of the rest
    hipLaunchKernelGGL((sc.dep_fast ? (st ? k_dep_chunks<true, true> : k_dep_chunks<false, true>)
                               : (st ? k_dep_chunks<true, false> : k_dep_chunks<false, false>)), dim3(w.phase_c_blocks),
                       dim3(kBlock), 0, stream, sc, cam, W, 0, 1, maxrec, w.dep_pix,
                       (const DepLine*)w.deprec, (CinG*)w.cin,
                       w.counters, out, w.patch, zcount, (TeamState*)w.team, w.epoch,
                       0x7fffffff);
  }
}

size_t team_state_bytes() { return sizeof(TeamState); }
size_t team_dq_offset() { return offsetof(TeamState, dq); }
size_t team_slot_offset() { return offsetof(TeamState, slot); }
int team_slot_bufs() { return kTeamBufs; }
int team_slot_blocks() { return kTeamMax; }
size_t team_handoff_diag_offset() {
#if RC_HANDOFF_DIAG
  return offsetof(TeamState, hd_err_t);
#else
  return 0;
#endif
}

// k_side workgroups per CU such that one resolver workgroup (one wave per SIMD) still fits
// beside them in every SIMD's 512 VGPRs: k_side waits for the resolver's census, so it must
// never be what keeps a resolver workgroup out.
// k_side's LDS reservation: more than a resolver workgroup leaves free on its CU (so k_side
// only runs on CUs the resolver has left: sharing a CU with the carry chains and the team
// measurably slows them), as small as that allows (more k_side workgroups per vacated CU).
int side_lds_bytes(int resolve_dyn_lds) {
  hipFuncAttributes a, b;
  if (hipFuncGetAttributes(&a, (const void*)k_resolve<true>) != hipSuccess ||
      hipFuncGetAttributes(&b, (const void*)k_resolve<false>) != hipSuccess)
    return 65 * 1024;
  const int lds_cu = 160 * 1024;
  const int stat = (int)(a.sharedSizeBytes < b.sharedSizeBytes ? a.sharedSizeBytes
                                                                : b.sharedSizeBytes);
  int guard = lds_cu - resolve_dyn_lds - stat + 512;   // the most a resolver CU leaves free
  guard = (guard + 511) / 512 * 512;
  if (guard < 1024) guard = 1024;
  return guard;
}

int phase_c_side_blocks(int cus, int side_lds) {
  (void)hipFuncSetAttribute((const void*)k_side<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, side_lds);
  (void)hipFuncSetAttribute((const void*)k_side<true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, side_lds);
  int per_cu = 0;   // the staged variant (more LDS) bounds both
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_side<true>, kSideBlock, side_lds) !=
          hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
#if RC_DIAG
  if (std::getenv("RC_SIDE_STATS"))
    std::fprintf(stderr, "side lds %d -> %d workgroups per CU\n", side_lds, per_cu);
#endif
  return per_cu * cus;
}

int resolve_blocks_resident(int cus, int lds_bytes) {
  // the attribute is an upper bound for every launch: keep it at the largest reservation in
  // use (lone frames 96 KiB, pipeline lanes 56 KiB)
  static int max_set = 0;
  const int cap = lds_bytes > 96 * 1024 ? lds_bytes : 96 * 1024;
  if (cap > max_set) {
    (void)hipFuncSetAttribute((const void*)k_resolve<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    (void)hipFuncSetAttribute((const void*)k_resolve<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, cap);
    max_set = cap;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_resolve<true>, kResolveBlock,
                                                   lds_bytes) != hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
  return per_cu * cus;
}

int resolve_resources(int lds_bytes, int* regs, int* scratch, int* wg_per_cu) {
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, (const void*)k_resolve<true>) != hipSuccess) return -1;
  if (regs) *regs = a.numRegs;
  if (scratch) *scratch = (int)a.localSizeBytes;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_resolve<true>, kResolveBlock,
                                                   lds_bytes) != hipSuccess)
    return -1;
  if (wg_per_cu) *wg_per_cu = per_cu;
  return 0;
}

// ----------------------------------------------------------- row-shard launchers --
size_t shard_entry_bytes() { return sizeof(ShardEntry); }
size_t shard_row_bytes() { return sizeof(RowShard); }

hipError_t launch_shard_local(const LaunchScene& s, int W, int H, int row0, int row_step,
                              int nrows, int maxrec, uint8_t* out, const ParityWork& w,
                              void* ent, void* rows, unsigned long long* zcount,
                              hipStream_t stream, void* img_rec, float4* img_wcarry) {
  const Scene sc = make_scene(s);
  const bool thin = img_rec && img_wcarry;
  const Cam cam = make_cam(s, W, H);
  const bool st = stage_fits(s);
  (void)hipMemsetAsync(w.counters, 0, 16 * sizeof(int), stream);
  (void)hipMemsetAsync(w.team, 0, sizeof(TeamState), stream);
  if (nrows <= 0) return hipGetLastError();
  dim3 grid((W + kTileW - 1) / kTileW, (nrows + kTileH - 1) / kTileH);
  hipLaunchKernelGGL(st ? k_phase_a<true> : k_phase_a<false>, grid, dim3(kBlock), 0, stream, sc,
                     cam, W, row0, row_step, nrows, maxrec, out, w.cls,
                     thin ? img_wcarry + (size_t)row0 * W : w.wcarry,
                     thin ? (DepLine*)img_rec + (size_t)row0 * W : (DepLine*)w.deprec, zcount,
                     thin ? row_step * W : W);
  const int row_blocks = (nrows + kRowWaves - 1) / kRowWaves;
  hipLaunchKernelGGL(k_row_stats, dim3(row_blocks), dim3(256), 0, stream, w.cls, W, nrows,
                     (RowStats*)w.row_stats, nullptr, nullptr, 0, nullptr, 0);
  hipLaunchKernelGGL(k_row_scan, dim3(1), dim3(kScanBlock), 0, stream, nrows,
                     (const RowStats*)w.row_stats, w.row_off, w.row_soff, w.row_prevw,
                     w.row_prevd, w.counters);
  hipLaunchKernelGGL(k_shard_pack, dim3(row_blocks), dim3(256), 0, stream, w.cls,
                     thin ? img_wcarry : w.wcarry, (const DepLine*)w.deprec, W, row0, row_step,
                     nrows, w.row_off, w.dep_pix, (ShardEntry*)ent, (RowShard*)rows, thin ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_shard_resolve(const LaunchScene& s, int W, int H, int G, int rmax,
                                const void* rows_all, const void* ent_all, const void* ent0,
                                const long long* offs, int maxrec, const ParityWork& w,
                                uint8_t* out, unsigned long long* zcount, hipStream_t stream,
                                const hipEvent_t* ev, int bound, int thin0) {
  if (G < 1 || G > kMaxShards || w.side || w.patch) return hipErrorInvalidValue;
  const Scene sc = make_scene(s);
  const Cam cam = make_cam(s, W, H);
  ShardOffs o{};
  for (int g = 0; g < G; ++g) o.off[g] = offs[g];
  const RowShard* rs = (const RowShard*)rows_all;
  (void)hipMemsetAsync(w.counters, 0, 16 * sizeof(int), stream);
  (void)hipMemsetAsync(w.team, 0, sizeof(TeamState), stream);
  hipLaunchKernelGGL(k_shard_rows, dim3((H + 255) / 256), dim3(256), 0, stream, rs, G, rmax, H,
                     (RowStats*)w.row_stats);
  hipLaunchKernelGGL(k_row_scan, dim3(1), dim3(kScanBlock), 0, stream, H, (const RowStats*)w.row_stats,
                     w.row_off, w.row_soff, w.row_prevw, w.row_prevd, w.counters);
  const int row_blocks = (H + kRowWaves - 1) / kRowWaves;
  hipLaunchKernelGGL(k_shard_unpack, dim3(row_blocks), dim3(256), 0, stream, rs,
                     (const ShardEntry*)ent_all, (const ShardEntry*)ent0, o, G, rmax, W, H,
                     w.row_off, w.row_soff,
                     w.row_prevw, w.row_prevd, (DepLine*)w.deprec, w.dep_pix, w.seg_start,
                     w.seg_key, w.wcarry, bound, thin0);
  hipLaunchKernelGGL(k_seg_order, dim3(1), dim3(kScanBlock), 0, stream, w.seg_start, w.counters,
                     w.seg_order, w.batch_state, w.batch_cnt, w.batch_rq, w.block_min,
                     w.resolve_blocks - w.team_blocks - w.helpers - w.headb_first, 1);
  if (ev) (void)hipEventRecord(ev[0], stream);
  // a lone frame's resolver from here on: phase C inside it (w.inres) shades every DEP entry
  // of the image into `out` — the root's image, whose non-DEP pixels the gathered row blocks
  // already hold — and k_finish takes what its waves left
  auto kres = s.n <= kLdsShapes ? k_resolve<true> : k_resolve<false>;
  hipLaunchKernelGGL(kres, dim3(w.resolve_blocks), dim3(kResolveBlock), w.resolve_lds, stream,
                     sc, maxrec, (const DepLine*)w.deprec, w.dep_pix, w.seg_key, w.wcarry,
                     w.seg_start, w.seg_order, w.counters, w.counters + 1, (CinG*)w.cin,
                     w.team_blocks, w.long_len, (TeamState*)w.team, w.trace, w.coop_group,
                     w.wave_k, w.resolve_k, w.resolve_clean > 0 ? w.resolve_clean : 1,
                     w.team_cscan, w.epoch, w.helpers, w.hand_run, w.inject, w.block_min,
                     w.headb_first, w.inres ? w.batch_cnt : nullptr, w.batch_rq, cam, W, out, (uint32_t*)nullptr,
                     zcount, w.batch_state, w.inres);
  if (ev) (void)hipEventRecord(ev[1], stream);
  enqueue_phase_c(sc, cam, stage_fits(s), W, H, maxrec, out, w, zcount, stream);
  return hipGetLastError();
}

hipError_t launch_deinterleave(const uint8_t* gathered, const uint8_t* block0, int G, int rmax,
                               int W, int H, uint8_t* img, hipStream_t stream) {
  if (H <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_deinterleave, dim3(H), dim3(256), 0, stream, gathered, block0, G, rmax, W,
                     H, img);
  return hipGetLastError();
}

size_t deprec_bytes() { return sizeof(DepLine); }   // one line per pixel (DepLine)
size_t row_stats_bytes() { return sizeof(RowStats); }

}  // namespace rc
