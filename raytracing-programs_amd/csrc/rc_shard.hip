// rc_shard.hip — row-sharded rendering over several GPUs (C/raycast.c:113-129 is
// the scan loop whose rows are dealt out).
//
// Rows are dealt cyclically: row y -> rank y % G (contiguous blocks are 1.7-2.1x imbalanced at
// 8 ranks).  A rank renders its rows into a compact local framebuffer (local row
// j = image row rank + j*G); the root (rank 0) gathers the row blocks over RCCL (ncclGather,
// xGMI) and undoes the interleave on the device (k_deinterleave).
//
// Parity mode adds the carry chain's exchange (C/raycast.c:340 scan-order carry): every rank
// runs phase A on its rows and packs its DEP entries (record + in-row writer key and carry +
// primary shade) and per-row summaries; the root gathers them (ncclGather of the row
// summaries, ncclGather / ncclSend-ncclRecv of the entry lists) and the row blocks, whose
// non-DEP pixels are final, rebuilds the image's scan order and runs a lone frame's carry
// resolver with phase C inside it, which shades every DEP entry into the root's image.  The
// resolver stays serial on the root, so parity scaling is capped by it.
//
// A group is either one rank of a multi-process job (one process per GPU, rc_group_create_rank,
// the ncclUniqueId shared by the caller) or every rank in this process (rc_group_create_local:
// one host thread drives all ranks' streams; RCCL communicators from ncclCommInitAll, or — when
// ranks share a device, which RCCL does not allow — device copies between the ranks' buffers).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <vector>

#include "raycast_hip.h"
#include "rc_kernels.h"
#include "rc_runtime.h"

using namespace rcrt;

namespace {

#define NCCL_TRY(expr)                                                                   \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess) {                                                             \
      std::fprintf(stderr, "Error: RCCL call failed: %s (%s) at %s:%d\n", #expr,        \
                   ncclGetErrorString(r_), __FILE__, __LINE__);                          \
      return -1;                                                                         \
    }                                                                                    \
  } while (0)

// One rank driven by this process.
struct Rank {
  int rank = 0;
  int device = 0;
  DevCtx* c = nullptr;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  hipEvent_t ready = nullptr;   // COPY transport: this rank's send buffers are complete
  FrameBufs fb;                 // rank-local phase A / phase C workspace
  DevBuf frame;                 // local framebuffer, rmax rows
  DevBuf ent, rows;             // wire: DEP entries, row summaries
  DevBuf small;                 // [0] int: DEP entries; [2..3] u64: zero-normalize events
  int* h_small = nullptr;       // pinned copy of `small` ([10..11]: the root's phase C events)
  int nrows = 0;
  long long ndep = 0;
  hipEvent_t rev[4] = {};       // this rank's timeline: start, rows done, sends done, frame end
  rc_rank_stats last{};
  // root only
  FrameBufs rootfb;             // image-wide resolver workspace
  DevBuf rows_all, ent_all, frames_all, small_all, image;
  int* h_small_all = nullptr;   // pinned, kMaxShards x 4 ints
  hipEvent_t ev[6] = {};        // root timeline: start, phase A, resolver start/end, phase C
                                // tail, image complete
};

}  // namespace

struct rc_group {
  int nranks = 1;
  int transport = RC_XFER_RCCL;
  std::vector<std::unique_ptr<Rank>> ranks;   // the ranks this process drives
  Rank* root = nullptr;                       // rank 0 when this process drives it
  unsigned epoch = 0;                         // carry-in tag of the last sharded parity frame
  rc_shard_stats last{};
  // Fixed-size entry exchange (no host synchronisation inside a frame): the DEP entries per
  // rank of the last frame with this key, an upper bound for the next one.  A frame whose
  // count exceeds it is detected at the frame's end and rendered again with exact sizes.
  // The key is the scene's CONTENT (a hash of its packed image), not its address: every
  // process of a multi-process group must take the same exchange (ncclGather/ncclScatter of
  // fixed blocks, or the exact-size ncclSend/ncclRecv), and the bound itself comes from the
  // frame's all-reduced count, so ranks rendering the same frames reach the same decision.
  struct {
    unsigned long long scene = 0;
    int W = 0, H = 0, maxrec = 0;
    long long per_rank = -1;
  } bound;
};

namespace {

int init_rank(Rank& r, int rank, int device) {
  r.rank = rank;
  r.device = device;
  HIP_TRY(hipSetDevice(device));
  if (ctx_get(device, &r.c)) return -1;
  HIP_TRY(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming));
  for (auto& e : r.rev) HIP_TRY(hipEventCreate(&e));
  HIP_TRY(hipHostMalloc((void**)&r.h_small, 64, hipHostMallocDefault));
  if (r.small.ensure(64) || r.fb.zcount.ensure(64)) return -1;
  if (rank == 0) {
    for (auto& e : r.ev) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hipHostMalloc((void**)&r.h_small_all, rc::kMaxShards * 16, hipHostMallocDefault));
  }
  return 0;
}

void free_buf(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

void free_frame(FrameBufs& f) {
  for (DevBuf* b : {&f.zcount, &f.scene, &f.cls, &f.wcarry, &f.deprec, &f.rows, &f.dep_pix,
                    &f.seg_key, &f.seg_start, &f.seg_order, &f.batch_state, &f.cin, &f.counters,
                    &f.team, &f.trace})
    free_buf(*b);
}

void release_rank(Rank& r) {
  (void)hipSetDevice(r.device);
  if (r.stream) (void)hipStreamSynchronize(r.stream);
  if (r.comm) (void)ncclCommDestroy(r.comm);
  r.comm = nullptr;
  free_frame(r.fb);
  free_frame(r.rootfb);
  for (DevBuf* b : {&r.frame, &r.ent, &r.rows, &r.small, &r.rows_all, &r.ent_all,
                    &r.frames_all, &r.small_all, &r.image})
    free_buf(*b);
  if (r.h_small) (void)hipHostFree(r.h_small);
  if (r.h_small_all) (void)hipHostFree(r.h_small_all);
  r.h_small = r.h_small_all = nullptr;
  for (auto& e : r.ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : r.rev)
    if (e) (void)hipEventDestroy(e);
  if (r.ready) (void)hipEventDestroy(r.ready);
  if (r.stream) (void)hipStreamDestroy(r.stream);
  r.stream = nullptr;
}

// ------------------------------------------------------------------ transports --
// Every primitive is issued for all ranks this process drives, inside one RCCL group (a
// process that drives several devices must group its calls), or as device copies.

// root.recv[r * bytes ..] <- rank r's send (every rank sends `bytes`)
int gather_fixed(rc_group& g, const std::vector<const void*>& send, void* recv, size_t bytes) {
  if (g.transport == RC_XFER_RCCL) {
    NCCL_TRY(ncclGroupStart());
    for (size_t i = 0; i < g.ranks.size(); ++i) {
      Rank& r = *g.ranks[i];
      NCCL_TRY(ncclGather(send[i], r.rank == 0 ? recv : nullptr, bytes, ncclUint8, 0, r.comm,
                          r.stream));
    }
    NCCL_TRY(ncclGroupEnd());
    return 0;
  }
  Rank& root = *g.root;
  for (size_t i = 0; i < g.ranks.size(); ++i) {
    Rank& r = *g.ranks[i];
    HIP_TRY(hipSetDevice(r.device));
    HIP_TRY(hipEventRecord(r.ready, r.stream));
  }
  HIP_TRY(hipSetDevice(root.device));
  for (size_t i = 0; i < g.ranks.size(); ++i) {
    Rank& r = *g.ranks[i];
    if (&r != &root) HIP_TRY(hipStreamWaitEvent(root.stream, r.ready, 0));
    HIP_TRY(hipMemcpyAsync((char*)recv + (size_t)r.rank * bytes, send[i], bytes, hipMemcpyDefault,
                           root.stream));
  }
  return 0;
}

// root.recv[off[r] ..] <- rank r's send (bytes[r] bytes; the root knows every rank's size, a
// rank its own).  self = false: the root's own part stays where it is (the reader takes it in
// place), so nothing is copied for rank 0 — at G = 1 nothing moves at all.
int gather_var(rc_group& g, const std::vector<const void*>& send, void* recv,
               const std::vector<size_t>& off, const std::vector<size_t>& bytes,
               bool self = true) {
  if (g.transport == RC_XFER_RCCL) {
    NCCL_TRY(ncclGroupStart());
    for (size_t i = 0; i < g.ranks.size(); ++i) {
      Rank& r = *g.ranks[i];
      if (r.rank != 0) {
        if (bytes[r.rank]) NCCL_TRY(ncclSend(send[i], bytes[r.rank], ncclUint8, 0, r.comm, r.stream));
        continue;
      }
      for (int q = 1; q < g.nranks; ++q)
        if (bytes[q])
          NCCL_TRY(ncclRecv((char*)recv + off[q], bytes[q], ncclUint8, q, r.comm, r.stream));
    }
    NCCL_TRY(ncclGroupEnd());
    if (self && g.root && bytes[0]) {   // the root's own part
      HIP_TRY(hipSetDevice(g.root->device));
      HIP_TRY(hipMemcpyAsync(recv, send[0], bytes[0], hipMemcpyDeviceToDevice, g.root->stream));
    }
    return 0;
  }
  Rank& root = *g.root;
  for (size_t i = 0; i < g.ranks.size(); ++i) {
    Rank& r = *g.ranks[i];
    HIP_TRY(hipSetDevice(r.device));
    HIP_TRY(hipEventRecord(r.ready, r.stream));
  }
  HIP_TRY(hipSetDevice(root.device));
  for (size_t i = 0; i < g.ranks.size(); ++i) {
    Rank& r = *g.ranks[i];
    if (&r != &root) HIP_TRY(hipStreamWaitEvent(root.stream, r.ready, 0));
    if (bytes[r.rank] && (self || &r != &root))
      HIP_TRY(hipMemcpyAsync((char*)recv + off[r.rank], send[i], bytes[r.rank], hipMemcpyDefault,
                             root.stream));
  }
  return 0;
}

int sync_all(rc_group& g) {
  for (auto& rp : g.ranks) {
    HIP_TRY(hipSetDevice(rp->device));
    HIP_TRY(hipStreamSynchronize(rp->stream));
  }
  return 0;
}

// FNV-1a of the packed scene image (header included): equal on every rank given equal scenes
unsigned long long scene_key(const rc_packed_header* h) {
  const unsigned char* p = (const unsigned char*)h;
  unsigned long long x = 1469598103934665603ull;
  for (int i = 0; i < h->bytes; ++i) x = (x ^ p[i]) * 1099511628211ull;
  return x;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// A group of one rank has nothing to exchange: the rank renders the whole image as a lone
// frame (rc_render_device's path, phase C inside the resolver) into d_image on its stream.
// The sharded machinery (wire records, gathers, the root's resolver on gathered entries,
// phase C after it) cost 1.2 ms more at 4096^2 (profiles/r03b_bench_force_group.log).
int render_one_rank(rc_group& g, const rc_scene* s, int W, int H, const rc_options* opt,
                    uint8_t* d_image, rc_timing* timing,
                    std::chrono::steady_clock::time_point t0) {
  Rank& r = *g.root;
  HIP_TRY(hipSetDevice(r.device));
  if (!d_image) {
    if (r.image.ensure((size_t)H * W * 3)) return -1;
    d_image = (uint8_t*)r.image.p;
  }
  DevCtx& c = *r.c;
  if (c.lone_log.earlier_failed()) {   // an earlier lone frame of this workspace failed
    c.lone_log.take(nullptr, nullptr);
    return -1;
  }
  // the scene upload and the phase events live on the ctx stream: the rank's stream here
  hipStream_t saved = c.stream;
  c.stream = r.stream;
  const long long own = c.lone_log.head;   // this frame's ring entry
  const int rc = enqueue_render(c, s, W, H, 0, 1, H, opt, d_image, r.stream, true);
  c.stream = saved;
  if (rc) return -1;
  HIP_TRY(hipStreamSynchronize(r.stream));
  const bool failed = c.lone_log.entry_failed(own);
  c.lone_log.poll();
  if (failed) {
    c.lone_log.take(nullptr, nullptr);
    return -1;
  }
  if (check_spin_error(c.fb, opt)) return -1;
  rc_timing t{};
  fill_device_timing(c, opt, &t);
  rc_shard_stats& st = g.last;
  std::memset(&st, 0, sizeof st);
  st.total_ms = ms_since(t0);
  st.ranks = 1;
  st.device_ms = t.kernel_ms;
  st.resolve_ms = t.resolve_ms;
  st.dep_pixels = t.dep_pixels;
  st.zero_normalize = t.zero_normalize;
  st.image_bytes = (long long)H * W * 3;
  if (timing) {
    std::memset(timing, 0, sizeof *timing);
    timing->total_ms = st.total_ms;
    timing->kernel_ms = st.device_ms;
    timing->resolve_ms = st.resolve_ms;
    timing->dep_pixels = st.dep_pixels;
    timing->zero_normalize = st.zero_normalize;
  }
  return 0;
}

// The whole sharded render; the caller holds every driven device's lock.
//   fast:   every rank renders its rows; the row blocks are gathered and de-interleaved.
//   parity: every rank runs phase A on its rows and packs its DEP entries (wire records with
//           each entry's primary shade) and row summaries; the root gathers them and the row
//           blocks (every non-DEP pixel is final after phase A) and de-interleaves the blocks
//           into its image; it rebuilds the image's scan order in a lone frame's layout and
//           runs a lone frame's resolver with phase C inside it, which shades every DEP entry
//           into that image.  Nothing returns to the ranks: no carry-in scatter, no phase C on
//           the ranks (round 3 did both, and gathered the row blocks only after phase C).
int render_sharded(rc_group& g, const rc_scene* s, int W, int H, const rc_options* opt,
                   uint8_t* d_image, rc_timing* timing) {
  const auto t0 = std::chrono::steady_clock::now();
  const int G = g.nranks;
  const int rmax = (H + G - 1) / G;
  const int maxrec = opt->max_recursion;
  const bool parity = opt->mode == RC_MODE_PARITY && maxrec > 1;
  const size_t row_bytes = (size_t)W * 3;
  const size_t block_bytes = (size_t)rmax * row_bytes;
  const size_t P = (size_t)W * H;
  Rank* root = g.root;
  if (G == 1 && root && tune().shard_lone)
    return render_one_rank(g, s, W, H, opt, d_image, timing, t0);
  uint8_t* img = d_image;   // parity: the root's own image (P + 1 pixels: one spare)
  if (root) {
    HIP_TRY(hipSetDevice(root->device));
    if (parity || !d_image) {
      if (root->image.ensure((P + 1) * 3)) return -1;
      img = (uint8_t*)root->image.p;
      if (!d_image) d_image = img;
    }
    if (root->frames_all.ensure((size_t)G * block_bytes) || root->small_all.ensure((size_t)G * 16))
      return -1;
    // parity: the root's own phase A writes its DEP lines and writer carries straight into the
    // resolver's image-indexed buffers (W*H + 1 pixels), so its entries never travel or unpack
    if (parity && (root->rootfb.deprec.ensure((P + 1) * rc::deprec_bytes()) ||
                   root->rootfb.wcarry.ensure((P + 1) * sizeof(float4)))) {
      std::fprintf(stderr, "Error: out of device memory for the root's resolver workspace\n");
      return -1;
    }
    HIP_TRY(hipEventRecord(root->ev[0], root->stream));
  }
  std::vector<rc::LaunchScene> ls(g.ranks.size());
  std::vector<rc::ParityWork> w(g.ranks.size());
  // 1. every rank: its rows (fast: the whole render; parity: phase A + the wire records)
  for (size_t i = 0; i < g.ranks.size(); ++i) {
    Rank& r = *g.ranks[i];
    HIP_TRY(hipSetDevice(r.device));
    HIP_TRY(hipEventRecord(r.rev[0], r.stream));
    r.nrows = (H - r.rank + G - 1) / G;
    if (r.nrows < 0) r.nrows = 0;
    if (r.frame.ensure(block_bytes)) return -1;
    if (upload_scene(r.fb, r.stream, s, ls[i])) return -1;
    unsigned long long* zc = (unsigned long long*)r.fb.zcount.p;
    HIP_TRY(hipMemsetAsync(zc, 0, sizeof(unsigned long long), r.stream));
    if (!parity) {
      if (r.nrows > 0)
        HIP_TRY(rc::launch_render(ls[i], W, H, r.rank, G, r.nrows, maxrec, (uint8_t*)r.frame.p,
                                  zc, r.stream, opt->mode == RC_MODE_CUDA));
      HIP_TRY(hipEventRecord(r.rev[1], r.stream));
      continue;
    }
    // workspace for rmax rows on every rank: the fixed-size exchange moves the same number of
    // entries (up to the bound, <= rmax * W) out of every rank's buffers
    if (ensure_parity(*r.c, r.fb, W, rmax, w[i], r.c->cus) ||
        r.ent.ensure((size_t)rmax * W * rc::shard_entry_bytes()) ||
        r.rows.ensure((size_t)rmax * rc::shard_row_bytes())) {
      std::fprintf(stderr, "Error: out of device memory for the shard workspace\n");
      return -1;
    }
    const bool thin = &r == root;
    HIP_TRY(rc::launch_shard_local(ls[i], W, H, r.rank, G, r.nrows, maxrec, (uint8_t*)r.frame.p,
                                   w[i], r.ent.p, r.rows.p, zc, r.stream,
                                   thin ? root->rootfb.deprec.p : nullptr,
                                   thin ? (float4*)root->rootfb.wcarry.p : nullptr));
    HIP_TRY(hipMemcpyAsync(r.small.p, w[i].counters + 2, sizeof(int), hipMemcpyDeviceToDevice,
                           r.stream));
    HIP_TRY(hipEventRecord(r.rev[1], r.stream));
  }
  if (root) HIP_TRY(hipEventRecord(root->ev[1], root->stream));
  // fixed-size exchange when the last frame with this key bounds the entry counts; a bound
  // beyond a rank's pixel count (rc_group_debug_bound) is that count (the buffers' size)
  const unsigned long long key = parity ? scene_key(s->img) : 0;
  const bool fixed = parity && g.bound.per_rank >= 0 && g.bound.scene == key &&
                     g.bound.W == W && g.bound.H == H && g.bound.maxrec == maxrec;
  const long long per_rank = std::min<long long>(g.bound.per_rank, (long long)rmax * W);
  std::vector<size_t> cnt(G, 0);
  std::vector<long long> offs(G, 0);
  if (parity) {
    // 2. row summaries and entry counts to the root
    std::vector<const void*> sr, sc;
    for (auto& rp : g.ranks) {
      sr.push_back(rp->rows.p);
      sc.push_back(rp->small.p);
    }
    if (root && (root->rows_all.ensure((size_t)G * rmax * rc::shard_row_bytes()))) return -1;
    if (gather_fixed(g, sr, root ? root->rows_all.p : nullptr, (size_t)rmax * rc::shard_row_bytes()) ||
        gather_fixed(g, sc, root ? root->small_all.p : nullptr, 16))
      return -1;
    std::vector<size_t> off(G, 0), eb(G), eo(G);
    if (fixed) {   // every rank's list padded to the bound: sizes known without the counts
      for (int q = 0; q < G; ++q) cnt[q] = (size_t)per_rank;
    } else {   // the counts first (host synchronisation), then the exact sizes
      for (auto& rp : g.ranks) {
        HIP_TRY(hipSetDevice(rp->device));
        HIP_TRY(hipMemcpyAsync(rp->h_small, rp->small.p, 16, hipMemcpyDeviceToHost, rp->stream));
      }
      if (root)
        HIP_TRY(hipMemcpyAsync(root->h_small_all, root->small_all.p, (size_t)G * 16,
                               hipMemcpyDeviceToHost, root->stream));
      if (sync_all(g)) return -1;
      for (auto& rp : g.ranks) rp->ndep = rp->h_small[0];
      for (int q = 0; q < G; ++q) cnt[q] = root ? (size_t)root->h_small_all[4 * q] : 0;
      for (auto& rp : g.ranks) cnt[rp->rank] = (size_t)rp->ndep;
    }
    size_t total = 0;
    for (int q = 0; q < G; ++q) {
      off[q] = total;
      offs[q] = (long long)total;
      total += cnt[q];
    }
    for (int q = 0; q < G; ++q) {
      eb[q] = cnt[q] * rc::shard_entry_bytes();
      eo[q] = off[q] * rc::shard_entry_bytes();
    }
    if (root) {
      HIP_TRY(hipSetDevice(root->device));
      // capacity for every rank's largest possible list (rmax * W): with the fixed-size
      // exchange a list longer than the bound is read (as garbage, the frame is rendered
      // again) beyond its block, never beyond the buffer
      const size_t cap = total > (size_t)G * rmax * W ? total : (size_t)G * rmax * W;
      if (root->ent_all.ensure(cap * rc::shard_entry_bytes() + 64)) {
        std::fprintf(stderr, "Error: out of device memory for the gathered DEP entries\n");
        return -1;
      }
    }
    // 3. the other ranks' entries to the root (its own are read in place); the same point-to-
    //    point pattern for the fixed-size and the exact exchange, only the sizes differ
    std::vector<const void*> se;
    for (auto& rp : g.ranks) se.push_back(rp->ent.p);
    if (gather_var(g, se, root ? root->ent_all.p : nullptr, eo, eb, false)) return -1;
  }
  // 4. the row blocks and the phase-A / render event counts to the root, the interleave undone
  //    there (parity: into the root's image, ahead of the resolver; its DEP pixels follow)
  std::vector<const void*> sf, sz;
  for (auto& rp : g.ranks) {
    HIP_TRY(hipSetDevice(rp->device));
    HIP_TRY(hipMemcpyAsync((char*)rp->small.p + 8, rp->fb.zcount.p, 8, hipMemcpyDeviceToDevice,
                           rp->stream));
    sf.push_back(rp->frame.p);
    sz.push_back(rp->small.p);
  }
  {   // the other ranks' blocks (the root de-interleaves its own in place)
    std::vector<size_t> fo(G), fb(G, block_bytes);
    for (int q = 0; q < G; ++q) fo[q] = (size_t)q * block_bytes;
    if (gather_var(g, sf, root ? root->frames_all.p : nullptr, fo, fb, false) ||
        gather_fixed(g, sz, root ? root->small_all.p : nullptr, 16))
      return -1;
  }
  for (auto& rp : g.ranks) {
    HIP_TRY(hipSetDevice(rp->device));
    HIP_TRY(hipEventRecord(rp->rev[2], rp->stream));
  }
  if (root) {
    HIP_TRY(hipSetDevice(root->device));
    HIP_TRY(rc::launch_deinterleave((const uint8_t*)root->frames_all.p,
                                    (const uint8_t*)root->frame.p, G, rmax, W, H,
                                    parity ? img : d_image, root->stream));
  }
  // 5. parity, the root: the resolver with phase C inside it, into the root's image
  unsigned long long* rz = nullptr;   // the root's phase C events
  if (parity) {
    // this frame's carry-in tag, the same on every rank (ranks render in lockstep)
    g.epoch = g.epoch + 1 >= 0x80000000u ? 1 : g.epoch + 1;
    if (root) {
      rc::ParityWork wr{};
      root->rootfb.epoch = g.epoch - 1;
      root->rootfb.scene_src = s->img;   // the resolver's evaluator is specialised by shape count
      // a lone frame's workspace over the whole image, plus the spare pixel P
      if (ensure_parity(*root->c, root->rootfb, W, H, wr, root->c->cus, 0) ||
          root->rootfb.deprec.ensure((P + 1) * rc::deprec_bytes()) ||
          root->rootfb.wcarry.ensure((P + 1) * sizeof(float4)) || root->rootfb.zcount.ensure(64)) {
        std::fprintf(stderr, "Error: out of device memory for the root's resolver workspace\n");
        return -1;
      }
      if (root->rootfb.epoch != g.epoch)   // ensure_parity cleared the tags on a wrap
        g.epoch = root->rootfb.epoch;
      // ensure_parity's buffers may have been reallocated: the work's pointers are current
      wr.deprec = root->rootfb.deprec.p;
      wr.wcarry = (float4*)root->rootfb.wcarry.p;
      wr.side = nullptr;
      wr.split_shade = 0;
      wr.patch = nullptr;
      if (maxrec < 3) wr.inres = 0;   // a lone frame's schedule: phase C after at depth 1
      rz = (unsigned long long*)root->rootfb.zcount.p;
      HIP_TRY(hipMemsetAsync(rz, 0, sizeof(unsigned long long), root->stream));
      hipEvent_t rev[2] = {root->ev[2], root->ev[3]};
      HIP_TRY(rc::launch_shard_resolve(ls[0], W, H, G, rmax, root->rows_all.p, root->ent_all.p,
                                       root->ent.p, offs.data(), maxrec, wr, img, rz,
                                       root->stream, rev,
                                       fixed ? (int)per_rank : 0x7fffffff, 1));
      HIP_TRY(hipEventRecord(root->ev[4], root->stream));
      if (d_image != img)
        HIP_TRY(hipMemcpyAsync(d_image, img, P * 3, hipMemcpyDeviceToDevice, root->stream));
    }
  } else if (root) {
    HIP_TRY(hipEventRecord(root->ev[2], root->stream));
    HIP_TRY(hipEventRecord(root->ev[3], root->stream));
    HIP_TRY(hipEventRecord(root->ev[4], root->stream));
  }
  if (root) {
    HIP_TRY(hipSetDevice(root->device));
    HIP_TRY(hipMemcpyAsync(root->h_small_all, root->small_all.p, (size_t)G * 16,
                           hipMemcpyDeviceToHost, root->stream));
    if (rz) HIP_TRY(hipMemcpyAsync(root->h_small + 10, rz, 8, hipMemcpyDeviceToHost, root->stream));
    HIP_TRY(hipEventRecord(root->ev[5], root->stream));
  }
  if (parity) {
    // every rank learns the frame's largest entry count (small[4]): the bound of the next
    // frame with this key, and the check of this one's (all ranks decide alike)
    if (g.transport == RC_XFER_RCCL) {
      NCCL_TRY(ncclGroupStart());
      for (auto& rp : g.ranks)
        NCCL_TRY(ncclAllReduce(rp->small.p, (int*)rp->small.p + 4, 1, ncclInt32, ncclMax,
                               rp->comm, rp->stream));
      NCCL_TRY(ncclGroupEnd());
    }
    for (auto& rp : g.ranks) {
      HIP_TRY(hipSetDevice(rp->device));
      HIP_TRY(hipMemcpyAsync(rp->h_small, rp->small.p, 32, hipMemcpyDeviceToHost, rp->stream));
    }
  }
  for (auto& rp : g.ranks) {
    HIP_TRY(hipSetDevice(rp->device));
    HIP_TRY(hipEventRecord(rp->rev[3], rp->stream));
  }
  if (sync_all(g)) return -1;
  int rc = 0;
  if (parity && root && report_spin_error(root->rootfb, "shard resolver")) rc = -1;
  if (parity) {
    // the largest entry count of the frame (RCCL: the all-reduce; device copies: every rank is
    // in this process), identical on every rank
    long long mx = 0;
    for (auto& rp : g.ranks) {
      const long long n = g.transport == RC_XFER_RCCL ? (long long)rp->h_small[4]
                                                      : (long long)rp->h_small[0];
      if (n > mx) mx = n;
    }
    if (fixed && mx > per_rank) {   // an entry list overflowed the padded exchange
      g.bound.per_rank = -1;
      return 1;   // render_sharded_retry renders the frame again with exact sizes
    }
    g.bound.scene = key;
    g.bound.W = W;
    g.bound.H = H;
    g.bound.maxrec = maxrec;
    g.bound.per_rank = mx;
  }
  for (auto& rp : g.ranks) {   // every driven rank's own timeline
    rc_rank_stats& q = rp->last;
    std::memset(&q, 0, sizeof q);
    q.rank = rp->rank;
    q.local_ms = event_ms(rp->rev[0], rp->rev[1]);
    q.exchange_ms = event_ms(rp->rev[1], rp->rev[2]);
    q.total_ms = event_ms(rp->rev[0], rp->rev[3]);
    q.rows = rp->nrows;
    q.dep_pixels = parity ? rp->h_small[0] : 0;   // the rank's own DEP entries
  }
  rc_shard_stats& st = g.last;
  std::memset(&st, 0, sizeof st);
  st.total_ms = ms_since(t0);
  if (root) {
    st.ranks = G;
    st.local_ms = event_ms(root->ev[0], root->ev[1]);
    st.device_ms = event_ms(root->ev[0], root->ev[5]);
    for (int q = 0; q < G; ++q) {
      long long z = 0;
      std::memcpy(&z, root->h_small_all + 4 * q + 2, sizeof z);
      st.zero_normalize += z;
    }
    st.image_bytes = (long long)G * (long long)block_bytes;
    if (parity) {
      long long z = 0;   // the root's phase C (inside its resolver)
      std::memcpy(&z, root->h_small + 10, sizeof z);
      st.zero_normalize += z;
      st.exchange_in_ms = event_ms(root->ev[1], root->ev[2]);
      st.resolve_ms = event_ms(root->ev[2], root->ev[3]);
      st.phase_c_ms = event_ms(root->ev[3], root->ev[4]);
      st.image_ms = event_ms(root->ev[4], root->ev[5]);
      for (int q = 0; q < G; ++q) st.dep_pixels += root->h_small_all[4 * q];
      // what moved: the other ranks' wire records (the root's own entries are read in place)
      st.entry_bytes = (st.dep_pixels - root->h_small_all[0]) * (long long)rc::shard_entry_bytes();
      st.carry_bytes = 0;
    } else {
      st.image_ms = event_ms(root->ev[1], root->ev[5]);
    }
  }
  if (timing) {
    std::memset(timing, 0, sizeof *timing);
    timing->total_ms = st.total_ms;
    timing->kernel_ms = st.device_ms;
    timing->resolve_ms = st.resolve_ms;
    timing->dep_pixels = st.dep_pixels;
    timing->zero_normalize = st.zero_normalize;
  }
  return rc;
}

// A frame whose DEP entries overflowed the fixed-size exchange (render_sharded returns 1, on
// every rank alike) is rendered again with exact sizes.
int render_sharded_retry(rc_group& g, const rc_scene* s, int W, int H, const rc_options* opt,
                         uint8_t* d_image, rc_timing* timing) {
  int rc = render_sharded(g, s, W, H, opt, d_image, timing);
  if (rc == 1) rc = render_sharded(g, s, W, H, opt, d_image, timing);
  return rc;
}

// Lock every driven device (ascending order: no lock-order inversion between groups).
struct DeviceLocks {
  std::vector<std::unique_lock<std::mutex>> held;
  explicit DeviceLocks(rc_group& g) {
    std::set<int> devs;
    for (auto& rp : g.ranks) devs.insert(rp->device);
    for (int d : devs) held.emplace_back(g_ctx[d].mu);
  }
};

}  // namespace

namespace rcrt {

// rc_render's multi-GPU path: a cached in-process group over devices first..first+n-1 (RCCL),
// or n ranks on device `first` (share: device copies, rc_tuning.share_device).
int render_local_group(int first, int n, bool share, const rc_scene* s, int W, int H,
                       const rc_options* opt, uint8_t** d_image, rc_timing* timing) {
  static std::mutex mu;
  static rc_group* cached = nullptr;
  static int c_first = -1, c_n = 0;
  static bool c_share = false;
  std::lock_guard<std::mutex> lk(mu);
  if (!cached || c_first != first || c_n != n || c_share != share) {
    if (cached) rc_group_destroy(cached);
    cached = nullptr;
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = share ? first : first + i;
    cached = rc_group_create_local(n, devs.data(), share ? RC_XFER_COPY : RC_XFER_AUTO);
    if (!cached) return -1;
    c_first = first;
    c_n = n;
    c_share = share;
  }
  DeviceLocks locks(*cached);
  if (render_sharded_retry(*cached, s, W, H, opt, nullptr, timing)) return -1;
  *d_image = (uint8_t*)cached->root->image.p;
  return 0;
}

}  // namespace rcrt

extern "C" {

int rc_group_unique_id(unsigned char id[RC_GROUP_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == RC_GROUP_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof u);
  return 0;
}

rc_group* rc_group_create_rank(int nranks, int rank, const unsigned char id[RC_GROUP_ID_BYTES],
                               int device) {
  if (nranks < 1 || nranks > rc::kMaxShards || rank < 0 || rank >= nranks || !id) return nullptr;
  auto g = std::make_unique<rc_group>();
  g->nranks = nranks;
  g->transport = RC_XFER_RCCL;
  auto r = std::make_unique<Rank>();
  if (init_rank(*r, rank, device)) return nullptr;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  if (ncclCommInitRank(&r->comm, nranks, u, rank) != ncclSuccess) {
    std::fprintf(stderr, "Error: ncclCommInitRank failed (rank %d of %d)\n", rank, nranks);
    release_rank(*r);
    return nullptr;
  }
  if (rank == 0) g->root = r.get();
  g->ranks.push_back(std::move(r));
  return g.release();
}

rc_group* rc_group_create_local(int nranks, const int* devices, int transport) {
  if (nranks < 1 || nranks > rc::kMaxShards || !devices) return nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return nullptr;
  std::set<int> distinct;
  for (int i = 0; i < nranks; ++i) {
    if (devices[i] < 0 || devices[i] >= ndev) {
      std::fprintf(stderr, "Error: device %d not available (%d devices)\n", devices[i], ndev);
      return nullptr;
    }
    distinct.insert(devices[i]);
  }
  if (transport == RC_XFER_AUTO)
    transport = (int)distinct.size() == nranks ? RC_XFER_RCCL : RC_XFER_COPY;
  if (transport == RC_XFER_RCCL && (int)distinct.size() != nranks) {
    std::fprintf(stderr, "Error: RCCL ranks need distinct devices (use RC_XFER_COPY)\n");
    return nullptr;
  }
  auto g = std::make_unique<rc_group>();
  g->nranks = nranks;
  g->transport = transport;
  for (int i = 0; i < nranks; ++i) {
    auto r = std::make_unique<Rank>();
    if (init_rank(*r, i, devices[i])) return nullptr;
    g->ranks.push_back(std::move(r));
  }
  g->root = g->ranks[0].get();
  if (transport == RC_XFER_RCCL) {
    std::vector<ncclComm_t> comms(nranks);
    if (ncclCommInitAll(comms.data(), nranks, devices) != ncclSuccess) {
      std::fprintf(stderr, "Error: ncclCommInitAll failed (%d devices)\n", nranks);
      for (auto& rp : g->ranks) release_rank(*rp);
      return nullptr;
    }
    for (int i = 0; i < nranks; ++i) g->ranks[i]->comm = comms[i];
  }
  return g.release();
}

void rc_group_destroy(rc_group* g) {
  if (!g) return;
  for (auto& rp : g->ranks) release_rank(*rp);
  delete g;
}

int rc_group_size(const rc_group* g) { return g ? g->nranks : 0; }

int rc_group_transport(const rc_group* g) { return g ? g->transport : -1; }

int rc_render_sharded(rc_group* g, const rc_scene* s, int W, int H, const rc_options* opt,
                      uint8_t* d_image, rc_timing* timing) {
  if (!g || !s || !opt || W <= 0 || H <= 0) return -1;
  if ((long long)W * H >= (1ll << 31)) return -1;   // DEP indices and wire pixels are 32-bit
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  int rc;
  {
    DeviceLocks locks(*g);
    rc = render_sharded_retry(*g, s, W, H, opt, d_image, timing);
  }
  (void)hipSetDevice(dev);
  return rc;
}

// Applies to the ranks this process drives: in a multi-process group every rank must make the
// same call before the same frame (the bound selects the exchange's collectives).
int rc_group_debug_bound(rc_group* g, long long per_rank) {
  if (!g || per_rank < -1) return -1;
  g->bound.per_rank = per_rank;
  return 0;
}

int rc_group_last_stats(const rc_group* g, rc_shard_stats* out) {
  if (!g || !out) return -1;
  *out = g->last;
  return 0;
}

int rc_group_rank_stats(const rc_group* g, int rank, rc_rank_stats* out) {
  if (!g || !out) return -1;
  for (auto& rp : g->ranks)
    if (rp->rank == rank) {
      *out = rp->last;
      return 0;
    }
  return -1;   // this process does not drive that rank
}

}  // extern "C"
