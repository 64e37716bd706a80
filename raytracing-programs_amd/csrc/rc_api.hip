// rc_api.hip — host runtime and C-ABI of libraycast_hip.so (declared in include/raycast_hip.h).
//
// raycast() is the drop-in for C/raycast.c:79-130: it flattens the lists (rc_scene.c),
// consumes them like the reference (C/raycast.c:104-107), renders on the GPU(s) and writes
// photo_data.pixmap.  Per-device state (stream, events, grow-only workspaces) is created on
// first use and kept for the life of the process, so repeated renders allocate nothing.
//
// Multi-GPU (RAYCAST_GPUS=N, both modes): row shards over RCCL, rc_shard.hip.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "raycast_hip.h"
#include "rc_kernels.h"
#include "rc_runtime.h"
#include "rc_scene.h"

#define RC_VERSION "raycast-mi355x 0.1 (gfx950)"

namespace rcrt {

DevCtx g_ctx[kMaxDevices];
std::mutex g_ctx_mu;

rc_tuning default_tuning() {
  rc_tuning t;
  t.side = 3;
  t.split_shade = 0;
  t.resolve_shared = 0;
  t.resolve_lds_kb = 0;
  t.resolve_grid = 0;
  t.team_blocks = -1;
  t.helpers = 16;    // round 4: 8 -> 16 with hand_run 512 -> 128 (lone quadric 4096^2 5.01 ->
  t.hand_run = 128;  // 4.65-4.77 ms, 8192^2 13.1 -> 12.3 ms; profiles/r04j_helpers_*.txt)
  t.long_len = 32768;
  t.wave_k = 2;
  t.resolve_k = 1;
  t.coop = 1;
  t.dep_fast = 1;
  t.o0 = 1;
  t.phase_c_finish = 0;
  t.single_res_cus = 0;
  t.pipe_res_cus = 0;
  t.pipe_resolvers = 2;
  t.pipe_slots = 4;
  t.pipe_timing = 1;
  t.pipe_slotstreams = 0;
  t.overlap_d2h = 1;
  t.staged_d2h = 1;
  t.prefault = 1;
  t.copy_threads = 8;
  t.side_blocks = 0;
  t.comp_stream = 2;
  t.pipe_inres = 0;
  t.x0 = 1;
  t.resolve_clean = 1;
  t.shard_lone = 1;
  t.team_cscan = 1;
  t.pipe_order = 0;
  t.pipe_helpers = 4;   // round 4: frames in flight 6.70-6.81e9 -> 6.83-6.90e9 at C4, C5 / C3 /
                        // simple 1024^2 +0.8 / +1.2 / +2.3 % (profiles/r04q_pipe_helpers_*.txt)
  t.patch_host = 2;   // round 4: rc_render end to end 5.39-5.47 (0) -> 5.29-5.33 (1) -> 5.02-5.07 ms
                      // (profiles/r04v_patch_ab.txt, r04z_e2e_anatomy.txt)
  // regular segments of >= 3000 entries on whole workgroups when there are workgroups for all
  // of them (k_seg_order): lone quadric 4096^2 5.19 -> 5.06 ms (its ~100 3856-entry segments
  // 4.4 -> 2.5 ms, under the team segment); 8192^2 and pipeline lanes have more such segments
  // than workgroups and keep one wave per segment
  t.block_min = 3000;
  t.share_device = 0;
  // round 5: 24 of the lone resolver's regular workgroups start on the per-wave queue at once,
  // so the dense runs reach the helpers ~0.5 ms earlier and the team segment alone bounds the
  // resolver (lone quadric 4096^2 4.66 -> 4.55-4.56 ms; profiles/r05e_lone_headb.txt)
  t.headb_first = 24;
  t.pipe_last_whole = 1;
  return t;
}
rc_tuning g_tune = default_tuning();
std::mutex g_tune_mu;   // rc_set_tuning writes g_tune while render threads read it
rc_tuning tune() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  return g_tune;
}
double g_last_kernel_ms = 0.0;
std::atomic<int> g_pool_threads{-1};   // copy_threads the host pool was built with (-1: not yet)
// rc_debug_inject_error: the parity frame (counted from the call, any path) whose resolver
// raises its error word; -1 = off
std::atomic<int> g_inject{-1};
int take_inject() {
  int v = g_inject.load();
  while (v >= 0 && !g_inject.compare_exchange_weak(v, v - 1)) {
  }
  return v == 0 ? 1 : 0;
}

const char* spin_site(int code) {
  static const char* site[] = {"", "team granule", "phase-C carry-in", "helper queue",
                               "injected (rc_debug_inject_error)"};
  return code >= 1 && code <= 4 ? site[code] : "?";
}

int FrameLog::enqueue(const void* team, hipStream_t st) {
  if (!ring) {
    HIP_TRY(hipHostMalloc((void**)&ring, kRing * sizeof(Entry), hipHostMallocDefault));
    for (int i = 0; i < kRing; ++i) ring[i].code = kPending;
  }
  if (head - tail >= kRing) {   // every entry still unread: wait for the frames, read them
    HIP_TRY(hipDeviceSynchronize());
    if (drain() < 0) return -1;
  }
  Entry* e = &ring[head % kRing];
  ((volatile Entry*)e)->code = kPending;
  HIP_TRY(hipMemcpyAsync(e, team, sizeof(Entry), hipMemcpyDeviceToHost, st));
  ++head;
  return 0;
}

long long FrameLog::poll() {
  long long found = 0;
  while (tail < head) {
    volatile Entry* e = &ring[tail % kRing];
    const int code = e->code;
    if (code == kPending) break;
    if (code != 0) {
      ++found;
      std::fprintf(stderr,
                   "Error: parity frame %lld (%s) is invalid: its hand-off failed (code %d: %s) "
                   "at workgroup %d, detail %d/%d\n",
                   tail, what, code, spin_site(code), e->block, e->info, e->info2);
    }
    ++diag.frames;
    diag.scan_max = e->n_scan > diag.scan_max ? e->n_scan : diag.scan_max;
    diag.cscan_max = e->n_cscan > diag.cscan_max ? e->n_cscan : diag.cscan_max;
    diag.resolve_max = e->n_resolve > diag.resolve_max ? e->n_resolve : diag.resolve_max;
    for (int q = 0; q < 4; ++q)
      if (e->spin_ticks[q] > diag.spin_ticks_max[q]) diag.spin_ticks_max[q] = e->spin_ticks[q];
    if (e->clock_mhz > 0) {
      if (diag.clock_min == 0 || e->clock_mhz < diag.clock_min) diag.clock_min = e->clock_mhz;
      if (e->clock_mhz > diag.clock_max) diag.clock_max = e->clock_mhz;
    }
    e->code = kPending;
    ++tail;
    ++checked;
  }
  failed += found;
  return found;
}

long long FrameLog::drain() {
  long long found = poll();
  if (tail < head) {
    std::fprintf(stderr, "Error: %lld parity frame(s) (%s) were never verified (their hand-off "
                 "words did not arrive after a synchronisation)\n", head - tail, what);
    found += head - tail;
    failed += head - tail;
    checked += head - tail;
    tail = head;
  }
  return found;
}

bool FrameLog::earlier_failed() {
  poll();
  return failed > 0;
}

bool FrameLog::entry_failed(long long k) const {
  if (!ring || k < tail || k >= head) return false;   // not logged, or already read back
  const int code = ((volatile const Entry*)&ring[k % kRing])->code;
  return code != 0 && code != kPending;
}

void FrameLog::take(long long* c, long long* f) {
  if (c) *c = checked;
  if (f) *f = failed;
  checked = failed = 0;
}

// rc_resolver_stats: the placement and resources part, and a window's frame diagnostics
int fill_resolver_stats(DevCtx& c, const FrameLog::Diag& d, int grid, int res_cus, int lds,
                        int team, rc_resolver_stats* r) {
  r->grid = grid;
  r->res_cus = res_cus;
  r->wg_per_cu = res_cus > 0 ? (grid + res_cus - 1) / res_cus : 0;
  r->lds_bytes = lds;
  r->team_blocks = team;
  int regs = 0, scratch = 0, per_cu = 0;
  if (rc::resolve_resources(lds > 0 ? lds : 0, &regs, &scratch, &per_cu) == 0) {
    r->regs = regs;
    r->scratch_bytes = scratch;
    r->wg_per_cu_max = per_cu;
  }
  r->scan_rounds_max = d.scan_max;
  r->cscan_rounds_max = d.cscan_max;
  r->resolve_rounds_max = d.resolve_max;
  for (int q = 0; q < 4; ++q) r->spin_wait_us_max[q] = d.spin_ticks_max[q] * 0.01;
  r->clock_mhz_min = d.clock_min;
  r->clock_mhz_max = d.clock_max;
  (void)c;
  return 0;
}

int ctx_get(int device, DevCtx** out) {
  if (device < 0 || device >= kMaxDevices) return -1;
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  DevCtx& c = g_ctx[device];
  if (!c.init) {
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    c.cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    for (auto& set : c.ev)
      for (auto& e : set) HIP_TRY(hipEventCreate(&e));
    if (c.fb.zcount.ensure(64)) return -1;
    HIP_TRY(hipEventCreateWithFlags(&c.ws_ev, hipEventDisableTiming));
    c.lone_log.what = "one frame at a time";
    c.pipe.log.what = "frames in flight";
    c.device = device;
    c.init = true;
  }
  *out = &c;
  return 0;
}

// ------------------------------------------------------------- device -> host copy --
// The drop-in path ends with the image in the caller's pageable pixmap (C/raycast.c:52-53
// mallocs it).  The runtime's own pageable copy stages through a bounce buffer and fills the
// destination from one host thread (~3.2 ms for 4096^2 RGB).  copy_to_host streams 8 MiB
// chunks into two pinned bounce buffers (DMA of chunk i+1 while chunk i is spread over host
// threads) and copies each chunk out with a small persistent thread pool.
constexpr size_t kStageChunk = 8u << 20;

// One pool per device: the in-frame scatter (scatter_progressive) keeps a device's pool busy
// for most of its frame, and rc_render callers on other devices must not wait for that.
class HostPool {
 public:
  static HostPool& get(int device) {   // never destroyed: its detached workers outlive main()
    static std::mutex mu;
    static HostPool* pools[kMaxDevices] = {};
    const int d = device >= 0 && device < kMaxDevices ? device : 0;
    std::lock_guard<std::mutex> lk(mu);
    if (!pools[d]) pools[d] = new HostPool();
    return *pools[d];
  }
  int parts() const { return nthreads_ + 1; }
  // fn(part, parts) on the workers and the calling thread (part 0), one call at a time (the
  // device's callers already hold its lock; this also orders calls that do not)
  void run(const std::function<void(int, int)>& fn) {
    std::lock_guard<std::mutex> one_at_a_time(call_mu_);
    {
      std::unique_lock<std::mutex> lk(mu_);
      fn_ = &fn;
      pending_ = nthreads_;
      ++gen_;
    }
    cv_.notify_all();
    fn(0, nthreads_ + 1);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
  }
  // memcpy(dst, src, n) split over the pool
  void copy(uint8_t* dst, const uint8_t* src, size_t n) {
    const size_t step = ((n + parts() - 1) / parts() + 4095) & ~(size_t)4095;
    run([&](int part, int) {
      const size_t off = (size_t)part * step;
      if (off < n) std::memcpy(dst + off, src + off, n - off < step ? n - off : step);
    });
  }

 private:
  HostPool() {
    // every device's pool has the size the first one was built with (rc_set_tuning warns)
    int want = g_pool_threads.load();
    if (want < 0) {
      want = tune().copy_threads;
      int expect = -1;
      if (!g_pool_threads.compare_exchange_strong(expect, want)) want = expect;
    }
    int t = want - 1;
    if (t < 0) t = 0;
    if (t > 31) t = 31;
    nthreads_ = t;
    for (int i = 0; i < t; ++i) workers_.emplace_back([this, i] { work(i + 1); });
    for (auto& w : workers_) w.detach();   // lives for the process
  }
  void work(int part) {
    unsigned long long seen = 0;
    for (;;) {
      const std::function<void(int, int)>* fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        fn = fn_;
      }
      (*fn)(part, nthreads_ + 1);
      std::unique_lock<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  int nthreads_ = 0;
  unsigned long long gen_ = 0;
  int pending_ = 0;
  const std::function<void(int, int)>* fn_ = nullptr;
};

int copy_to_host(DevCtx& c, uint8_t* host, const uint8_t* dev, size_t bytes, hipStream_t st,
                 const rc_tuning& tu) {
  if (!tu.staged_d2h) {   // the runtime's pageable copy
    HIP_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  for (int b = 0; b < 2; ++b) {
    if (!c.stage[b]) {
      HIP_TRY(hipHostMalloc((void**)&c.stage[b], kStageChunk, hipHostMallocDefault));
      HIP_TRY(hipEventCreateWithFlags(&c.stage_ev[b], hipEventDisableTiming));
    }
  }
  const size_t n = (bytes + kStageChunk - 1) / kStageChunk;
  auto chunk = [&](size_t i) { return i + 1 < n ? kStageChunk : bytes - i * kStageChunk; };
  for (size_t i = 0; i < 2 && i < n; ++i) {
    HIP_TRY(hipMemcpyAsync(c.stage[i], dev + i * kStageChunk, chunk(i), hipMemcpyDeviceToHost,
                           st));
    HIP_TRY(hipEventRecord(c.stage_ev[i], st));
  }
  for (size_t i = 0; i < n; ++i) {
    const int b = (int)(i & 1);
    HIP_TRY(hipEventSynchronize(c.stage_ev[b]));
    HostPool::get(c.device).copy(host + i * kStageChunk, c.stage[b], chunk(i));
    if (i + 2 < n) {
      HIP_TRY(hipMemcpyAsync(c.stage[b], dev + (i + 2) * kStageChunk, chunk(i + 2),
                             hipMemcpyDeviceToHost, st));
      HIP_TRY(hipEventRecord(c.stage_ev[b], st));
    }
  }
  return 0;
}

// Fault the caller's fresh pixmap in (C/raycast.c:52-53 mallocs it) over the host pool while the
// GPU renders, instead of inside the copy (every byte is overwritten afterwards).
void prefault(DevCtx& c, uint8_t* p, size_t n, const rc_tuning& tu) {
  if (!n || !tu.prefault) return;
  HostPool::get(c.device).run([&](int part, int parts) {
    const size_t per = ((n + parts - 1) / parts + 4095) & ~(size_t)4095;
    const size_t a = (size_t)part * per, b = a + per < n ? a + per : n;
    volatile uint8_t* q = p;
    for (size_t o = a; o < b; o += 4096) q[o] = 0;
    if (a < b) q[b - 1] = 0;
  });
}

int ensure_pinned(DevCtx& c, size_t entries) {
  if (!c.pin_cnt) HIP_TRY(hipHostMalloc((void**)&c.pin_cnt, 64, hipHostMallocDefault));
  if (entries <= c.pin_bytes) return 0;
  if (c.pin_pix) (void)hipHostFree(c.pin_pix);
  if (c.pin_patch) (void)hipHostFree(c.pin_patch);
  c.pin_pix = c.pin_patch = nullptr;
  c.pin_bytes = 0;
  HIP_TRY(hipHostMalloc((void**)&c.pin_pix, entries * sizeof(long long), hipHostMallocDefault));
  HIP_TRY(hipHostMalloc((void**)&c.pin_patch, entries * sizeof(uint32_t), hipHostMallocDefault));
  c.pin_bytes = entries;
  return 0;
}

// patch_host: the DEP entries' packed colours go straight to pinned, mapped host memory from
// phase C's stores (a batch of 64 entries is one 256-byte write), during the resolver, instead
// of an 11 MB copy (quadric 4096^2) after the frame's last kernel.  Each entry carries its
// frame's mark (rc::patch_mark of the frame's epoch) and the host never stores to the array
// while a frame runs: a frame's entries are known by the mark alone.  Marks repeat every
// rc::kPatchMarks epochs, so before a frame of epoch `epoch` is enqueued the array's possibly
// marked entries (host_patch_dirty) are cleared once `epoch` is that far past the last clear.
// rc_render raises host_patch_dirty to the whole image before it enqueues a frame that writes
// the array and lowers it to the largest DEP count since the clear once the frame's own is
// known.
int ensure_host_patch(DevCtx& c, size_t entries, unsigned epoch) {
  if (entries <= c.host_patch_entries) {
    if (c.host_patch_dirty &&
        (epoch <= c.host_patch_epoch0 || epoch - c.host_patch_epoch0 >= rc::kPatchMarks)) {
      std::memset(c.host_patch, 0, c.host_patch_dirty * sizeof(uint32_t));
      c.host_patch_dirty = 0;
    }
    if (!c.host_patch_dirty) c.host_patch_epoch0 = epoch - 1;   // nothing marked
    return 0;
  }
  if (c.host_patch) (void)hipHostFree(c.host_patch);
  c.host_patch = c.host_patch_dev = nullptr;
  c.host_patch_entries = 0;
  HIP_TRY(hipHostMalloc((void**)&c.host_patch, entries * sizeof(uint32_t),
                        hipHostMallocMapped | hipHostMallocCoherent));
  void* d = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&d, c.host_patch, 0));
  c.host_patch_dev = (uint32_t*)d;
  c.host_patch_entries = entries;
  std::memset(c.host_patch, 0, entries * sizeof(uint32_t));
  c.host_patch_dirty = 0;
  c.host_patch_epoch0 = epoch - 1;
  return 0;
}

// The scatter of a mapped colour patch while the frame still runs (patch_host): each host
// thread sweeps its share of the DEP list and scatters every entry phase C has marked, until
// its share is done; once the frame's last kernel has completed (ev_done), one more sweep takes
// everything left.  The framebuffer copy must already be in `host` (it carries the DEP pixels'
// phase-A bytes, which the patch overwrites).  The array is only read: an entry is this
// frame's once its top byte is `mark`.
// Entries go in blocks of kScatterBlock (phase C's batch, one 256-byte store), each with a
// cursor at its first unconsumed entry; a sweep before the frame's end moves on to the next
// block at the first entry not yet marked, so it costs about one read per pending block rather
// than one per entry left.  Blocks go in chunks a thread locks while it sweeps them.  A thread
// sweeps its own band of chunks (contiguous, so its pixels are a band of rows: spreading every
// thread over the whole image made the scatter ~5x slower per entry, TLB and cache misses on
// the caller's pixmap, profiles/r06n_scatter_diag.txt) and, once its band is done, helps with
// the others' (frames of kScatterHelpMin entries or more).  A sweep that found nothing yields; the event is queried by one thread at a
// time, at most once per kScatterQueryNs (every thread querying after each short sweep
// contends in the runtime); any status other than "not ready" ends every thread's sweeps (the
// frame failed: returns -1, the caller reports it).
constexpr size_t kScatterBlock = 64;
constexpr size_t kScatterChunk = 32;   // blocks per chunk: the unit a thread locks (2048 entries)
constexpr long long kScatterQueryNs = 20000;
// below this many entries a thread sweeps its own band only: helping costs ~1 % end to end on
// frames whose scatter is short (reflection 2048^2 d4, 0.29 M entries; simple 1024^2 d6) and
// saves 0.04-0.1 ms at quadric 4096^2 (2.8 M; profiles/r06y_scatter_help_ab.txt)
constexpr size_t kScatterHelpMin = (size_t)1 << 20;

// The sweep itself, on `pool`, with the frame's end as `probe()` (1 complete, 0 not yet, a
// negative value a failure, returned as is); rc_debug_scatter_selftest drives it without a GPU.
template <class Probe>
int scatter_sweep(HostPool& pool, uint8_t* host, const long long* pix, const uint32_t* patch,
                  size_t ndep, uint32_t mark, Probe probe) {
  std::atomic<bool> over{false};
  std::atomic<int> status{0};
  std::atomic<long long> next_query{0};
  const auto t0 = std::chrono::steady_clock::now();
  const size_t nblk = (ndep + kScatterBlock - 1) / kScatterBlock;
  const size_t nch = (nblk + kScatterChunk - 1) / kScatterChunk;
  // per block: entries consumed from its start; per chunk: 0 free, 1 held by a thread, 2 done
  // (a chunk's cursors are read and written only by the thread holding it)
  std::vector<uint8_t> cur(nblk, 0);
  std::unique_ptr<std::atomic<int>[]> state(new std::atomic<int>[nch]);
  for (size_t k = 0; k < nch; ++k) state[k].store(0, std::memory_order_relaxed);
  const bool help = ndep >= kScatterHelpMin;
  pool.run([&](int part, int parts) {
    const size_t per = (nch + parts - 1) / parts;
    const size_t h0 = std::min((size_t)part * per, nch), h1 = std::min(h0 + per, nch);
    const size_t span = help ? nch : h1 - h0;
    // one chunk's ready entries; true once every entry is consumed (after the frame's end,
    // `last`, an unmarked entry is passed over: it stays unmarked)
    auto sweep = [&](size_t k, bool last, size_t& got) {
      bool done = true;
      const size_t bend = std::min((k + 1) * kScatterChunk, nblk);
      for (size_t bl = k * kScatterChunk; bl < bend; ++bl) {
        const size_t base = bl * kScatterBlock, end = std::min(base + kScatterBlock, ndep);
        size_t j = base + cur[bl];
        for (; j < end; ++j) {
          const uint32_t v = *(const volatile uint32_t*)(patch + j);
          if ((v & 0xFF000000u) != mark) {
            if (last) continue;
            break;
          }
          uint8_t* q = host + 3 * (size_t)pix[j];
          q[0] = (uint8_t)v;
          q[1] = (uint8_t)(v >> 8);
          q[2] = (uint8_t)(v >> 16);
          ++got;
        }
        cur[bl] = (uint8_t)(j - base);
        if (j < end) done = false;
      }
      return done;
    };
    for (;;) {
      const bool last = over.load(std::memory_order_acquire);
      if (status.load(std::memory_order_relaxed) != 0) return;
      size_t got = 0;
      bool home_left = false, any_left = false;
      // the thread's own chunks first (a band of rows: the caller's pixmap stays local); once
      // they are all done, every other chunk not held by another thread, from the next
      // thread's band on — the frame's last entries (the longest chains') sit in one or two
      // bands, and every idle thread shares them
      for (size_t i = 0; i < span; ++i) {
        const size_t k = (h0 + i) % nch;
        const bool home = k >= h0 && k < h1;
        if (!home && home_left && !last) break;
        int st = state[k].load(std::memory_order_acquire);
        if (st == 2) continue;
        any_left = true;
        if (home) home_left = true;
        if (st != 0 || !state[k].compare_exchange_strong(st, 1, std::memory_order_acquire))
          continue;
        const bool done = sweep(k, last, got);
        state[k].store(done ? 2 : 0, std::memory_order_release);
      }
      if (!any_left) return;
      if (got || last) {
        if (last) std::this_thread::yield();   // chunks another thread still holds
        continue;
      }
      const long long now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now() - t0).count();
      long long due = next_query.load(std::memory_order_relaxed);
      if (now < due || !next_query.compare_exchange_strong(due, now + kScatterQueryNs)) {
        std::this_thread::yield();
        continue;
      }
      const int q = probe();
      if (q == 1) {
        over.store(true, std::memory_order_release);
      } else if (q != 0) {
        status.store(q, std::memory_order_relaxed);
        return;
      } else {
        std::this_thread::yield();
      }
    }
  });
  return status.load();
}

int scatter_progressive(DevCtx& c, uint8_t* host, const long long* pix, const uint32_t* patch,
                        size_t ndep, uint32_t mark, hipEvent_t ev_done) {
  const int st = scatter_sweep(HostPool::get(c.device), host, pix, patch, ndep, mark, [&] {
    const hipError_t q = hipEventQuery(ev_done);
    return q == hipSuccess ? 1 : q == hipErrorNotReady ? 0 : -(int)q;
  });
  // a query's hipErrorNotReady is not a failure: clear it from this thread's last error (the
  // pool's threads keep theirs; nothing reads them)
  (void)hipGetLastError();
  if (st != 0) {
    std::fprintf(stderr, "Error: HIP call failed: hipEventQuery (%s) during the in-frame scatter\n",
                 hipGetErrorString((hipError_t)(-st)));
    return -1;
  }
  return 0;
}

// RC_E2E_TRACE=1: rc_render prints its host-side marks (ms from entry) to stderr, to split the
// end-to-end time into the enqueue, the wait for the device frame and what follows it.
struct E2eTrace {
  static bool on() {
    static const bool v = std::getenv("RC_E2E_TRACE") != nullptr;
    return v;
  }
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double at[8] = {};
  void mark(int i) {
    if (on()) at[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  void print() const {
    if (on())
      std::fprintf(stderr,
                   "rc_e2e: enqueued %.3f prefaulted %.3f phaseA+compact %.3f copy %.3f frame %.3f "
                   "scatter %.3f synced %.3f end %.3f\n",
                   at[0], at[1], at[2], at[3], at[4], at[5], at[6], at[7]);
  }
};
// set for the duration of one traced rc_render, on its own thread (renders on other devices
// run concurrently)
thread_local E2eTrace* g_e2e = nullptr;

// The parity render's device-to-host copy, overlapped with the render (the
// drop-in rate spans upload + kernels + copy).  Once phase A and the compaction are done
// (ev[2]), every pixel except the DEP pixels is final: the framebuffer streams out on the copy
// stream while the carry resolver runs, together with the DEP list (pixel per entry).  After
// phase C (ev[4]) only the DEP entries' packed colours follow (4 B per entry, ~17 % of the
// pixels), and the host pool scatters them over the copy — or, with patch_host, phase C wrote
// them into mapped host memory and the pool scatters each as it arrives (scatter_progressive),
// so only the frame's last entries are left once it ends.
// host_patch: the mapped array phase C writes (patch_host 1 or 2, tu.patch_host says which),
// its entries marked with rc::patch_mark of this frame's epoch (c.fb.epoch); prev_dirty: its
// entries marked since the last clear before this frame (rc_render has raised host_patch_dirty
// to the whole image for this frame; it drops to the bound of both here).
int copy_overlapped(DevCtx& c, uint8_t* host, const uint8_t* dev, size_t bytes,
                    const hipEvent_t* ev, uint32_t* host_patch, size_t prev_dirty,
                    const rc_tuning& tu) {
  if (ensure_pinned(c, 0)) return -1;
  HIP_TRY(hipEventSynchronize(ev[2]));
  if (g_e2e) g_e2e->mark(2);
  HIP_TRY(hipMemcpyAsync(c.pin_cnt, c.fb.counters.p, 4 * sizeof(int), hipMemcpyDeviceToHost,
                         c.d2h));
  HIP_TRY(hipStreamSynchronize(c.d2h));
  const size_t ndep = (size_t)c.pin_cnt[2];
  // the frame writes (and marks) only entries below its DEP count
  if (host_patch) c.host_patch_dirty = std::max(prev_dirty, ndep);
  const uint32_t mark = rc::patch_mark(c.fb.epoch);
  if (ensure_pinned(c, ndep)) return -1;
  if (ndep)
    HIP_TRY(hipMemcpyAsync(c.pin_pix, c.fb.dep_pix.p, ndep * sizeof(long long),
                           hipMemcpyDeviceToHost, c.d2h));
  if (copy_to_host(c, host, dev, bytes, c.d2h, tu)) return -1;
  if (g_e2e) g_e2e->mark(3);
  if (host_patch && ndep && tu.patch_host == 2) {   // consumed as it arrives
    HIP_TRY(hipStreamSynchronize(c.d2h));   // the DEP list's copy
    if (scatter_progressive(c, host, (const long long*)c.pin_pix, host_patch, ndep, mark,
                            ev[4]))
      return -1;
    HIP_TRY(hipEventSynchronize(ev[4]));
    if (g_e2e) {
      g_e2e->mark(4);
      g_e2e->mark(5);
    }
    return 0;
  }
  HIP_TRY(hipEventSynchronize(ev[4]));
  if (g_e2e) g_e2e->mark(4);
  if (!ndep) return 0;
  const uint32_t* rgb = host_patch;   // written by phase C itself (patch_host 1)
  if (rgb) {
    HIP_TRY(hipStreamSynchronize(c.d2h));   // the DEP list's copy
  } else {
    HIP_TRY(hipMemcpyAsync(c.pin_patch, c.patch.p, ndep * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, c.d2h));
    HIP_TRY(hipStreamSynchronize(c.d2h));
    rgb = (const uint32_t*)c.pin_patch;
  }
  const long long* pix = (const long long*)c.pin_pix;
  HostPool::get(c.device).run([&](int part, int parts) {
    const size_t per = (ndep + parts - 1) / parts;
    const size_t a = (size_t)part * per, b = a + per < ndep ? a + per : ndep;
    for (size_t j = a; j < b; ++j) {
      uint8_t* q = host + 3 * (size_t)pix[j];
      const uint32_t v = rgb[j];
      q[0] = (uint8_t)v;
      q[1] = (uint8_t)(v >> 8);
      q[2] = (uint8_t)(v >> 16);
    }
  });
  if (g_e2e) g_e2e->mark(5);
  return 0;
}

}  // namespace rcrt

using namespace rcrt;


extern "C" {

const char* rc_version(void) { return RC_VERSION; }

void rc_default_tuning(rc_tuning* t) {
  if (t) *t = default_tuning();
}

void rc_get_tuning(rc_tuning* t) {
  if (t) *t = tune();
}

int rc_set_tuning(const rc_tuning* t) {
  if (!t) return -1;
  auto in = [](int v, int lo, int hi) { return v >= lo && v <= hi; };
  const bool ok =
      in(t->side, 0, 4) && in(t->split_shade, 0, 1) && in(t->resolve_shared, 0, 1) &&
      in(t->resolve_lds_kb, 0, 152) && (t->resolve_grid == 0 || in(t->resolve_grid, 8, 1 << 16)) &&
      in(t->team_blocks, -1, 256) && in(t->helpers, 0, rc::kDenseSlots) &&
      in(t->hand_run, 1, 1 << 30) && in(t->long_len, 64, 1 << 30) && in(t->wave_k, 1, 64) &&
      in(t->resolve_k, 1, 64) && in(t->coop, 0, 1) && in(t->dep_fast, 0, 1) && in(t->o0, 0, 1) &&
      in(t->phase_c_finish, 0, 1) && in(t->single_res_cus, 0, 1 << 16) &&
      in(t->pipe_res_cus, 0, 1 << 16) && in(t->pipe_resolvers, 1, 4) && in(t->pipe_slots, 1, 8) &&
      in(t->pipe_timing, 0, 1) && in(t->pipe_slotstreams, 0, 1) && in(t->overlap_d2h, 0, 1) &&
      in(t->staged_d2h, 0, 1) && in(t->prefault, 0, 1) && in(t->copy_threads, 1, 32) &&
      in(t->comp_stream, 0, 2) && in(t->side_blocks, 0, 1 << 16) &&
      in(t->block_min, 0, 1 << 30) && in(t->pipe_inres, 0, 2) && in(t->x0, 0, 1) &&
      in(t->resolve_clean, 1, 64) && in(t->shard_lone, 0, 1) && in(t->team_cscan, 0, 1) &&
      in(t->pipe_order, 0, 4) && in(t->pipe_helpers, 0, rc::kDenseSlots) &&
      in(t->patch_host, 0, 2) && in(t->share_device, 0, 1) && in(t->headb_first, 0, 1 << 16) && in(t->pipe_last_whole, 0, 1) &&
      !(t->split_shade && !t->side);
  if (!ok) {
    std::fprintf(stderr, "Error: rc_set_tuning: a field is out of range\n");
    return -1;
  }
  // fields read once: the host pool's size at its first use, the frame pipeline's layout at
  // its build (rc_pipe_reset rebuilds it)
  const int pool = g_pool_threads.load();
  if (pool >= 0 && t->copy_threads != pool)
    std::fprintf(stderr, "Warning: rc_set_tuning: copy_threads is fixed at the host pool's "
                 "first use (%d threads); the new value is ignored\n", pool);
  for (auto& c : g_ctx) {
    if (!c.pipe.init) continue;
    if (t->pipe_resolvers != c.pipe.built_lanes || t->pipe_slots != c.pipe.built_slots ||
        t->pipe_res_cus != c.pipe.built_res || (t->pipe_timing != 0) != c.pipe.rt_on ||
        (t->pipe_slotstreams == 0) != c.pipe.fifo || t->pipe_order != c.pipe.built_order) {
      std::fprintf(stderr, "Warning: rc_set_tuning: the pipe_* fields take effect when device "
                   "%d's frame pipeline is rebuilt (rc_pipe_reset)\n", c.device);
      break;
    }
  }
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tune = *t;
  return 0;
}

double rc_last_kernel_ms(void) { return g_last_kernel_ms; }

void rc_default_options(rc_options* opt, int use_env) {
  opt->max_recursion = 7;   // C/raycast.c:14
  opt->mode = RC_MODE_PARITY;
  opt->num_gpus = 1;
  opt->device = 0;
  if (!use_env) return;
  if (const char* m = std::getenv("RAYCAST_MODE")) {
    if (!std::strcmp(m, "fast")) opt->mode = RC_MODE_FAST;
    else if (!std::strcmp(m, "parity")) opt->mode = RC_MODE_PARITY;
    else if (!std::strcmp(m, "cuda")) opt->mode = RC_MODE_CUDA;
    else std::fprintf(stderr, "Warning: unknown RAYCAST_MODE '%s', using parity\n", m);
  }
  if (opt->mode == RC_MODE_CUDA) opt->max_recursion = 51;   // MAX_ITER 50 bounces
  if (const char* d = std::getenv("RAYCAST_DEPTH")) opt->max_recursion = std::atoi(d) + 1;
  if (const char* g = std::getenv("RAYCAST_GPUS")) opt->num_gpus = std::atoi(g);
  if (const char* v = std::getenv("RAYCAST_DEVICE")) opt->device = std::atoi(v);
  if (opt->num_gpus < 1) opt->num_gpus = 1;
}

rc_scene* rc_scene_create(const json_data_t* js) {
  if (!js) return nullptr;
  rc_packed_header* img = rc_pack_scene(js);
  if (!img) return nullptr;
  rc_scene* s = (rc_scene*)std::calloc(1, sizeof(rc_scene));
  if (!s) {
    std::free(img);
    return nullptr;
  }
  s->img = img;
  return s;
}

void rc_scene_destroy(rc_scene* s) {
  if (!s) return;
  // forget device copies that were uploaded from this image
  for (auto& c : g_ctx) {
    if (c.fb.scene_src == s->img) c.fb.scene_src = nullptr;
    for (auto& f : c.pipe.fb)
      if (f.scene_src == s->img) f.scene_src = nullptr;
  }
  std::free(s->img);
  std::free(s);
}

int rc_scene_parity_defined(const rc_scene* s) { return s ? s->img->phantom_defined : 0; }

}  // extern "C"

namespace rcrt {

int upload_scene(FrameBufs& b, hipStream_t stream, const rc_scene* s, rc::LaunchScene& ls) {
  const rc_packed_header* h = s->img;
  if (b.scene_src != h) {
    if (b.scene.ensure((size_t)h->bytes)) return -1;
    HIP_TRY(hipMemcpyAsync(b.scene.p, h, (size_t)h->bytes, hipMemcpyHostToDevice, stream));
    b.scene_src = h;
  }
  const char* base = (const char*)b.scene.p;
  ls.shapes = (const rc_shape*)(base + h->off_shapes);
  ls.lights = (const rc_light*)(base + h->off_lights);
  ls.pairs = (const rc_shade_pair*)(base + h->off_pairs);
  ls.n = h->n;
  ls.m = h->m;
  ls.cam_w = h->cam_w;
  ls.cam_h = h->cam_h;
  ls.refl_mask = 0;
  ls.has_quadric = 0;
  ls.o0_ok = h->o0_ok && tune().o0;
  const rc_shape* hs = (const rc_shape*)((const char*)h + h->off_shapes);
  for (int k = 0; k < h->n && k < 64; ++k)
    if (hs[k].refl > 0.0f) ls.refl_mask |= 1ull << k;
  bool cross = false;   // some quadric has cross terms (d, e, f)
  for (int k = 0; k < h->n; ++k)
    if (hs[k].type == RC_SHAPE_QUADRIC) {
      ls.has_quadric = 1;
      if (hs[k].qd != 0.0f || hs[k].qe != 0.0f || hs[k].qf != 0.0f) cross = true;
    }
  if (ls.has_quadric && !cross && tune().x0) ls.has_quadric = 2;   // rc_device.hpp quad_x0
  // Clean DEP entries' colour = phase A's primary shade exactly when every bounce level's
  // shade of them is zero: the phantom (shapes_list[-1], index n) is black, and the
  // reflectivity product T stays finite (0 * T == 0).
  ls.dep_fast = !(hs[h->n].opacity > 0.0f) && tune().dep_fast;
  for (int k = 0; k < h->n; ++k)
    if (!(std::fabs(hs[k].refl) < 1.0e5f)) ls.dep_fast = 0;
  return 0;
}

// The epoch of a workspace's next parity frame: tags keep bit 31 for a flag, so they wrap to 1
// (ensure_parity then clears the carry-ins once; a fresh buffer starts at tag 0, which no frame
// uses).
unsigned next_epoch(unsigned e) { return e + 1 >= 0x80000000u ? 1u : e + 1; }

// res_cus: CUs the resolver grid may occupy (all of them, or the pipeline's partition);
// piped: a pipeline lane (< 0: whenever res_cus is not the whole device).
int ensure_parity(DevCtx& c, FrameBufs& b, int W, int H, rc::ParityWork& w, int res_cus,
                  int piped_lane) {
  const size_t P = (size_t)W * H;
  if (b.cls.ensure(P) || b.wcarry.ensure(P * sizeof(float4)) ||
      b.deprec.ensure(P * rc::deprec_bytes()) ||
      b.rows.ensure((size_t)H * (rc::row_stats_bytes() + 2 * sizeof(int) +
                                 2 * sizeof(long long)) + 256) ||
      b.dep_pix.ensure(P * sizeof(long long)) || b.seg_key.ensure(P * sizeof(long long)) ||
      b.seg_start.ensure(P * sizeof(int)) ||
      b.seg_order.ensure((size_t)rc::kSegOrderMax * sizeof(int)) ||
      b.batch_state.ensure(3 * (P / 64 + 2) * sizeof(int)) ||
      b.counters.ensure(64) || b.team.ensure(rc::team_state_bytes()))
    return -1;
  if (P >= (size_t)1 << 31) return -1;   // DEP indices are 32-bit
  // carry-ins are tagged with a per-frame epoch: a fresh buffer starts at tag 0, which no
  // frame uses
  if (b.cin.bytes < P * rc::kCinBytes) {
    if (b.cin.ensure(P * rc::kCinBytes) || hipMemset(b.cin.p, 0, P * rc::kCinBytes) != hipSuccess)
      return -1;
  }
  b.epoch = next_epoch(b.epoch);
  if (b.epoch == 1 && hipMemset(b.cin.p, 0, b.cin.bytes) != hipSuccess) return -1;
  const bool piped = piped_lane >= 0 ? piped_lane != 0 : res_cus != c.cus;
  // Resolver placement by its dynamic LDS reservation: one workgroup (4 waves, one per SIMD)
  // per CU for a lone frame, whose critical path is its carry chains (and k_side must stay off
  // the resolver's CUs); two per CU for a pipeline lane, whose grid is small (64 CUs) — there
  // the longest segments outnumber one-per-CU's waves and the chains that start late set the
  // resolver's time (measured: 4.9e9 -> 5.4e9 rays/s with frames in flight, 6.37 -> 6.49 ms
  // for a lone frame).
  const rc_tuning tu = tune();
  const int one_per_cu = tu.resolve_shared ? 0 : 1;
  int lds = !one_per_cu ? 0 : piped ? 56 * 1024 : 96 * 1024;
  if (tu.resolve_lds_kb > 0) lds = tu.resolve_lds_kb * 1024;
  int slot = 0;
  while (slot < DevCtx::kResCache && c.res_lds[slot] != lds && c.res_blocks[slot]) ++slot;
  if (slot == DevCtx::kResCache) slot = 0;
  if (!c.res_blocks[slot] || c.res_lds[slot] != lds) {
    c.res_blocks[slot] = rc::resolve_blocks_resident(c.cus, lds);
    c.res_lds[slot] = lds;
  }
  c.resident_blocks = c.res_blocks[slot];
  c.resident_lds = lds;
  char* r = (char*)b.rows.p;
  w.cls = (uint8_t*)b.cls.p;
  w.wcarry = (float4*)b.wcarry.p;
  w.deprec = b.deprec.p;
  w.row_prevw = (long long*)r;   r += (size_t)H * sizeof(long long);
  w.row_prevd = (long long*)r;   r += (size_t)H * sizeof(long long);
  w.row_stats = r;               r += (size_t)H * rc::row_stats_bytes();
  w.row_off = (int*)r;           r += (size_t)H * sizeof(int);
  w.row_soff = (int*)r;
  w.dep_pix = (long long*)b.dep_pix.p;
  w.seg_key = (long long*)b.seg_key.p;
  w.seg_start = (int*)b.seg_start.p;
  w.seg_order = (int*)b.seg_order.p;
  w.cin = b.cin.p;
  w.batch_state = (int*)b.batch_state.p;   // claim words, then completion counts, then queue
  w.batch_cnt = w.batch_state + (P / 64 + 2);
  w.batch_rq = w.batch_state + 2 * (P / 64 + 2);
  w.batch_ints = (int)(3 * (P / 64 + 2));
  w.side = nullptr;
  w.rstream = nullptr;
  w.pstream = nullptr;
  w.rready = w.rdone = w.rt0 = w.rt1 = nullptr;
  w.split_shade = tu.split_shade ? 1 : 0;
  if (piped) w.split_shade = 0;   // phase C after the resolver, on the pixel partition
  // phase C beside the resolver: always (side 1), or (side 2, the default) for images of
  // >= 8 Mpixel — below that phase C after the resolver is short and the side kernel's
  // census / k_finish tail costs more (lone simple 1024^2 d6 0.746 -> 0.680 ms, reflection
  // 2048^2 d4 1.045 -> 1.003 ms without it; quadric 4096^2 +0.5 ms, 8192^2 +2.2 ms)
  const bool side = tu.side == 1 || (tu.side == 2 && P >= ((size_t)8 << 20));
  if (!piped && side) {   // phase C overlapped with the resolver
    if (!c.side) {
      if (hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&c.fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c.join, hipEventDisableTiming) != hipSuccess)
        return -1;
    }
    // k_side's LDS request must exceed what a resolver workgroup leaves free on its CU, for
    // the reservation this call's resolver actually makes (the tuning may change it)
    if (lds > 0 && c.side_for_lds != lds) {
      c.side_lds = rc::side_lds_bytes(lds);
      c.side_blocks = rc::phase_c_side_blocks(c.cus, c.side_lds);
      c.side_for_lds = lds;
    }
    if (c.side_blocks > 0 && lds > 0) {   // the guard needs the resolver's LDS reservation
      w.side = c.side;
      w.fork = c.fork;
      w.join = c.join;
      // one k_side workgroup per CU by default (of the two that fit): phase C still finishes
      // beside the resolver, and the resolver's chains lose less to the side kernel's memory
      // traffic (lone quadric 4096^2 5.72 -> 5.67 ms, 8192^2 15.77 -> 15.26 ms)
      w.side_blocks = c.side_blocks;
      const int cap = tu.side_blocks > 0 ? tu.side_blocks : c.cus;
      if (cap < w.side_blocks) w.side_blocks = cap;
      w.side_lds = c.side_lds;
    }
  }
  if (!w.side) w.split_shade = 0;   // split shading needs the side kernel
  // side 3: phase C inside the resolver (its waves shade ready batches once their own work is
  // done), a lone frame only
  w.inres = (!piped && tu.side == 3) ? 1 : (!piped && tu.side == 4) ? 2 : 0;
  w.epoch = b.epoch;
  w.counters = (int*)b.counters.p;
  w.team = b.team.p;
  // The team spins on a counter barrier: its blocks (the first of the grid) and the grid as
  // a whole must be co-resident, so the grid never exceeds the resident capacity.
  w.resolve_blocks = c.resident_blocks / c.cus * res_cus;   // whole CUs' worth
  if (tu.resolve_grid >= 8 && tu.resolve_grid < w.resolve_blocks)   // experiments: a smaller grid
    w.resolve_blocks = tu.resolve_grid;
  w.resolve_lds = c.resident_lds;
  // team size: 128 of a whole-device grid.  A pipelined resolver's grid: half of it for the
  // 8-32 Mpixel images, whose resolver lanes hold half the device (quadric 4096^2: 5.70e9 ->
  // 5.87e9 rays/s at 64 of 128, 5.82e9 at 56, 5.45e9 at 80: a larger team scans the 707k-entry
  // clean stretch in fewer rounds), 3/8 otherwise (reflection 2048^2 d4 7.6e9 vs 7.4e9 at half,
  // simple 1024^2 d6 3.1e9 vs 2.9e9; quadric 8192^2 unchanged, its resolvers slower at half)
  const bool half_team = P >= ((size_t)8 << 20) && P < ((size_t)32 << 20);
  w.team_blocks = !piped ? 128 : half_team ? w.resolve_blocks / 2 : w.resolve_blocks * 3 / 8;
  if (tu.team_blocks >= 0) w.team_blocks = tu.team_blocks;
  if (w.team_blocks > 256) w.team_blocks = 256;
  if (w.team_blocks > w.resolve_blocks / 2) w.team_blocks = w.resolve_blocks / 2;
  // the placement rc_resolver_stats_get reports
  if (piped) {
    c.pipe_grid = w.resolve_blocks;
    c.pipe_res_cus = res_cus;
    c.pipe_lds = w.resolve_lds;
    c.pipe_team = w.team_blocks;
  } else {
    c.lone_grid = w.resolve_blocks;
    c.lone_res_cus = res_cus;
    c.lone_lds = w.resolve_lds;
    c.lone_team = w.team_blocks;
  }
  // helper blocks for handed-off dense runs (k_resolve): 16 of the grid for a lone frame,
  // runs handed off after 128 changes (quadric 4096^2 5.01 -> 4.65 ms); 4 in a pipeline lane
  // (pipe_helpers), whose grid is a partition's and whose regular waves need most of the slots
  // (round 2, hand-offs after 512 changes: 8 helpers per lane lost 1-6 %)
  w.helpers = piped ? tu.pipe_helpers : tu.helpers;
  if (w.helpers < 0) w.helpers = 0;
  if (w.helpers > rc::kDenseSlots) w.helpers = rc::kDenseSlots;   // one ring slot per helper
  if (w.team_blocks + w.helpers > w.resolve_blocks * 3 / 4) w.helpers = 0;
  w.hand_run = tu.hand_run;
  w.long_len = tu.long_len;
  w.block_min = tu.block_min;
  w.headb_first = piped ? 0 : tu.headb_first;
  if (w.headb_first > w.resolve_blocks - w.team_blocks - w.helpers)
    w.headb_first = w.resolve_blocks - w.team_blocks - w.helpers;
  if (w.headb_first < 0) w.headb_first = 0;
  w.wave_k = tu.wave_k;
  w.resolve_k = tu.resolve_k;
  w.resolve_clean = tu.resolve_clean;
  w.team_cscan = tu.team_cscan;
  w.coop_group = 0;
  if (tu.coop && b.scene_src) {
    const int n = ((const rc_packed_header*)b.scene_src)->n;
    int g = 4;   // groups of >= 4 lanes: the evaluator is specialised for 4, 8 and 16
    while (g < n) g <<= 1;
    if (n >= 1 && g <= 64) w.coop_group = g;
  }
  w.trace = nullptr;
#if RC_DIAG   // diagnostic build (make stamps): per-segment resolver trace
  if (std::getenv("RC_RESOLVE_TRACE")) {
    if (b.trace.ensure(P * 7 * sizeof(unsigned))) return -1;
    if (hipMemset(b.trace.p, 0, b.trace.bytes) != hipSuccess) return -1;
    w.trace = (unsigned*)b.trace.p;
  }
#endif
  w.phase_c_blocks = (piped ? c.cus - res_cus : c.cus) * 8;
  w.phase_c_finish = tu.phase_c_finish ? 1 : 0;
  return 0;
}

// The pending phase C (Pipe::cdefer) of the last submitted frame: on its lane's phase C
// stream, or with `whole` on the device stream over every CU — the window's last frame, whose
// phase C otherwise ran alone on the pixel partition after the last resolver (0.8 ms of a
// 20-frame window's drain at quadric 4096^2 against ~0.47 ms on every CU).
int flush_phase_c(DevCtx& c, bool whole) {
  Pipe& p = c.pipe;
  if (!p.cdefer) return 0;
  p.cdefer = false;
  rc::ParityWork& w = p.cdefer_w;
  hipStream_t s = p.pc[p.cdefer_lane];
  if (whole) {
    s = c.stream;
    w.phase_c_blocks = c.cus * 8;
  }
  HIP_TRY(rc::launch_phase_c(p.cdefer_ls, p.cdefer_W, p.cdefer_H, p.cdefer_maxrec, p.cdefer_out,
                             w, p.cdefer_zc, s));
  // the frame's hand-off words, before the event that lets slot k's next frame reset them
  if (p.log.enqueue(w.team, s)) return -1;
  HIP_TRY(hipEventRecord(p.cdone[p.cdefer_k], s));
  p.cpend[p.cdefer_k] = true;
  return 0;
}

int enqueue_render_ws(DevCtx& c, const rc_scene* s, int W, int H, int row0, int row_step,
                      int nrows, const rc_options* opt, uint8_t* d_out, hipStream_t stream,
                      bool timed, uint32_t* patch, hipEvent_t** evset);

// Enqueue one render of rows (row0 + k*row_step) into d_out on `stream`, using the device's
// one-frame workspace c.fb: after the previous render that used it, whatever its stream.
int enqueue_render(DevCtx& c, const rc_scene* s, int W, int H, int row0, int row_step, int nrows,
                   const rc_options* opt, uint8_t* d_out, hipStream_t stream, bool timed,
                   uint32_t* patch, hipEvent_t** evset) {
  // a frame in flight's held-back phase C goes out first, so that a device synchronisation
  // after this call completes it (rc_frames_wait stays the frames' completion point)
  if (flush_phase_c(c, false)) return -1;
  if (c.ws_valid && c.ws_stream != stream) HIP_TRY(hipStreamWaitEvent(stream, c.ws_ev, 0));
  const int rc = enqueue_render_ws(c, s, W, H, row0, row_step, nrows, opt, d_out, stream, timed,
                                   patch, evset);
  // recorded even after a failed enqueue: whatever was enqueued stays ordered
  HIP_TRY(hipEventRecord(c.ws_ev, stream));
  c.ws_stream = stream;
  c.ws_valid = true;
  return rc;
}

int enqueue_render_ws(DevCtx& c, const rc_scene* s, int W, int H, int row0, int row_step,
                      int nrows, const rc_options* opt, uint8_t* d_out, hipStream_t stream,
                      bool timed, uint32_t* patch, hipEvent_t** evset) {
  rc::LaunchScene ls;
  if (upload_scene(c.fb, stream, s, ls)) return -1;
  unsigned long long* zc = (unsigned long long*)c.fb.zcount.p;
  HIP_TRY(hipMemsetAsync(zc, 0, sizeof(unsigned long long), stream));
  const int maxrec = opt->max_recursion;
  const bool parity = opt->mode == RC_MODE_PARITY && maxrec > 1;
  hipEvent_t* ev = c.ev[0];
  if (c.prof_active) {
    ev = c.ev[c.prof_calls % DevCtx::kEvSets];
    c.prof_calls++;
    c.prof_parity = parity;
  }
  if (evset) *evset = ev;
  if (timed) HIP_TRY(hipEventRecord(ev[0], stream));
  if (!parity) {
    HIP_TRY(rc::launch_render(ls, W, H, row0, row_step, nrows, maxrec, d_out, zc, stream,
                              opt->mode == RC_MODE_CUDA));
    if (timed) HIP_TRY(hipEventRecord(ev[1], stream));
    return 0;
  }
  if (row0 != 0 || row_step != 1 || nrows != H) {
    std::fprintf(stderr, "Error: parity mode renders whole images only\n");
    return -1;
  }
  rc::ParityWork w{};
  int res_cus = c.cus;   // experiment: single_res_cus sizes the resolver like a pipeline lane's
  if (tune().single_res_cus > 0) res_cus = tune().single_res_cus;
  if (res_cus < 8 || res_cus > c.cus) res_cus = c.cus;
  if (ensure_parity(c, c.fb, W, H, w, res_cus, 0)) {
    std::fprintf(stderr, "Error: out of device memory for the parity workspace\n");
    return -1;
  }
  if (w.split_shade) ls.dep_fast = 0;   // k_classify leaves no primary shade
  // phase C inside the resolver needs a resolver long enough to hide it: at depth 1 (two
  // levels) the chains are short and the resolver's one wave per SIMD shades more slowly than
  // k_dep_chunks' full occupancy (simple 1024^2 d1 0.143 -> 0.175 ms; from depth 2 it gains:
  // 1024^2 d6 0.678 -> 0.663, reflection 2048^2 d4 0.966 -> 0.873, quadric 4096^2 5.58 -> 5.18)
  if (maxrec < 3) w.inres = 0;
  w.patch = patch;
  w.inject = take_inject();
  HIP_TRY(rc::launch_parity(ls, W, H, maxrec, d_out, w, zc, stream, timed ? ev + 1 : nullptr));
  return c.lone_log.enqueue(w.team, stream);
}

// After a synchronised parity render: the resolver's and phase C's bounded spins set
// TeamState.error (first word) if a hand-off never completed; the image is then invalid.
// The report names the first spin that failed (TeamState: code, workgroup, site detail), the
// helper queue's counters and, for a missing carry-in, the segment it belongs to and how many
// entries of the frame were never published.
int report_spin_error(const FrameBufs& b, const char* where) {
  int e[4] = {0, 0, 0, 0};
  if (hipMemcpy(e, b.team.p, sizeof e, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (!e[0]) return 0;
  int dq[3] = {0, 0, 0}, cnt[16] = {};
  (void)hipMemcpy(dq, (const char*)b.team.p + rc::team_dq_offset(), sizeof dq,
                  hipMemcpyDeviceToHost);
  (void)hipMemcpy(cnt, b.counters.p, sizeof cnt, hipMemcpyDeviceToHost);
  std::fprintf(stderr,
               "Error: parity resolver hand-off timed out (code %d: %s; %s) at workgroup %d, "
               "detail %d/%d; segments %d, DEP entries %d, resolver census %d, helper queue "
               "prod %d claim %d finished %d, side workgroups go %d gave-up %d\n",
               e[0], spin_site(e[0]), where, e[1], e[2], e[3], cnt[0],
               cnt[2], cnt[5], dq[0], dq[1], dq[2], cnt[12], cnt[13]);
  if (e[0] == 1) {   // a team hand-off: each team block's latest published round (its slots)
    const int nb = rc::team_slot_bufs(), nt = rc::team_slot_blocks();
    std::vector<unsigned long long> sl((size_t)nb * nt * 4);
    if (hipMemcpy(sl.data(), (const char*)b.team.p + rc::team_slot_offset(),
                  sl.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess) {
      std::vector<int> last(nt, 0);   // the latest round whose four granules all arrived
      for (int q = 0; q < nb; ++q)
        for (int k = 0; k < nt; ++k) {
          int r = 1 << 30;
          for (int g = 0; g < 4; ++g)
            r = std::min(r, (int)(unsigned)(sl[((size_t)q * nt + k) * 4 + g] >> 32));
          last[k] = std::max(last[k], r);
        }
      int lo = 1 << 30, hi = 0;
      for (int k = 0; k < nt; ++k)
        if (last[k] > 0) lo = std::min(lo, last[k]), hi = std::max(hi, last[k]);
      std::fprintf(stderr, "  team slots: latest round per block %d .. %d; behind:", lo, hi);
      int shown = 0;
      for (int k = 0; k < nt && shown < 16; ++k)
        if (last[k] > 0 && last[k] < hi) std::fprintf(stderr, " %d:%d", k, last[k]), ++shown;
      std::fprintf(stderr, "\n  slot[round %% %d][block %d] tags:", nb, e[3]);
      for (int q = 0; q < nb && e[3] >= 0 && e[3] < nt; ++q)
        for (int g = 0; g < 4; ++g)
          std::fprintf(stderr, " %u", (unsigned)(sl[((size_t)q * nt + e[3]) * 4 + g] >> 32));
      std::fprintf(stderr, "\n");
    }
    if (const size_t off = rc::team_handoff_diag_offset()) {   // RC_HANDOFF_DIAG builds
      unsigned long long t[1 + 4] = {};
      int r[4] = {};
      const int nb = std::min(rc::team_slot_bufs(), 4);
      if (hipMemcpy(t, (const char*)b.team.p + off, sizeof(unsigned long long) * (1 + nb),
                    hipMemcpyDeviceToHost) == hipSuccess &&
          hipMemcpy(r, (const char*)b.team.p + off + sizeof(unsigned long long) * (1 + nb),
                    sizeof(int) * nb, hipMemcpyDeviceToHost) == hipSuccess) {
        std::fprintf(stderr, "  block 0 published (round: us relative to the first failed spin):");
        for (int q = 0; q < nb; ++q)
          std::fprintf(stderr, " %d: %.1f", r[q], ((double)t[1 + q] - (double)t[0]) / 100.0);
        std::fprintf(stderr, "\n");
      }
    }
  }
  const int nseg = cnt[0], ndep = cnt[2];
  if (nseg > 0 && ndep > 0 && b.cin.p && b.seg_start.p) {
    std::vector<int> starts(nseg);
    std::vector<unsigned long long> g((size_t)ndep * 3);
    if (hipMemcpy(starts.data(), b.seg_start.p, starts.size() * sizeof(int),
                  hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(g.data(), b.cin.p, g.size() * sizeof(unsigned long long),
                  hipMemcpyDeviceToHost) == hipSuccess) {
      long long missing = 0;
      int shown = 0;
      for (int s = 0; s < nseg; ++s) {
        const int end = s + 1 < nseg ? starts[s + 1] : ndep;
        int first = -1, n = 0;
        for (int j = starts[s]; j < end; ++j) {
          const unsigned t0 = (unsigned)(g[3 * (size_t)j] >> 32) & 0x7fffffffu;
          if (t0 != b.epoch) {
            if (first < 0) first = j;
            ++n;
          }
        }
        missing += n;
        if (n && shown++ < 8)
          std::fprintf(stderr, "  segment %d [%d, %d) length %d: %d entries unpublished from %d\n",
                       s, starts[s], end, end - starts[s], n, first);
      }
      std::fprintf(stderr, "  %lld of %d carry-ins unpublished\n", missing, ndep);
    }
  }
  return -1;
}

int check_spin_error(FrameBufs& b, const rc_options* opt) {
  if (!(opt->mode == RC_MODE_PARITY && opt->max_recursion > 1) || !b.team.p) return 0;
  return report_spin_error(b, "one frame");
}

double event_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();   // not sticky: later launches check hipGetLastError()
    return 0.0;
  }
  return ms;
}

// tail (optional): the frame's zero-normalize count (8 B) and counters[0..3] (at +16), copied
// into pinned memory on the frame's stream behind its last kernel (rc_render), so reading them
// costs no extra round trip after the frame
void fill_device_timing(DevCtx& c, const rc_options* opt, rc_timing* t,
                        const uint8_t* tail) {
  const bool parity = opt->mode == RC_MODE_PARITY && opt->max_recursion > 1;
  hipEvent_t* ev = c.ev[0];
  double k = parity ? event_ms(ev[0], ev[4]) : event_ms(ev[0], ev[1]);
  g_last_kernel_ms = parity ? event_ms(ev[2], ev[3]) : k;
  if (!t) return;
  t->kernel_ms = k;
  t->resolve_ms = parity ? event_ms(ev[2], ev[3]) : 0.0;
  unsigned long long z = 0;
  if (tail)
    std::memcpy(&z, tail, sizeof z);
  else if (hipMemcpy(&z, c.fb.zcount.p, sizeof z, hipMemcpyDeviceToHost) != hipSuccess)
    z = 0;
  t->zero_normalize = (int64_t)z;
  if (parity) {
    int cnt[4] = {0, 0, 0, 0};
    if (tail)
      std::memcpy(cnt, tail + 16, sizeof cnt);
    else if (hipMemcpy(cnt, c.fb.counters.p, sizeof cnt, hipMemcpyDeviceToHost) != hipSuccess)
      cnt[2] = 0;
    t->dep_pixels = cnt[2];
#if RC_DIAG
    if (std::getenv("RC_SIDE_STATS")) {
      int cc[16];
      if (hipMemcpy(cc, c.fb.counters.p, sizeof cc, hipMemcpyDeviceToHost) == hipSuccess)
        std::fprintf(stderr,
                     "side: blocks go %d gave-up %d, tiles side %d finish %d, batches side %d "
                     "finish %d (side_blocks %d)\n",
                     cc[12], cc[13], cc[8], cc[10], cc[9], cc[11], c.side_blocks);
    }
    const char* path = std::getenv("RC_RESOLVE_TRACE");
    if (path && c.fb.trace.p && cnt[0] > 0) {   // debug: per-segment resolver trace
      std::vector<int> starts(cnt[0]);
      std::vector<unsigned> tr(3 * (size_t)cnt[0]);
      (void)hipMemcpy(starts.data(), c.fb.seg_start.p, starts.size() * sizeof(int),
                      hipMemcpyDeviceToHost);
      (void)hipMemcpy(tr.data(), c.fb.trace.p, tr.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
      if (FILE* f = std::fopen(path, "w")) {
        std::fprintf(f, "# seg start len ticks_100MHz evals(team: rounds|0x80000000) cycles\n");
        for (int k = 0; k < cnt[0]; ++k) {
          const int end = k + 1 < cnt[0] ? starts[k + 1] : cnt[2];
          std::fprintf(f, "%d %d %d %u %u %u\n", k, starts[k], end - starts[k], tr[3 * k],
                       tr[3 * k + 1], tr[3 * k + 2]);
        }
        std::fclose(f);
      }
      {   // per-segment start times (regular waves)
        std::vector<unsigned> st(cnt[0]);
        (void)hipMemcpy(st.data(),
                        (const unsigned*)c.fb.trace.p + 3 * (size_t)cnt[2] + 4 * (size_t)cnt[0] +
                            8 * 8192,
                        st.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        std::string p4 = std::string(path) + ".start";
        if (FILE* f = std::fopen(p4.c_str(), "w")) {
          for (int k = 0; k < cnt[0]; ++k) std::fprintf(f, "%d %u\n", k, st[k]);
          std::fclose(f);
        }
      }
      {   // when each resolver wave left (block * 4 + wave)
        std::vector<unsigned> we(4096);
        (void)hipMemcpy(we.data(),
                        (const unsigned*)c.fb.trace.p + 3 * (size_t)cnt[2] + 5 * (size_t)cnt[0] +
                            8 * 8192,
                        we.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        std::string p5 = std::string(path) + ".waves";
        if (FILE* f = std::fopen(p5.c_str(), "w")) {
          for (int k = 0; k < 4096; ++k)
            if (we[k]) std::fprintf(f, "%d %u\n", k, we[k]);
          std::fclose(f);
        }
      }
      {   // k_side's ready-queue items: pop time, carries ready, batch shaded
        const int nb = (cnt[2] + 63) / 64;
        std::vector<unsigned> tq(3 * (size_t)nb);
        (void)hipMemcpy(tq.data(),
                        (const unsigned*)c.fb.trace.p + 3 * (size_t)cnt[2] + 5 * (size_t)cnt[0] +
                            200000,
                        tq.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        std::string p7 = std::string(path) + ".side";
        if (FILE* f = std::fopen(p7.c_str(), "w")) {
          for (int k = 0; k < nb; ++k)
            if (tq[3 * k]) std::fprintf(f, "%d %u %u %u\n", k, tq[3 * k], tq[3 * k + 1], tq[3 * k + 2]);
          std::fclose(f);
        }
      }
      {   // team rounds' eval/step cycles and the helper items
        const unsigned* b0 = (const unsigned*)c.fb.trace.p + 3 * (size_t)cnt[2] +
                             5 * (size_t)cnt[0] + 8 * 8192 + 4096;
        std::vector<unsigned> te(16384 + 8 * 64 + 8192);
        (void)hipMemcpy(te.data(), b0, te.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        std::string p6 = std::string(path) + ".cyc";
        if (FILE* f = std::fopen(p6.c_str(), "w")) {
          for (int r = 0; r < 8192; ++r)
            if (te[2 * r] | te[2 * r + 1])
              std::fprintf(f, "round %d eval %u step %u wait %u\n", r, te[2 * r], te[2 * r + 1],
                           te[16384 + 8 * 64 + r]);
          for (int k = 0; k < 64; ++k) {
            const unsigned* ti = &te[16384 + 8 * k];
            if (ti[2])
              std::fprintf(f, "item %d seg %u wait %u t0 %u t1 %u coop %u changers %u eval %u step %u\n",
                           k, ti[0], ti[1], ti[2], ti[3], ti[4], ti[5], ti[6], ti[7]);
          }
          std::fclose(f);
        }
      }
      {   // per-round team log (k_resolve, team blocks)
        std::vector<unsigned> tl(8 * 8192);
        (void)hipMemcpy(tl.data(),
                        (const unsigned*)c.fb.trace.p + 3 * (size_t)cnt[2] + 4 * (size_t)cnt[0],
                        tl.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        std::string p3 = std::string(path) + ".team";
        if (FILE* f = std::fopen(p3.c_str(), "w")) {
          std::fprintf(f, "# round mode(0 scan/1 resolve) j0 j1 cycles lane_passes coop_steps changers\n");
          for (int r = 1; r < 8192; ++r)
            if (tl[8 * r + 7] == 0xA5A5A5A5u)
              std::fprintf(f, "%d %u %u %u %u %u %u %u\n", r, tl[8 * r], tl[8 * r + 1],
                           tl[8 * r + 2], tl[8 * r + 3], tl[8 * r + 4], tl[8 * r + 5],
                           tl[8 * r + 6]);
          std::fclose(f);
        }
      }
#if RC_STAMPS
      std::vector<unsigned> sp(4 * (size_t)cnt[0]);
      (void)hipMemcpy(sp.data(), (const unsigned*)c.fb.trace.p + 3 * (size_t)cnt[2],
                      sp.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
      std::string p2 = std::string(path) + ".stamps";
      if (FILE* f = std::fopen(p2.c_str(), "w")) {
        for (int k = 0; k < cnt[0]; ++k)
          if (sp[4 * k] | sp[4 * k + 1])
            std::fprintf(f, "%d norm %u test %u argmin %u hit+loop %u\n", k, sp[4 * k],
                         sp[4 * k + 1], sp[4 * k + 2], sp[4 * k + 3]);
        std::fclose(f);
      }
#endif
    }
#endif  // RC_DIAG
  }
}

}  // namespace rcrt

extern "C" {

int rc_render_device(const rc_scene* s, int W, int H, int row0, int row_step, int nrows,
                     const rc_options* opt, uint8_t* d_out, void* stream, rc_timing* timing) {
  if (!s || !opt || !d_out || W <= 0 || H <= 0 || nrows < 0 || row_step < 1) return -1;
  if (row0 < 0 || (nrows > 0 && row0 + (long long)(nrows - 1) * row_step >= H)) return -1;
  if (nrows == 0) return 0;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  // an earlier frame of this workspace whose hand-off failed is reported by the next call
  // (once: the report consumes the counts)
  if (c->lone_log.earlier_failed()) {
    c->lone_log.take(nullptr, nullptr);
    return -1;
  }
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  const long long own = c->lone_log.head;   // this frame's ring entry (parity frames log one)
  // the scene upload and events live on the ctx stream: order them with the caller's stream
  if (st != c->stream) {
    hipStream_t saved = c->stream;
    c->stream = st;
    int rc = enqueue_render(*c, s, W, H, row0, row_step, nrows, opt, d_out, st, true);
    c->stream = saved;
    if (rc) return rc;
  } else if (enqueue_render(*c, s, W, H, row0, row_step, nrows, opt, d_out, st, true)) {
    return -1;
  }
  if (timing) {
    std::memset(timing, 0, sizeof *timing);
    HIP_TRY(hipStreamSynchronize(st));
    const long long before = c->lone_log.checked;
    const bool failed = c->lone_log.entry_failed(own);
    c->lone_log.poll();
    if (failed) {
      c->lone_log.take(nullptr, nullptr);
      return -1;
    }
    if (check_spin_error(c->fb, opt)) return -1;
    timing->frames_checked = c->lone_log.checked - before;
    fill_device_timing(*c, opt, timing);
    timing->total_ms = timing->kernel_ms;
  }
  return 0;
}

// ------------------------------------------------------------ pipelined frames --
}  // extern "C"

namespace {

// Release the pipelines' CU-masked streams and events before the runtime's own teardown
// (left to process exit they crash a profiled process's finalisation).
void pipe_release(DevCtx& c) {
  Pipe& p = c.pipe;
  if (!p.init) return;
  (void)hipSetDevice(c.device);
  (void)hipDeviceSynchronize();
  for (int k = 0; k < p.slots; ++k) {
    if (p.pix[k]) (void)hipStreamDestroy(p.pix[k]);
    (void)hipEventDestroy(p.ready[k]);
    (void)hipEventDestroy(p.done[k]);
    (void)hipEventDestroy(p.cdone[k]);
    (void)hipEventDestroy(p.adone[k]);
  }
  for (int r = 0; r < p.lanes; ++r) {
    (void)hipStreamDestroy(p.res[r]);
    if (r < 2 && p.comp[r]) (void)hipStreamDestroy(p.comp[r]);
    if (p.pc[r] && (r == 0 || !p.pc_shared)) (void)hipStreamDestroy(p.pc[r]);
  }
  p.pc_shared = false;
  for (auto& e : p.rt) {
    (void)hipEventDestroy(e[0]);
    (void)hipEventDestroy(e[1]);
  }
  p.init = false;
  p.cdefer = false;   // nothing launched stays pending across a rebuilt pipeline
  p.submitted = 0;
  p.frames = 0;
  p.last = -1;
  for (int k = 0; k < Pipe::kSlots; ++k) {
    p.cpend[k] = false;
    p.pix[k] = nullptr;
  }
  for (int r = 0; r < Pipe::kLanes; ++r) p.pc[r] = nullptr;
  p.comp[0] = p.comp[1] = nullptr;
  for (auto& sp : p.spare) {
    if (sp) (void)hipStreamDestroy(sp);
    sp = nullptr;
  }
}

void pipe_release_all() {
  for (auto& c : g_ctx) pipe_release(c);
}

int pipe_init(DevCtx& c, long long pixels) {
  Pipe& p = c.pipe;
  if (p.init) return 0;
  static bool registered = false;
  if (!registered) {
    std::atexit(pipe_release_all);
    registered = true;
  }
  // partition A: the low `res` bits of the CU mask, which the driver deals round-robin over
  // the XCDs (bit i -> XCD i mod 8), so both partitions span every XCD.
  // Resolver partition by image size, fixed at the first pipelined frame (measured with frames
  // in flight, scripts/pipe_sweep.sh): a quarter of the CUs below 8 Mpixel, where the pixel
  // phases are the bound (reflection 2048^2 d4 6.9e9 -> 7.9e9, simple 1024^2 d6 3.5e9 -> 3.7e9
  // rays/s vs half); half up to 32 Mpixel (quadric 4096^2: 5.7e9 at 128 CUs, 5.1e9 at 112);
  // 3/8 above (quadric 8192^2: 7.4e9 at 96 CUs, 6.4e9 at 128, 6.0e9 at 80).
  const rc_tuning tu = tune();
  int res = pixels < (8ll << 20) ? c.cus / 4 : pixels < (32ll << 20) ? c.cus / 2 : c.cus * 3 / 8;
  if (tu.pipe_res_cus > 0) res = tu.pipe_res_cus;
  p.lanes = tu.pipe_resolvers;
  if (p.lanes < 1) p.lanes = 1;
  if (p.lanes > Pipe::kLanes) p.lanes = Pipe::kLanes;
  p.slots = tu.pipe_slots;
  if (p.slots < p.lanes + 1) p.slots = p.lanes + 1;
  if (p.slots > Pipe::kSlots) p.slots = Pipe::kSlots;
  p.rt_on = tu.pipe_timing != 0;
  p.fifo = tu.pipe_slotstreams == 0;
  res = res / (8 * p.lanes) * (8 * p.lanes);   // whole CUs per XCD for every resolver
  if (res < 16 * p.lanes) res = 16 * p.lanes;
  if (res > c.cus - 16) res = (c.cus - 16) / (8 * p.lanes) * (8 * p.lanes);
  const int words = (c.cus + 31) / 32;
  std::vector<uint32_t> ma(words, 0), mb(words, 0);
  for (int i = 0; i < c.cus; ++i) (i < res ? ma : mb)[i / 32] |= 1u << (i % 32);
  // the CU-masked streams, in the order tu.pipe_order names (the runtime assigns hardware
  // queues in creation order, and a queue's dispatcher serves one kernel's workgroups at a time)
  const bool comp = tu.comp_stream == 1 || (tu.comp_stream == 2 && pixels >= (32ll << 20));
  auto mk_res = [&]() -> int {
    for (int r = 0; r < p.lanes; ++r) {
      HIP_TRY(hipExtStreamCreateWithCUMask(&p.res[r], (uint32_t)words, ma.data()));
      // compaction off the pixel partition (any CU, first): quadric 8192^2 8.38e9 -> 8.49e9
      // rays/s; at 4096^2 its workgroups on the resolver partition cost more (5.91e9 -> 5.85e9)
      if (r < 2 && comp) {
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&p.comp[r], hipStreamNonBlocking, hi));
      }
    }
    return 0;
  };
  auto mk_pc = [&]() -> int {
    for (int r = 0; r < p.lanes; ++r)
      if (p.fifo) HIP_TRY(hipExtStreamCreateWithCUMask(&p.pc[r], (uint32_t)words, mb.data()));
    return 0;
  };
  auto mk_pix = [&]() -> int {
    for (int k = 0; k < p.slots; ++k)
      if (!p.fifo || k < 2)
        HIP_TRY(hipExtStreamCreateWithCUMask(&p.pix[k], (uint32_t)words, mb.data()));
    return 0;
  };
  if (tu.pipe_order == 0) {   // lane by lane (resolver, its phase C), then the pixel streams
    for (int r = 0; r < p.lanes; ++r) {
      HIP_TRY(hipExtStreamCreateWithCUMask(&p.res[r], (uint32_t)words, ma.data()));
      if (r < 2 && comp) {
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&p.comp[r], hipStreamNonBlocking, hi));
      }
      if (p.fifo) HIP_TRY(hipExtStreamCreateWithCUMask(&p.pc[r], (uint32_t)words, mb.data()));
    }
    if (mk_pix()) return -1;
  } else if (tu.pipe_order == 1) {
    if (mk_res() || mk_pix() || mk_pc()) return -1;
  } else if (tu.pipe_order == 3 && p.fifo && p.lanes == 2) {
    // four hardware queues dealt in creation order: each resolver lane alone on its queue
    // (with an idle placeholder stream), the two pixel streams on one (their phase A run one
    // at a time anyway) and the two phase C streams on the other
    if (mk_res()) return -1;
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pix[0], (uint32_t)words, mb.data()));
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pc[0], (uint32_t)words, mb.data()));
    for (int r = 0; r < 2; ++r)
      HIP_TRY(hipExtStreamCreateWithCUMask(&p.spare[r], (uint32_t)words, ma.data()));
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pix[1], (uint32_t)words, mb.data()));
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pc[1], (uint32_t)words, mb.data()));
  } else if (tu.pipe_order == 4 && p.fifo && p.lanes == 2) {
    // one phase C stream for both lanes (consecutive frames' phase C never overlap: a lane's
    // resolver ends half a frame period after the other's), so with the device stream created
    // first and four hardware queues dealt in creation order each resolver lane shares its
    // queue only with an idle placeholder: {device stream, pix[0]}, {res[0], spare},
    // {res[1], spare}, {pc, pix[1]}
    for (int r = 0; r < 2; ++r)
      HIP_TRY(hipExtStreamCreateWithCUMask(&p.res[r], (uint32_t)words, ma.data()));
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pc[0], (uint32_t)words, mb.data()));
    p.pc[1] = p.pc[0];
    p.pc_shared = true;
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pix[0], (uint32_t)words, mb.data()));
    for (int r = 0; r < 2; ++r)
      HIP_TRY(hipExtStreamCreateWithCUMask(&p.spare[r], (uint32_t)words, ma.data()));
    HIP_TRY(hipExtStreamCreateWithCUMask(&p.pix[1], (uint32_t)words, mb.data()));
  } else {
    if (tu.pipe_order >= 3)
      std::fprintf(stderr, "Warning: pipe_order %d needs two resolver lanes and the default "
                   "stream layout (pipe_resolvers %d, pipe_slotstreams %d): using order 2\n",
                   tu.pipe_order, p.lanes, p.fifo ? 0 : 1);
    if (mk_pix() || mk_pc() || mk_res()) return -1;
  }
  for (int k = 0; k < p.slots; ++k) {
    HIP_TRY(hipEventCreateWithFlags(&p.adone[k], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&p.ready[k], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&p.done[k], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&p.cdone[k], hipEventDisableTiming));
  }
  for (auto& e : p.rt) {
    HIP_TRY(hipEventCreate(&e[0]));
    HIP_TRY(hipEventCreate(&e[1]));
  }
  p.res_cus = res;
  p.built_lanes = tu.pipe_resolvers;
  p.built_slots = tu.pipe_slots;
  p.built_res = tu.pipe_res_cus;
  p.built_order = tu.pipe_order;
  p.init = true;
  return 0;
}

}  // namespace

extern "C" {

int rc_frame_submit(const rc_scene* s, int W, int H, const rc_options* opt, uint8_t* d_out) {
  if (!s || !opt || !d_out || W <= 0 || H <= 0) return -1;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  const int maxrec = opt->max_recursion;
  if (!(opt->mode == RC_MODE_PARITY && maxrec > 1)) {   // no serial stage: whole GPU, in order
    if (enqueue_render(*c, s, W, H, 0, 1, H, opt, d_out, c->stream, false)) return -1;
    c->pipe.frames++;
    return 0;
  }
  if (pipe_init(*c, (long long)W * H)) return -1;
  Pipe& p = c->pipe;
  // fail fast: a frame in flight whose hand-off already failed (its entry has arrived)
  p.log.poll();
  if (p.log.failed > 0) {
    std::fprintf(stderr, "Error: rc_frame_submit: %lld frame(s) in flight failed; call "
                 "rc_frames_wait\n", p.log.failed);
    return -1;
  }
  // the previous frame's phase C on its lane (it was held back in case that frame was the
  // window's last), before anything of this frame: the frame log stays in submission order
  if (flush_phase_c(*c, false)) return -1;
  const int k = (int)(p.total % p.slots);
  const int lane = (int)(p.total % p.lanes);
  FrameBufs& b = p.fb[k];
  // A frame submitted into an empty pipeline has no resolver to hide behind: its phase A
  // and compaction take the whole device (then phase C returns to the slot's partition).
  // Slot k's previous frame is complete (rc_frames_wait synchronised every slot).
  const bool first = p.submitted == 0;
  hipStream_t st = first ? c->stream : p.pix[p.fifo ? (int)(p.total & 1) : k];
  if (p.fifo && p.cpend[k]) HIP_TRY(hipStreamWaitEvent(st, p.cdone[k], 0));
  if (p.fifo && !first) HIP_TRY(hipStreamWaitEvent(st, p.adone[p.last], 0));
  rc::LaunchScene ls;
  if (upload_scene(b, st, s, ls) || b.zcount.ensure(64)) return -1;
  unsigned long long* zc = (unsigned long long*)b.zcount.p;
  HIP_TRY(hipMemsetAsync(zc, 0, sizeof(unsigned long long), st));
  rc::ParityWork w{};
  if (ensure_parity(*c, b, W, H, w, p.res_cus / p.lanes)) {
    std::fprintf(stderr, "Error: out of device memory for the parity workspace\n");
    return -1;
  }
  // phase C in the resolver lanes (off by default): it pays where the pixel partition is the
  // bound (reflection 2048^2 d4 8.2e9 -> 9.0e9 rays/s) and loses elsewhere (quadric 2048^2
  // 3.27e9 -> 2.83e9, 4096^2 6.28e9 -> 5.36e9, 8192^2 8.6e9 -> 5.8e9, simple 1024^2 d6 3.16e9
  // -> 2.98e9); mode 2 (no new batch once the lane's own work is over) does not change that
  const int pin = tune().pipe_inres;
  if (maxrec >= 3 && pin > 0) w.inres = pin;
  w.rstream = p.res[lane];
  w.pstream = first ? p.pix[p.fifo ? 0 : k] : nullptr;
  w.defer_c = p.fifo ? 1 : 0;
  w.adone = p.fifo ? p.adone[k] : nullptr;
  w.cstream = (p.fifo && !first && p.comp[p.total & 1]) ? p.comp[p.total & 1] : nullptr;
  w.rready = p.ready[k];
  w.rdone = p.done[k];
  const int e = (int)(p.submitted % Pipe::kEv);
  w.rt0 = p.rt_on ? p.rt[e][0] : nullptr;
  w.rt1 = p.rt_on ? p.rt[e][1] : nullptr;
  w.inject = take_inject();
  HIP_TRY(rc::launch_parity(ls, W, H, maxrec, d_out, w, zc, st, nullptr));
  if (p.fifo) {   // phase C after the resolver: at the next submit or rc_frames_wait
    p.cdefer = true;
    p.cdefer_lane = lane;
    p.cdefer_k = k;
    p.cdefer_W = W;
    p.cdefer_H = H;
    p.cdefer_maxrec = maxrec;
    p.cdefer_ls = ls;
    p.cdefer_w = w;
    p.cdefer_out = d_out;
    p.cdefer_zc = zc;
  } else if (p.log.enqueue(w.team, st)) {   // slot streams: the frame ends on its slot's stream
    return -1;
  }
  p.submitted++;
  p.frames++;
  p.total++;
  p.last = k;
  p.used[k] = true;
  return 0;
}

int rc_frames_wait(rc_timing* timing) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  Pipe& p = c->pipe;
  if (timing) std::memset(timing, 0, sizeof *timing);
  const int fl = p.init ? flush_phase_c(*c, tune().pipe_last_whole != 0) : 0;
  HIP_TRY(hipStreamSynchronize(c->stream));
  int rc = fl;
  if (p.init) {
    for (int k = 0; k < p.slots; ++k)
      if (p.pix[k]) HIP_TRY(hipStreamSynchronize(p.pix[k]));
    for (int r = 0; r < p.lanes; ++r) HIP_TRY(hipStreamSynchronize(p.res[r]));
    for (int r = 0; r < p.lanes; ++r)
      if (p.pc[r]) HIP_TRY(hipStreamSynchronize(p.pc[r]));
    for (int k = 0; k < p.slots; ++k) p.cpend[k] = false;
    // every frame since the last wait, from its latched hand-off words (FrameLog)
    if (p.log.drain() > 0) rc = -1;
    long long checked = 0, failed = 0;
    p.log.take(&checked, &failed);   // the window's frames, also those an earlier poll read
    if (failed > 0) rc = -1;
    if (timing) {
      timing->frames_checked = checked;
      timing->frames_failed = failed;
    }
    // the details of a failure from the last frame of each slot (the log already holds every
    // frame's words: without a failure in the window there is nothing to read back)
    for (int k = 0; failed > 0 && k < p.slots; ++k) {
      if (!p.used[k] || !p.fb[k].team.p) continue;
      if (report_spin_error(p.fb[k], "frames in flight")) rc = -1;
    }
    const int n = !p.rt_on ? 0 : p.submitted < Pipe::kEv ? (int)p.submitted : Pipe::kEv;
    double sum = 0.0, lo = 0.0, hi = 0.0;
    for (int e = 0; e < n; ++e) {
      const double ms = event_ms(p.rt[e][0], p.rt[e][1]);
      sum += ms;
      lo = (e == 0 || ms < lo) ? ms : lo;
      hi = ms > hi ? ms : hi;
    }
    if (n > 0) g_last_kernel_ms = sum / n;
    // the window's resolver record (rc_resolver_stats_get(0, ..))
    {
      const FrameLog::Diag d = p.log.diag_take();
      rc_resolver_stats& r = c->pipe_stats;
      std::memset(&r, 0, sizeof r);
      r.frames = d.frames;
      r.resolve_ms_min = lo;
      r.resolve_ms_max = hi;
      r.resolve_ms_mean = n > 0 ? sum / n : 0.0;
      fill_resolver_stats(*c, d, c->pipe_grid, c->pipe_res_cus, c->pipe_lds, c->pipe_team, &r);
    }
    if (timing && n > 0 && p.last >= 0) {
      timing->resolve_ms = sum / n;
      FrameBufs& b = p.fb[p.last];
      int cnt[4] = {0, 0, 0, 0};
      if (b.counters.p &&
          hipMemcpy(cnt, b.counters.p, sizeof cnt, hipMemcpyDeviceToHost) == hipSuccess)
        timing->dep_pixels = cnt[2];
      unsigned long long z = 0;
      if (hipMemcpy(&z, b.zcount.p, sizeof z, hipMemcpyDeviceToHost) == hipSuccess)
        timing->zero_normalize = (int64_t)z;
    }
  }
  p.frames = 0;
  p.submitted = 0;
  return rc;
}

int rc_pipe_reset(void) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  const int rc = rc_frames_wait(nullptr);
  std::lock_guard<std::mutex> lk(c->mu);
  pipe_release(*c);
  return rc;
}

int rc_lone_frames_check(int64_t* checked, int64_t* failed) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  // the lock first: a frame another thread enqueues after the synchronisation would otherwise
  // be drained while still pending (counted as never verified)
  std::lock_guard<std::mutex> lk(c->mu);
  if (flush_phase_c(*c, false)) return -1;   // a frame in flight's held-back phase C
  HIP_TRY(hipDeviceSynchronize());   // the frames ran on the callers' streams
  c->lone_log.drain();
  long long ch = 0, f = 0;
  c->lone_log.take(&ch, &f);
  if (checked) *checked = ch;
  if (failed) *failed = f;
  // the details of the device workspace's last frame (the failed one when the caller checks
  // after each frame): the spin that failed, the helper queue, the team's slots
  if (f && c->fb.team.p) (void)report_spin_error(c->fb, "the device workspace's last frame");
  return f ? -1 : 0;
}

int rc_resolver_stats_get(int lone, rc_resolver_stats* out) {
  if (!out) return -1;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!lone) {
    *out = c->pipe_stats;
    return 0;
  }
  c->lone_log.poll();   // the frames whose words have arrived
  std::memset(out, 0, sizeof *out);
  const FrameLog::Diag d = c->lone_log.diag_take();
  out->frames = d.frames;
  return fill_resolver_stats(*c, d, c->lone_grid, c->lone_res_cus, c->lone_lds, c->lone_team, out);
}

int rc_debug_inject_error(int nth_frame) {
  if (nth_frame < -1) return -1;
  g_inject = nth_frame;
  return 0;
}

// Test aid: the in-frame scatter (scatter_sweep) on the host alone, a writer thread standing in
// for phase C.  ndep DEP entries at increasing pixels (scan order); half the patch entries
// start with an earlier frame's mark; the writer stores this frame's entries in shuffled
// 64-entry batches, each batch's entries in a shuffled order (k_dep_chunks stores a batch in
// pieces), with pauses, then reports the frame complete.  skip > 0: entries j % skip == 0 are
// never stored (a frame that ended early: the sweep must still end, those pixels untouched);
// skip < 0: entries j % -skip == 0 are never stored and the frame reports a failure instead of
// completing.  Returns the number of pixmap bytes that differ from the expected image, or the
// sweep's failure status (< 0).
int rc_debug_scatter_selftest(int64_t ndep, int64_t seed, int skip) {
  if (ndep <= 0 || ndep > ((int64_t)1 << 24)) return -1;
  const size_t n = (size_t)ndep;
  std::mt19937_64 rng((uint64_t)seed);
  const size_t gap = skip > 0 ? (size_t)skip : skip < 0 ? (size_t)-(int64_t)skip : 0;
  std::vector<long long> pix(n);
  long long p = 0;
  for (size_t j = 0; j < n; ++j) {
    p += 1 + (long long)(rng() % 3);
    pix[j] = p;
  }
  std::vector<uint8_t> host(3 * ((size_t)p + 1), 0), want(host.size(), 0);
  std::vector<uint32_t> patch(n), colour(n);
  const uint32_t mark = rc::patch_mark(7), stale = rc::patch_mark(6);
  for (size_t j = 0; j < n; ++j) {
    colour[j] = (uint32_t)rng() & 0xFFFFFFu;
    patch[j] = (rng() & 1) ? (stale | ((uint32_t)rng() & 0xFFFFFFu)) : 0u;
    if (gap && j % gap == 0) continue;
    uint8_t* q = want.data() + 3 * (size_t)pix[j];
    q[0] = (uint8_t)colour[j];
    q[1] = (uint8_t)(colour[j] >> 8);
    q[2] = (uint8_t)(colour[j] >> 16);
  }
  const size_t nb = (n + kScatterBlock - 1) / kScatterBlock;
  std::vector<size_t> order(nb);
  for (size_t b = 0; b < nb; ++b) order[b] = b;
  std::shuffle(order.begin(), order.end(), rng);
  std::atomic<int> done{0};
  std::thread writer([&] {
    std::mt19937_64 wr((uint64_t)seed + 1);
    size_t idx[kScatterBlock];
    for (size_t i = 0; i < nb; ++i) {
      const size_t b0 = order[i] * kScatterBlock, cnt = std::min(kScatterBlock, n - b0);
      for (size_t k = 0; k < cnt; ++k) idx[k] = b0 + k;
      std::shuffle(idx, idx + cnt, wr);
      for (size_t k = 0; k < cnt; ++k) {
        const size_t j = idx[k];
        if (gap && j % gap == 0) continue;
        __atomic_store_n(&patch[j], mark | colour[j], __ATOMIC_RELEASE);
      }
      if (wr() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(wr() % 40));
    }
    done.store(skip < 0 ? -2 : 1, std::memory_order_release);
  });
  const int st = scatter_sweep(HostPool::get(0), host.data(), pix.data(), patch.data(), n, mark,
                               [&] { return done.load(std::memory_order_acquire); });
  writer.join();
  if (st != 0) return st;
  long long bad = 0;
  for (size_t i = 0; i < host.size(); ++i) bad += host[i] != want[i];
  return (int)std::min<long long>(bad, 1 << 30);
}

int rc_profile_begin(void) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  c->prof_active = 1;
  c->prof_calls = 0;
  return 0;
}

int rc_profile_end(rc_phase_stats* out) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  DevCtx* c;
  if (ctx_get(dev, &c)) return -1;
  c->prof_active = 0;
  std::memset(out, 0, sizeof *out);
  const int n = c->prof_calls < DevCtx::kEvSets ? c->prof_calls : DevCtx::kEvSets;
  out->calls = n;
  out->parity = c->prof_parity;
  for (int i = 0; i < n; ++i) {
    hipEvent_t* ev = c->ev[i];
    HIP_TRY(hipEventSynchronize(ev[c->prof_parity ? 4 : 1]));
    if (c->prof_parity) {
      out->phase_a_ms += event_ms(ev[0], ev[1]);
      out->compact_ms += event_ms(ev[1], ev[2]);
      out->resolve_ms += event_ms(ev[2], ev[3]);
      out->phase_c_ms += event_ms(ev[3], ev[4]);
      out->total_ms += event_ms(ev[0], ev[4]);
    } else {
      out->render_ms += event_ms(ev[0], ev[1]);
      out->total_ms += event_ms(ev[0], ev[1]);
    }
  }
  if (n > 0) {
    out->phase_a_ms /= n;
    out->compact_ms /= n;
    out->resolve_ms /= n;
    out->phase_c_ms /= n;
    out->render_ms /= n;
    out->total_ms /= n;
  }
  return 0;
}

int rc_render(const rc_scene* s, int W, int H, const rc_options* opt, uint8_t* pixmap,
              rc_timing* timing) {
  if (!s || !opt || !pixmap || W <= 0 || H <= 0) return -1;
  auto t0 = std::chrono::steady_clock::now();
  if (timing) std::memset(timing, 0, sizeof *timing);
  // one snapshot of the tuning for the whole call (rc_set_tuning may run concurrently)
  const rc_tuning tu = tune();
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  int G = opt->num_gpus;
  if (opt->device < 0 || opt->device >= ndev) {
    std::fprintf(stderr, "Error: device %d not available (%d devices)\n", opt->device, ndev);
    return -1;
  }
  // share_device: every rank on opt->device (device copies between the ranks: tests of the
  // multi-GPU entry on a one-GPU box); otherwise one device per rank
  const int avail = tu.share_device ? rc::kMaxShards : ndev - opt->device;
  if (G > avail || G > rc::kMaxShards || G > H) {
    const int want = G;
    if (G > avail) G = avail;
    if (G > rc::kMaxShards) G = rc::kMaxShards;
    if (G > H) G = H;
    static std::atomic<bool> warned{false};   // once per process, like the reference's notices
    if (!warned.exchange(true))
      std::fprintf(stderr,
                   "Warning: %d GPUs requested (RAYCAST_GPUS / num_gpus); rendering on %d (%d "
                   "devices from device %d, at most %d shards, %d rows)\n",
                   want, G, ndev - opt->device, opt->device, rc::kMaxShards, H);
  }
  const bool parity = opt->mode == RC_MODE_PARITY && opt->max_recursion > 1;
  const size_t row_bytes = (size_t)W * 3;
  if (G > 1) {   // row shards over RCCL (rc_shard.hip), the image on the first device
    // one sharded call at a time: d_image is the cached group's root buffer, which the next
    // caller's render would overwrite before this caller's copy-out
    static std::mutex group_call_mu;
    std::lock_guard<std::mutex> one_group_call(group_call_mu);
    uint8_t* d_image = nullptr;
    rc_timing tg;
    if (render_local_group(opt->device, G, tu.share_device != 0, s, W, H, opt, &d_image, &tg))
      return -1;
    DevCtx* c;
    if (hipSetDevice(opt->device) != hipSuccess || ctx_get(opt->device, &c)) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    prefault(*c, pixmap, (size_t)H * row_bytes, tu);
    auto td = std::chrono::steady_clock::now();
    if (copy_to_host(*c, pixmap, d_image, (size_t)H * row_bytes, c->stream, tu)) return -1;
    if (timing) {
      *timing = tg;
      timing->d2h_ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td).count();
      timing->total_ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    g_last_kernel_ms = tg.resolve_ms > 0.0 ? tg.resolve_ms : tg.kernel_ms;
    return 0;
  }
  // one device
  const int dev = opt->device;
  DevCtx* c;
  if (hipSetDevice(dev) != hipSuccess || ctx_get(dev, &c)) return -1;
  // the lock covers the workspace from its (re)allocation on: a concurrent caller's ensure()
  // could otherwise free the buffer another caller is rendering into
  std::lock_guard<std::mutex> lk(c->mu);
  // an earlier frame's failure (rc_render_device on another stream) is reported before this
  // frame is enqueued, as rc_render_device does, so the result below is this frame's own
  if (c->lone_log.earlier_failed()) {
    c->lone_log.take(nullptr, nullptr);
    return -1;
  }
  if (c->out.ensure((size_t)H * row_bytes)) return -1;
  uint8_t* d_out = (uint8_t*)c->out.p;
  // parity: the copy overlaps the resolver (copy_overlapped); split shading leaves the non-DEP
  // colours to phase C, so its framebuffer is not final after phase A
  const bool overlap = parity && !tu.split_shade && tu.overlap_d2h;
  uint32_t* patch = nullptr;
  const bool hpatch = overlap && tu.patch_host;
  size_t prev_dirty = 0;
  const unsigned epoch = next_epoch(c->fb.epoch);   // the frame's (ensure_parity assigns it)
  if (overlap) {
    if (!c->d2h && hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking) != hipSuccess) return -1;
    if (hpatch) {
      if (ensure_host_patch(*c, (size_t)W * H, epoch)) return -1;
      patch = c->host_patch_dev;
      // until the frame's DEP count is known (copy_overlapped), any entry may get a mark
      prev_dirty = c->host_patch_dirty;
      c->host_patch_dirty = (size_t)W * H;
    } else {
      if (c->patch.ensure((size_t)W * H * sizeof(uint32_t))) return -1;
      patch = (uint32_t*)c->patch.p;
    }
  }
  hipEvent_t* ev = nullptr;
  const long long own = c->lone_log.head;   // this frame's ring entry (parity frames log one)
  E2eTrace trace;
  trace.t0 = t0;
  struct Unset {
    ~Unset() { g_e2e = nullptr; }
  } unset;
  if (E2eTrace::on()) g_e2e = &trace;
  if (enqueue_render(*c, s, W, H, 0, 1, H, opt, d_out, c->stream, true, patch, &ev)) return -1;
  if (hpatch && c->fb.epoch != epoch) {   // the array's clearing assumed this epoch
    std::fprintf(stderr, "Error: rc_render: frame epoch %u, expected %u\n", c->fb.epoch, epoch);
    return -1;
  }
  // the frame's counts for rc_timing / raycast()'s stderr lines, behind its last kernel
  if (!c->pin_tail) HIP_TRY(hipHostMalloc((void**)&c->pin_tail, 64, hipHostMallocDefault));
  HIP_TRY(hipMemcpyAsync(c->pin_tail, c->fb.zcount.p, 8, hipMemcpyDeviceToHost, c->stream));
  if (parity)
    HIP_TRY(hipMemcpyAsync(c->pin_tail + 16, c->fb.counters.p, 16, hipMemcpyDeviceToHost,
                           c->stream));
  trace.mark(0);
  prefault(*c, pixmap, (size_t)H * row_bytes, tu);
  trace.mark(1);
  auto td = std::chrono::steady_clock::now();
  if (overlap) {
    if (copy_overlapped(*c, pixmap, d_out, (size_t)H * row_bytes, ev,
                        hpatch ? c->host_patch : nullptr, prev_dirty, tu))
      return -1;
  } else if (copy_to_host(*c, pixmap, d_out, (size_t)H * row_bytes, c->stream, tu)) {
    return -1;
  }
  // this frame's latched hand-off words: its own failure is reported by this call and
  // consumed; another stream's frame that failed meanwhile is left to the next call
  HIP_TRY(hipStreamSynchronize(c->stream));
  trace.mark(6);
  if (c->lone_log.entry_failed(own)) {
    c->lone_log.poll();
    (void)check_spin_error(c->fb, opt);   // the details, while the workspace still holds them
    c->lone_log.take(nullptr, nullptr);
    return -1;
  }
  c->lone_log.poll();
  if (timing) {
    fill_device_timing(*c, opt, timing, c->pin_tail);
    timing->d2h_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td).count();
    timing->total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  } else {
    fill_device_timing(*c, opt, nullptr, c->pin_tail);
  }
  trace.mark(7);
  trace.print();
  return 0;
}

static void consume_lists(json_data_t* js) {
  for (shape_t* p = js->shapes_list; p;) {
    shape_t* n = p->next;
    std::free(p);
    p = n;
  }
  for (light_t* p = js->lights_list; p;) {
    light_t* n = p->next;
    std::free(p);
    p = n;
  }
  js->shapes_list = nullptr;
  js->lights_list = nullptr;
}

// Drop-in for C/raycast.c:79-130.
void raycast(json_data_t* json_struct, PPMFormat photo_data) {
  rc_options opt;
  rc_default_options(&opt, 1);
  // The reference's main mallocs json_struct and zeroes num_shapes but not num_lights
  // (C/raycast.c:41-44): it relies on a fresh, zeroed heap chunk.  Linked against this library
  // the heap has been used before main (the HIP runtime), so the count can be garbage.  A count
  // above the list's length (which the reference would walk off the end of) or below zero is
  // taken as the list's length — what the zeroed chunk gives the reference — and written back,
  // so main's own report of the counts (C/raycast.c:66-67) is right too.
  {
    int ns = 0, nl = 0;
    for (const shape_t* p = json_struct->shapes_list; p; p = p->next) ++ns;
    for (const light_t* p = json_struct->lights_list; p; p = p->next) ++nl;
    if (json_struct->num_shapes < 0 || json_struct->num_shapes > ns) json_struct->num_shapes = ns;
    if (json_struct->num_lights < 0 || json_struct->num_lights > nl) json_struct->num_lights = nl;
  }
  rc_scene* s = rc_scene_create(json_struct);
  if (!s) {
    std::fprintf(stderr, "Error: could not flatten the scene lists\n");
    std::exit(1);
  }
  if (!rc_scene_parity_defined(s) && opt.mode == RC_MODE_PARITY)
    std::fprintf(stderr,
                 "Warning: the reference reads undefined memory for this scene "
                 "(phantom record, C/raycast.c:382); its output is not reproducible\n");
  // the reference consumes the lists (C/raycast.c:104-107)
  consume_lists(json_struct);
  if (photo_data.width <= 0 || photo_data.height <= 0) {   // the reference's loops do not run
    rc_scene_destroy(s);
    return;
  }
  rc_timing t;
  if (rc_render(s, photo_data.width, photo_data.height, &opt, photo_data.pixmap, &t)) {
    std::fprintf(stderr, "Error: GPU render failed\n");
    std::exit(1);
  }
  // C/v3math.c:183-187 prints one line per zero-length normalize
  for (int64_t k = 0; k < t.zero_normalize; ++k)
    std::fprintf(stderr, "v3_length returned 0, exiting program\n");
  if (const char* st = std::getenv("RAYCAST_STATS")) {
    if (st[0] == '1')
      std::fprintf(stderr,
                   "{\"rays_per_s\": %.1f, \"total_ms\": %.3f, \"kernel_ms\": %.3f, "
                   "\"resolve_ms\": %.3f, \"d2h_ms\": %.3f, \"dep_pixels\": %lld, "
                   "\"mode\": \"%s\", \"gpus\": %d}\n",
                   (double)photo_data.width * photo_data.height / (t.total_ms * 1e-3),
                   t.total_ms, t.kernel_ms, t.resolve_ms, t.d2h_ms, (long long)t.dep_pixels,
                   opt.mode == RC_MODE_FAST ? "fast" : opt.mode == RC_MODE_CUDA ? "cuda" : "parity",
                   opt.num_gpus);
  }
  rc_scene_destroy(s);
}

}  // extern "C"
