// rc_runtime.h — internal host-runtime state of libraycast_hip.so shared by rc_api.hip (one
// device: rc_render, frames in flight) and rc_shard.hip (row shards over several devices).
// Not part of the C-ABI (include/raycast_hip.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <mutex>

#include "raycast_hip.h"
#include "rc_kernels.h"
#include "rc_scene.h"

namespace rcrt {

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "Error: HIP call failed: %s (%s) at %s:%d\n", #expr,        \
                   hipGetErrorString(e_), __FILE__, __LINE__);                          \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)

constexpr int kMaxDevices = 16;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, need) != hipSuccess) return -1;
    bytes = need;
    return 0;
  }
};

// One frame's device state: the uploaded scene, the zero-normalize counter and the parity
// workspace.  The plain path has one (DevCtx::fb); pipelined frames alternate two (Pipe).
struct FrameBufs {
  unsigned epoch = 0;   // carry-in tag of the last parity frame in this workspace
  DevBuf zcount;        // zero-normalize counter
  DevBuf scene;         // uploaded packed scene
  const void* scene_src = nullptr;   // host image last uploaded
  DevBuf cls, wcarry, deprec, rows, dep_pix, seg_key, seg_start, seg_order, batch_state, cin,
      counters, team, trace;
};

// Per-frame verification of parity frames.  A frame's carry hand-offs (the resolver team's
// granules, phase C's carry-ins, the helper queue) are bounded spins that record the first
// failure in the frame's TeamState (rc_kernels.hip); the next frame in the same workspace
// resets that state.  So after every parity frame's last kernel the TeamState's first four
// words are copied, on the frame's own stream, into a pinned ring entry the host pre-filled
// with kPending: once the copy has run the entry holds 0 (every hand-off completed) or the
// failure's code, workgroup and details.  The copy precedes the event that gates the
// workspace's next use, so no later frame can erase a failure before the host has read it.
struct FrameLog {
  static constexpr int kRing = 4096;
  static constexpr int kPending = 0x7fffffff;
  struct Entry {
    int code, block, info, info2;   // TeamState.error, err_block, err_info, err_info2
    int rq_prod, rq_cons, helpers_out;
    int n_scan, n_cscan, n_resolve; // the frame's team rounds by kind
    int spin_ticks[4];              // its longest bounded waits per spin site (10 ns ticks)
    int clock_mhz;                  // shader clock over its resolver's run (0: not measured)
    int team_row;                   // TeamState::team_row: 1 + last row of a long segment
  };
  // Frame diagnostics of the entries read back since the last diag_take(): frames, the most
  // team rounds of each kind in one frame, the longest wait per spin site.
  struct Diag {
    long long frames = 0;
    int scan_max = 0, cscan_max = 0, resolve_max = 0;
    int spin_ticks_max[4] = {0, 0, 0, 0};
    int clock_min = 0, clock_max = 0;   // MHz, over the frames that measured it
  };
  Diag diag;
  Entry* ring = nullptr;     // pinned host memory, kRing entries
  long long head = 0;        // frames logged
  long long tail = 0;        // frames whose entry has been read back (in order)
  long long checked = 0;     // entries read back since the last take()
  long long failed = 0;      // of them, frames whose hand-off failed
  const char* what = "";
  // Log the frame whose TeamState is `team` (device) on `st`, after its last kernel.
  int enqueue(const void* team, hipStream_t st);
  // Read back the entries whose copy has run (in order, stopping at the first still
  // pending); reports each failure on stderr.  Returns the failures found.
  long long poll();
  // After the frames' streams are synchronised: every entry must have run (a pending one
  // counts as a failure).  Returns the failures found.
  long long drain();
  // A failure read back now or earlier and not yet taken (poll() first).
  bool earlier_failed();
  // Entry k (a frame's index at its enqueue) has run and its hand-off failed.  Only for an
  // entry whose stream has been synchronised and that poll() has not read back yet.
  bool entry_failed(long long k) const;
  // checked / failed since the last take(), then reset.
  void take(long long* c, long long* f);
  // the diagnostics since the last diag_take(), then reset
  Diag diag_take() {
    Diag d = diag;
    diag = Diag{};
    return d;
  }
};

// Pipelined parity frames (rc_frame_submit).  The device's CUs are split in two partitions
// (hipExtStreamCreateWithCUMask).  Partition A runs the carry resolvers: kLanes resolver
// streams, each resolver grid sized to A/kLanes CUs (one workgroup per CU), so the resolvers in
// flight are always wholly resident side by side (a team spins on co-resident workgroups;
// at most kLanes resolvers are in flight since each stream runs its resolvers in order).
// Partition B runs the pixel phases: the frames' phase A one at a time in submission order
// (each waits for the previous frame's, adone), so the frame whose resolver comes next always
// has the whole partition; two streams (pix[0], pix[1]) alternate so a frame's compaction —
// a chain of small latency-bound kernels — overlaps the next frame's phase A; each lane's
// phase C runs on a stream of its own (pc[lane], after the frame's resolver); a slot's next
// phase A waits for the slot's previous phase C (cdone).  A resolver is
// latency-bound (its carry chains), so overlapping kLanes of them multiplies the frame rate
// until partition B's pixel work becomes the bound.  (RC_PIPE_SLOTSTREAMS: the earlier form,
// one stream per slot running A, compaction and C in turn.)
struct Pipe {
  static constexpr int kSlots = 8;   // frame workspaces (a frame re-uses slot k after k's end)
  static constexpr int kLanes = 4;   // resolvers in flight (at most)
  bool init = false;
  int res_cus = 0;                   // CUs in partition A
  int lanes = 2;                     // resolver streams in use (RC_PIPE_RESOLVERS)
  int slots = 4;                     // workspaces / pixel streams in use (RC_PIPE_SLOTS)
  hipStream_t pix[kSlots] = {}, res[kLanes] = {};
  hipStream_t comp[2] = {};          // compaction: no CU mask, highest priority (comp_stream)
  hipEvent_t ready[kSlots] = {}, done[kSlots] = {};
  bool fifo = true;                  // pa = pix[0] + pc[] (false: RC_PIPE_SLOTSTREAMS)
  hipStream_t pc[kLanes] = {};
  hipStream_t spare[2] = {};         // pipe_order 3/4: placeholders that keep a queue per lane
  bool pc_shared = false;            // pipe_order 4: both lanes' phase C on one stream (pc[0])
  hipEvent_t cdone[kSlots] = {};
  bool cpend[kSlots] = {};           // slot k's phase C is enqueued and not yet synchronised
  hipEvent_t adone[kSlots] = {};     // after slot k's phase A
  static constexpr int kEv = 64;     // resolver timing events of the last kEv frames
  hipEvent_t rt[kEv][2] = {};
  FrameBufs fb[kSlots];
  long long submitted = 0;           // parity frames since the last rc_frames_wait
  long long frames = 0;              // frames of any mode since the last rc_frames_wait
  long long total = 0;               // parity frames ever (slot / stream rotation)
  long long last = -1;               // slot of the last parity frame
  bool used[kSlots] = {};
  bool rt_on = true;                 // resolver timing events recorded (RC_PIPE_NO_RT: off)
  int built_lanes = 0, built_slots = 0, built_res = 0, built_order = 0;   // the tuning it was built with
  FrameLog log;                      // every pipelined parity frame, in submission order
  // the last submitted parity frame's phase C: launched at the next submit (on its lane's
  // phase C stream) or by rc_frames_wait (on every CU: nothing else is left to run beside it)
  bool cdefer = false;
  int cdefer_lane = 0, cdefer_k = 0, cdefer_W = 0, cdefer_H = 0, cdefer_maxrec = 0;
  rc::LaunchScene cdefer_ls{};
  rc::ParityWork cdefer_w{};
  uint8_t* cdefer_out = nullptr;
  unsigned long long* cdefer_zc = nullptr;
};

struct DevCtx {
  bool init = false;
  int device = 0;
  hipStream_t side = nullptr;   // phase C's side stream
  hipEvent_t fork = nullptr, join = nullptr;
  int side_blocks = 0, side_lds = 0;
  int side_for_lds = -1;        // the resolver LDS reservation side_lds / side_blocks were sized for
  int cus = 256;
  hipStream_t stream = nullptr;
  // event sets: [0] start, then per phase ends (fast: [1] = render; parity: [1] phase A,
  // [2] compaction, [3] resolver, [4] phase C).  Set 0 serves plain calls; inside an
  // rc_profile_begin/end window every call takes the next set of the pool.
  static constexpr int kEvSets = 64;
  hipEvent_t ev[kEvSets][5] = {};
  int prof_active = 0, prof_calls = 0, prof_parity = 0;
  DevBuf out;          // rc_render output pixmap
  uint8_t* stage[2] = {nullptr, nullptr};   // pinned bounce buffers of copy_to_host
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  FrameBufs fb;        // scene, counter and parity workspace of the plain path
  Pipe pipe;
  int resident_blocks = 0;
  int resident_lds = -1;
  static constexpr int kResCache = 4;   // resident resolver grids per LDS reservation
  int res_lds[kResCache] = {};
  int res_blocks[kResCache] = {};
  size_t parity_pixels = 0;
  int parity_rows = 0;
  // rc_render's overlapped copy (parity): the framebuffer leaves on `d2h` while the resolver
  // runs, then only the DEP entries' colours (`patch`, packed RGB per entry) follow
  hipStream_t d2h = nullptr;
  DevBuf patch;
  uint8_t* pin_pix = nullptr;     // pinned: DEP pixel indices (int64 per entry)
  uint8_t* pin_patch = nullptr;   // pinned: DEP entries' packed RGB
  size_t pin_bytes = 0;           // capacity of each pinned buffer, in entries
  int* pin_cnt = nullptr;         // pinned: counters[0..3]
  uint8_t* pin_tail = nullptr;    // pinned: rc_render's frame counts (fill_device_timing)
  uint32_t* host_patch = nullptr;     // pinned, mapped: phase C's packed RGB per DEP entry
  uint32_t* host_patch_dev = nullptr; // its device address (patch_host)
  size_t host_patch_entries = 0;
  size_t host_patch_dirty = 0;       // entries below it may hold a mark since the last clear
  unsigned host_patch_epoch0 = 0;    // epoch before the first frame since that clear
  FrameLog lone_log;   // every parity frame rendered in `fb` (rc_render, rc_render_device)
  // rc_resolver_stats: the last rc_frames_wait window's record (frames in flight), and the
  // resolver placement of the last frame of each kind (grid, CUs it may use)
  rc_resolver_stats pipe_stats{};
  int lone_grid = 0, lone_res_cus = 0, lone_lds = 0, lone_team = 0;
  int pipe_grid = 0, pipe_res_cus = 0, pipe_lds = 0, pipe_team = 0;
  // `fb` is shared by every one-frame-at-a-time call on this device, and rc_render_device
  // returns before its frame has run: the next enqueue on `fb` from another stream waits for
  // the previous one (ws_ev, recorded after it on ws_stream).
  hipEvent_t ws_ev = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_valid = false;
  // One render at a time per device: the workspace, TeamState, events and streams above are
  // shared by every call on this device (rc_render, rc_render_device, rc_frame_submit).
  std::mutex mu;
};

extern DevCtx g_ctx[kMaxDevices];

// process-wide schedule tuning (rc_set_tuning; defaults = the product's schedule): a copy
// taken under the tuning lock, so a render reads one consistent set of fields
rc_tuning tune();
int ctx_get(int device, DevCtx** out);
int fill_resolver_stats(DevCtx& c, const FrameLog::Diag& d, int grid, int res_cus, int lds,
                        int team, rc_resolver_stats* r);
// the host-side copy helpers take the caller's one tuning snapshot (rc_render)
int copy_to_host(DevCtx& c, uint8_t* host, const uint8_t* dev, size_t bytes, hipStream_t st,
                 const rc_tuning& tu);
int ensure_host_patch(DevCtx& c, size_t entries, unsigned epoch);
void prefault(DevCtx& c, uint8_t* p, size_t n, const rc_tuning& tu);
int upload_scene(FrameBufs& b, hipStream_t stream, const rc_scene* s, rc::LaunchScene& ls);
int ensure_parity(DevCtx& c, FrameBufs& b, int W, int H, rc::ParityWork& w, int res_cus,
                  int piped_lane = -1);
int report_spin_error(const FrameBufs& b, const char* where);
double event_ms(hipEvent_t a, hipEvent_t b);
// One render of rows row0 + k*row_step into d_out on `stream` through the device's one-frame
// workspace (rc_render_device's path; the caller holds c.mu).  timed: phase events c.ev[0].
int enqueue_render(DevCtx& c, const rc_scene* s, int W, int H, int row0, int row_step, int nrows,
                   const rc_options* opt, uint8_t* d_out, hipStream_t stream, bool timed,
                   uint32_t* patch = nullptr, hipEvent_t** evset = nullptr);
int check_spin_error(FrameBufs& b, const rc_options* opt);
void fill_device_timing(DevCtx& c, const rc_options* opt, rc_timing* t,
                        const uint8_t* tail = nullptr);
// rc_shard.hip: rc_render's multi-GPU path (a cached in-process group over devices
// first..first+n-1, or n ranks sharing device `first` with device copies between them when
// `share`); *d_image = the root's de-interleaved image.  The caller holds no lock.
int render_local_group(int first, int n, bool share, const rc_scene* s, int W, int H,
                       const rc_options* opt, uint8_t** d_image, rc_timing* timing);

}  // namespace rcrt

// the packed scene behind the opaque rc_scene handle
struct rc_scene {
  rc_packed_header* img;   // host packed image
};
