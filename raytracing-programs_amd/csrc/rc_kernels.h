// rc_kernels.h — launch interface between the host runtime (rc_api.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "rc_scene.h"

namespace rc {

// Device view of an uploaded packed scene (rc_scene.h).
struct LaunchScene {
  const rc_shape* shapes;
  const rc_light* lights;
  const rc_shade_pair* pairs;
  int n, m;
  float cam_w, cam_h;
  unsigned long long refl_mask;   // bit k: shape k reflective (n <= 64)
  int has_quadric;                // the scene has a quadric (2: none with cross terms, quad_x0)
  int o0_ok;                      // primary rays may use rc_shape::o0
  int dep_fast;                   // clean DEP entries take phase A's primary shade (Scene)
};

// Parity-mode workspace (device pointers), sized for W*H pixels.
struct ParityWork {
  uint8_t* cls;             // [P]   pixel class (ident / writer / dep)
  float4* wcarry;           // [P]   writer carry-out
  void* deprec;             // [P]   DepRec (phase A -> B/C)
  void* row_stats;          // [H]   RowStats (k_row_stats)
  int* row_off;             // [H]   DEP offset of each row
  int* row_soff;            // [H]   segment offset of each row
  long long* row_prevw;     // [H]   last writer pixel before each row (-1: none)
  long long* row_prevd;     // [H]   last DEP pixel before each row (-1: none)
  long long* dep_pix;       // [P]   DEP pixels in scan order
  long long* seg_key;       // [P]   per segment: the writer pixel before it (-1: none)
  int* seg_start;           // [P]   segment starts, in scan order
  void* cin;                // [P]   resolved carry-in per DEP entry (CinG tagged granules)
  int* counters;            // [16]  nseg, head, ndep, ordered, phase-C tickets, census, ...
  int* batch_state;         // [P/64+1] phase-C batch claim words (0 free, 1 claimed)
  int* batch_cnt;           // [P/64+1] entries of each batch with a published carry-in
  int* batch_rq;            // [P/64+1] batches in the order they became complete (+1; 0 empty)
  hipStream_t side;         // phase C's side stream (null: phase C after the resolver only)
  hipEvent_t fork, join;    // side stream waits on fork; the main stream waits on join
  int side_blocks;          // resident k_side workgroups
  int side_lds;             // k_side's dynamic LDS reservation (keeps it off resolver CUs)
  int split_shade;          // k_classify + colours in k_side (measured slower: off by default)
  unsigned epoch;           // this frame's carry-in tag (never 0)
  int* seg_order;           // [kSegOrderMax] segments longest first (k_seg_order)
  void* team;               // TeamState of the long-segment team
  int resolve_blocks;       // persistent resolver grid (<= resident capacity)
  int resolve_lds;          // dynamic LDS per resolver block (occupancy control)
  int team_blocks;          // workgroups in the long-segment team (0: no team)
  int helpers;              // workgroups taking handed-off dense runs (0: none)
  int hand_run;             // changes in a row before a regular wave hands its run off
  int long_len;             // segments with >= long_len entries go to the team
  int phase_c_blocks;       // grid-stride phase C grid
  int phase_c_finish;       // phase C after the resolver through k_finish's claims (RC_PHASE_C_FINISH)
  int wave_k;               // clean cooperative steps before a wave window goes back to LANE
  int resolve_k;            // the same for the team leader's block window
  int resolve_clean;        // clean windows in a row that end a RESOLVE round
  int team_cscan;           // cooperative SCAN rounds after RESOLVE rounds (early hand-back)
  int coop_group;           // lanes per entry of the cooperative evaluator (0: off)
  unsigned* trace;          // optional [2*nseg] per-segment {ticks, evals} (debug)
  // Pipelined frames (rc_frame_submit): the resolver runs on its own stream (a CU partition
  // of its own) between two hand-off events; null rstream = everything on the main stream.
  hipStream_t rstream;
  hipStream_t pstream;      // phase C's stream (null: the main stream)
  hipEvent_t rready, rdone; // main -> rstream after compaction; rstream -> pstream after it
  hipEvent_t rt0, rt1;      // optional: resolver start / end on rstream
  hipEvent_t adone;         // optional: recorded after phase A (pipelined phase A order)
  hipStream_t cstream;      // optional (with adone): compaction on this stream after adone
  uint32_t* patch;          // optional [P] packed RGB of DEP entry j (rc_render's overlapped copy)
  int defer_c;              // pipelined: launch_parity stops after the resolver; phase C is
                            // enqueued later by launch_phase_c (after rdone)
  int inject;               // test aid: the resolver raises its error word (code 4) at start
  int batch_ints;           // ints from batch_state on (claims, counts, queue), cleared by k_row_stats
  int inres;                // phase C inside the resolver: its waves shade ready batches once
                            // their own work is done (rc_tuning.side 3)
  int block_min;            // regular segments of >= block_min entries get a whole workgroup
  int headb_first;          // regular workgroups that start on the per-wave queue (head B) at once
};

constexpr int kSegOrderMax = 65536;   // segments ordered for the resolver queue (else FIFO)
constexpr int kCinBytes = 24;         // one carry-in = three tagged 8-byte granules
constexpr int kLdsShapesMax = 64;     // k_resolve stages up to this many shapes in LDS
constexpr int kDenseSlots = 64;       // k_resolve's hand-off ring (helper workgroups at most)

// cuda_sem: RC_MODE_CUDA (the CUDA port's arithmetic, rc_cudasem.hpp) instead of fast mode
hipError_t launch_render(const LaunchScene& s, int W, int H, int row0, int row_step, int nrows,
                         int maxrec, uint8_t* out, unsigned long long* zcount,
                         hipStream_t stream, bool cuda_sem = false);

hipError_t launch_parity(const LaunchScene& s, int W, int H, int maxrec, uint8_t* out,
                         const ParityWork& w, unsigned long long* zcount, hipStream_t stream,
                         const hipEvent_t* ev);

// Top byte of a colour-patch entry (ParityWork::patch) once phase C has stored it: the frame's
// mark, 0x80 | (epoch & 0x7f) of its carry-in epoch (never 0, the cleared value); the low three
// bytes are R, G, B.  rc_render's host side
// only reads the array during a frame (an entry is this frame's once its top byte is this
// frame's mark) and never stores to it then: a host store into a line that phase C is still
// writing in pieces (k_dep_chunks) was seen undone by the device's later store to that line,
// leaving a stale mark (round 6, profiles/r06n_patch_marks.txt).  Marks of kPatchMarks
// consecutive epochs are distinct, so the array is cleared once per kPatchMarks epochs
// (ensure_host_patch).
constexpr unsigned kPatchMarks = 128;
__host__ __device__ constexpr uint32_t patch_mark(unsigned epoch) {
  return (epoch << 24) | 0x80000000u;
}

// Phase C of a frame launched with defer_c: waits for w.rdone on `stream`.
hipError_t launch_phase_c(const LaunchScene& s, int W, int H, int maxrec, uint8_t* out,
                          const ParityWork& w, unsigned long long* zcount, hipStream_t stream);

// Row shards (rc_shard.hip; wire formats in rc_kernels.hip).  kMaxShards ranks at most.
constexpr int kMaxShards = 16;
size_t shard_entry_bytes();   // one DEP entry on the wire
size_t shard_row_bytes();     // one row summary on the wire
// A rank: phase A on rows row0 + k*row_step (k < nrows) into rank-local buffers, the local
// DEP list (w.dep_pix, local pixels; w.counters[2] = entries) and the wire entries / rows.
// img_rec / img_wcarry (the root): DEP lines and writer carries go straight to the root
// resolver's image-indexed buffers and its entries are thin {image pixel, writer} pairs.
hipError_t launch_shard_local(const LaunchScene& s, int W, int H, int row0, int row_step,
                              int nrows, int maxrec, uint8_t* out, const ParityWork& w,
                              void* ent, void* rows, unsigned long long* zcount,
                              hipStream_t stream, void* img_rec = nullptr,
                              float4* img_wcarry = nullptr);
// The root: image scan order from the gathered rows ([G][rmax]) and entries (rank g's at
// offs[g]) in a lone frame's layout (pixel-indexed records, primary shades and writer carries
// in w.deprec / w.wcarry, which hold W*H + 1 pixels: the last is a spare for entries beyond a
// fixed-size exchange's bound), the carry resolver with phase C inside it (w.inres) and the
// phase C tail, shading every DEP entry into `out` (W*H + 1 pixels; its non-DEP pixels are the
// gathered row blocks).  ev (optional): [0] resolver start, [1] resolver end.  bound: entries
// delivered per rank (the fixed-size exchange; beyond it a rank's list is not read as records).
// ent0 (optional): rank 0's entries, read in place (the root's own list is not gathered).
hipError_t launch_shard_resolve(const LaunchScene& s, int W, int H, int G, int rmax,
                                const void* rows_all, const void* ent_all, const void* ent0,
                                const long long* offs, int maxrec, const ParityWork& w,
                                uint8_t* out, unsigned long long* zcount, hipStream_t stream,
                                const hipEvent_t* ev, int bound = 0x7fffffff, int thin0 = 0);
// The root: image <- gathered row blocks [G][rmax][W*3]; block0 (optional): rank 0's block in
// place of gathered[0] (the root's own rows are not copied).
hipError_t launch_deinterleave(const uint8_t* gathered, const uint8_t* block0, int G, int rmax,
                               int W, int H, uint8_t* img, hipStream_t stream);

size_t deprec_bytes();
size_t row_stats_bytes();
size_t team_state_bytes();
size_t team_dq_offset();   // DenseQueue {prod, claim, finished} inside TeamState
size_t team_slot_offset(); // the team's hand-off slots: [team_slot_bufs()][team_slot_blocks()]
int team_slot_bufs();      //   x 4 tagged granules {payload, round}
int team_slot_blocks();
size_t team_handoff_diag_offset();   // 0 unless an RC_HANDOFF_DIAG build
int resolve_blocks_resident(int cus, int lds_bytes);
// k_resolve<true>'s resources: registers per lane (VGPRs + AGPRs), scratch bytes per lane, and
// the workgroups one CU can hold with `lds_bytes` of dynamic LDS each (occupancy API).
int resolve_resources(int lds_bytes, int* regs, int* scratch, int* wg_per_cu);
int side_lds_bytes(int resolve_dyn_lds);
int phase_c_side_blocks(int cus, int side_lds);

}  // namespace rc
