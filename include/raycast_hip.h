/*
 * raycast_hip.h — C-ABI of the MI355X raycast library (libraycast_hip.so).
 *
 * Drop-in boundary: the reference's render entry point
 *     void raycast(json_data_t *json_struct, PPMFormat photo_data);   // C/raycast.h:8
 * is exported with the identical signature and by-value PPMFormat, so the reference's
 * own main (C/raycast.c:19-69) links against this library instead of C/raycast.c.
 *
 * The record layouts below are byte-identical to the reference's:
 *   shape_t  (104 B)  C/objects.h:15-49
 *   light_t  ( 72 B)  C/objects.h:51-61
 *   json_data_t       C/parse.h:11-18
 *   PPMFormat         C/ppm.h:6-12
 * They sit behind the reference's own include guards (objects_h, parse_h, ppm_h): include
 * the reference headers FIRST if both are used in one translation unit.
 *
 * Everything beyond raycast() is an extension: explicit options (mode, bounce depth, GPU
 * count), a reusable packed scene, and device-resident rendering for benchmarks and the
 * multi-GPU driver.  No torch types cross this boundary: plain pointers and sizes only.
 */
#ifndef RAYCAST_HIP_H
#define RAYCAST_HIP_H

#include <stdio.h>
#include <stdint.h>
#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference record layouts (ABI) ------------------------------------------------- */
#ifndef objects_h
#define objects_h
typedef enum { SPHERE, PLANE, QUADRIC } shape_type_t;        /* C/objects.h:4-8   */
typedef enum { POINT, SPOTLIGHT } light_type_t;               /* C/objects.h:10-13 */

typedef struct shape_t {                                      /* C/objects.h:15-49 */
  float diffuse_color[3];
  float specular_color[3];
  float position[3];
  float reflectivity;
  float refractivity;
  float ior;
  union {
    struct { float normal[3]; };                              /* plane   */
    struct { float radius; };                                 /* sphere  */
    struct { float a, b, c, d, e, f, g, h, i, j; };           /* quadric */
  };
  shape_type_t type;
  struct shape_t *next;
} shape_t;

typedef struct light_t {                                      /* C/objects.h:51-61 */
  float position[3];
  float color[3];
  float radial_coef[3];
  float theta;
  float cos_theta;
  float a0;
  float direction[3];
  light_type_t type;
  struct light_t *next;
} light_t;

/* list builders of the host front end (same names/semantics as C/objects.c:20-221) */
shape_t *add_new_sphere(shape_t *head, float *diffuse, float *specular, float *position,
                        float radius, float reflectivity, float refractivity, float ior);
shape_t *add_new_plane(shape_t *head, float *diffuse, float *specular, float *position,
                       float *normal, float reflectivity);
shape_t *add_new_quadric(shape_t *head, float *diffuse, float *specular, float a, float b,
                         float c, float d, float e, float f, float g, float h, float i,
                         float j, float reflectivity);
shape_t *free_shape_list(shape_t *head);
light_t *free_light_list(light_t *head);
light_t *add_new_spot_light(light_t *head, float *color, float *position, float theta,
                            float a0, float *direction, float *radial_coef);
light_t *add_new_point_light(light_t *head, float *color, float *position, float *radial_coef);
#endif

#ifndef parse_h
#define parse_h
typedef struct json_data_t {                                  /* C/parse.h:11-18 */
  float camera_width;
  float camera_height;
  shape_t *shapes_list;
  light_t *lights_list;
  int num_shapes;
  int num_lights;
} json_data_t;

/* scene front end (same grammar, messages and exit(1) behaviour as C/parse.c:13-436) */
void parse_json(FILE *json, json_data_t *json_data);
void set_to_black(float *input);
#endif

#ifndef ppm_h
#define ppm_h
typedef struct PPMFormat {                                    /* C/ppm.h:6-12 */
  int width, height, size;
  uint8_t maxColor;
  uint8_t depth;
  char *tupleType;
  uint8_t *pixmap;
} PPMFormat;

void ppm_WriteOutP3(PPMFormat inData, FILE *outFile);        /* C/ppm.c:168-184 */
float ppm_clamp(float value, float lower_bound, float upper_bound);  /* C/ppm.c:350-359 */
#endif

_Static_assert(sizeof(shape_t) == 104, "shape_t must match C/objects.h layout");
_Static_assert(sizeof(light_t) == 72, "light_t must match C/objects.h layout");

/* ---- drop-in entry point ------------------------------------------------------------ */

/* Replaces C/raycast.c:79-130.  Consumes both lists exactly like the reference
 * (C/raycast.c:104-107: frees them; num_shapes/num_lights stay valid; the list pointers are
 * left NULL instead of dangling).  Writes every byte of photo_data.pixmap (W*H*3, RGB,
 * row-major, top row first).  Options come from the environment:
 *   RAYCAST_MODE   = parity (default) | fast
 *   RAYCAST_DEPTH  = bounce depth d, MAX_RECURSION = d+1 (default 6 == C/raycast.c:14)
 *   RAYCAST_GPUS   = number of GPUs for row-cyclic sharding over RCCL (default 1; both modes)
 *   RAYCAST_DEVICE = first HIP device ordinal (default 0)
 *   RAYCAST_STATS  = 1: one JSON metrics line on stderr
 * Any HIP failure prints a message to stderr and exit(1)s (reference error convention). */
void raycast(json_data_t *json_struct, PPMFormat photo_data);

/* ---- extended API ------------------------------------------------------------------- */

enum { RC_MODE_PARITY = 0,  /* byte-identical to gcc -O3 C/raycast.c (scan-order carry)   */
       RC_MODE_FAST   = 1,  /* reflection miss ends the bounce loop (CUDA/raycast.cu:224-237) */
       RC_MODE_CUDA   = 2   /* the CUDA port's semantics: fast's control flow, powf-on-float
                               arithmetic (CUDA/raycast.cu:455-634, v3math.cu:168), 50 bounces
                               by default (MAX_ITER, CUDA/raycast.cu:13); parity unpinned */ };

typedef struct rc_options {
  int max_recursion;   /* C/raycast.c:14 MAX_RECURSION; bounce depth = max_recursion - 1 */
  int mode;            /* RC_MODE_* */
  int num_gpus;        /* >= 1 */
  int device;          /* first device ordinal */
} rc_options;

typedef struct rc_timing {
  double total_ms;       /* whole call, host wall clock                                 */
  double kernel_ms;      /* sum of kernel spans (HIP events)                            */
  double resolve_ms;     /* parity: carry-chain resolution span                        */
  double d2h_ms;         /* device -> host copy of the pixmap                          */
  int64_t dep_pixels;    /* parity: pixels whose first reflection missed               */
  int64_t zero_normalize;/* count of zero-length normalize events (C/v3math.c:183-187) */
  int64_t frames_checked;/* parity frames whose hand-off words were read back: rc_frames_wait
                            (every frame since the previous wait), rc_render_device with
                            timing (1)                                                  */
  int64_t frames_failed; /* of them, frames whose carry hand-off failed (image invalid)  */
} rc_timing;

/* Fill *opt with the defaults (then the RAYCAST_* environment overrides if use_env). */
void rc_default_options(rc_options *opt, int use_env);

/* Opaque packed scene: flattened shape/light arrays + the out-of-bounds "phantom" record
 * the reference reads as shapes_list[-1] (C/raycast.c:382).  Does NOT consume the lists. */
typedef struct rc_scene rc_scene;
rc_scene *rc_scene_create(const json_data_t *json_struct);
void rc_scene_destroy(rc_scene *scene);
/* 1 when the reference output is well defined for this scene (phantom reads only defined
 * bytes or is black), 0 when the reference itself is run-to-run nondeterministic. */
int rc_scene_parity_defined(const rc_scene *scene);

/* Render W x H into a host pixmap (W*H*3 bytes).  Returns 0 on success. */
int rc_render(const rc_scene *scene, int width, int height, const rc_options *opt,
              uint8_t *pixmap, rc_timing *timing);

/* Device-resident render on the current device: rows row0, row0+row_step, ... (nrows rows)
 * of a W x H image into d_out (nrows*W*3 bytes, device memory, compact row order) on the
 * given HIP stream (NULL = default stream).  Parity mode requires row0=0,row_step=1,nrows=H.
 * Asynchronous unless timing is requested.  Returns 0 on success. */
int rc_render_device(const rc_scene *scene, int width, int height, int row0, int row_step,
                     int nrows, const rc_options *opt, uint8_t *d_out, void *stream,
                     rc_timing *timing);

/* Frames in flight (an extension for rendering frame sequences; no reference
 * counterpart).  rc_frame_submit enqueues one whole W x H image of `scene` into d_out
 * (W*H*3 bytes, device memory, ready for use: synchronise the stream that produced it
 * first) and returns.  It is byte-identical to rc_render_device's.  In parity mode up to
 * two frames are in flight on the current device.  The device's CUs are split in two
 * partitions (hipExtStreamCreateWithCUMask; RC_PIPE_RES_CUS sets the resolver's share).
 * One runs the frames' carry resolvers in submission order.  The other runs the next frame's
 * phase A and compaction and the previous frame's phase C beside it.  A frame then costs
 * about its resolver's time instead of the sum of its phases.  Fast mode (no serial stage)
 * renders the frames back to back on the whole device.
 * Completion: rc_frames_wait is the only completion point for submitted parity frames.  The
 * last submitted frame's phase C is held back until the next rc_frame_submit (on its lane's
 * stream) or rc_frames_wait (on every CU), so synchronising a stream or the device after
 * rc_frame_submit does NOT complete that frame: its DEP pixels may still hold phase A's
 * bytes.  rc_lone_frames_check, rc_render_device and rc_render launch a pending phase C
 * first, so a later device synchronisation completes it; rc_pipe_reset waits for it.
 * rc_frames_wait blocks until every
 * submitted frame is complete.  It reports a failed resolver hand-off (returns -1) and fills
 * *timing (may be NULL): resolve_ms = mean resolver span; dep_pixels and zero_normalize of
 * the last frame. */
int rc_frame_submit(const rc_scene *scene, int width, int height, const rc_options *opt,
                    uint8_t *d_out);
int rc_frames_wait(rc_timing *timing);
/* Every parity frame is verified: after its last kernel the words its bounded carry
 * hand-offs set on a failure (timed-out spin: code, workgroup, details) are copied on the
 * frame's own stream into a pinned per-frame ring, before the frame's workspace can be reused.
 * rc_frames_wait reads back every frame since the previous wait (frames_checked /
 * frames_failed in *timing) and returns -1 if any failed; rc_frame_submit refuses new frames
 * once a frame in flight is known to have failed.  One-frame-at-a-time renders
 * (rc_render_device, rc_render) are read back at the next call on the device (which then
 * returns -1) or by rc_lone_frames_check, which synchronises the current device and returns
 * the count since its previous call (-1 if any failed). */
int rc_lone_frames_check(int64_t *checked, int64_t *failed);
/* Test aid: the nth_frame-th parity frame from now (0 = the next, any entry point, any
 * device) fails its hand-off as a timed-out spin would (error code 4); -1 cancels. */
int rc_debug_inject_error(int nth_frame);
/* Test aid (no GPU needed): rc_render's in-frame scatter of the mapped colour patch against a
 * host thread standing in for phase C — ndep entries stored in shuffled batches, each batch in
 * pieces, over an earlier frame's marks; skip != 0 leaves entries j % |skip| == 0 unstored,
 * and skip < 0 then ends the frame with a failure (-2).  Returns the number of wrong pixmap bytes (0) or the
 * sweep's failure status (< 0); -1 for ndep outside 1 .. 2^24. */
int rc_debug_scatter_selftest(int64_t ndep, int64_t seed, int skip);
/* Wait for every submitted frame, then release the current device's frame pipeline (its
 * CU-partitioned streams and events; the frame workspaces stay allocated).  The next
 * rc_frame_submit builds it again, re-reading RC_PIPE_* from the environment.  Returns what
 * rc_frames_wait would. */
int rc_pipe_reset(void);

/* Resolver diagnostics of the current device (a slow frame's own record): lone = 1 covers the
 * one-frame-at-a-time renders read back since the previous call with lone = 1 (reset), lone =
 * 0 the last rc_frames_wait window.  resolve_ms_* per frame from the resolver's HIP events (frames
 * in flight; 0 for lone frames); grid / res_cus = the last frame's resolver workgroups and the CUs
 * its stream may use; wg_per_cu = workgroups per CU of that placement, wg_per_cu_max = what one
 * CU can hold with k_resolve's registers and LDS reservation (occupancy API): fewer than the
 * placement needs would leave the grid partly queued behind resident workgroups; team rounds
 * = the most rounds of each kind one frame's team made; spin_wait_us_max[site] = the longest
 * bounded wait of any frame (sites: team hand-off, phase C carry-in, ready queue, helper
 * queue; waits under 10 us are not recorded); clock_mhz_* = the shader clock each frame's
 * resolver ran at (a throttled box explains a slow frame). */
typedef struct rc_resolver_stats {
  int64_t frames;
  double resolve_ms_min, resolve_ms_max, resolve_ms_mean;
  int32_t grid, res_cus, wg_per_cu, wg_per_cu_max;
  int32_t regs, scratch_bytes, lds_bytes, team_blocks;
  int32_t scan_rounds_max, cscan_rounds_max, resolve_rounds_max, pad;
  double spin_wait_us_max[4];
  int32_t clock_mhz_min, clock_mhz_max;   /* shader clock over each frame's resolver run
                                             (s_memtime vs s_memrealtime in workgroup 0) */
} rc_resolver_stats;
_Static_assert(sizeof(rc_resolver_stats) == 120, "rc_resolver_stats layout (ctypes binding)");
int rc_resolver_stats_get(int lone, rc_resolver_stats *out);

/* Duration (ms) of the last call's dominant kernel on the current device (the carry
 * resolver in parity mode, the render kernel otherwise), from HIP events on its stream. */
double rc_last_kernel_ms(void);

/* Per-phase kernel timing averaged over every render of the current device issued between
 * rc_profile_begin() and rc_profile_end() (HIP events on the render stream; no extra
 * synchronisation inside the window; at most 64 calls are kept). */
typedef struct rc_phase_stats {
  int calls;
  int parity;
  double phase_a_ms;    /* parity: phase A (all pixels, first-bounce-miss pixels deferred) */
  double compact_ms;    /* parity: scan-order DEP compaction + segment table               */
  double resolve_ms;    /* parity: carry-chain resolver                                    */
  double phase_c_ms;    /* parity: shading of the deferred pixels                          */
  double render_ms;     /* fast / depth 0: the single render kernel                        */
  double total_ms;      /* first kernel start to last kernel end                           */
} rc_phase_stats;
int rc_profile_begin(void);
int rc_profile_end(rc_phase_stats *out);

/* ---- schedule tuning (process-wide) -------------------------------------------------
 * The product's schedule is fixed by rc_default_tuning(); these fields exist so tests and
 * experiments can select the measured alternatives explicitly instead of
 * through the environment.  rc_set_tuning validates every field (returns -1 and changes
 * nothing when one is out of range); the resolver's co-residency limits are enforced on
 * top of it.  Takes effect at the next render (the frame pipeline's layout at its next
 * build: rc_pipe_reset). */
typedef struct rc_tuning {
  int side;               /* a lone parity frame's phase C: 0 after the resolver, 1 beside
                             it (k_side), 2 beside it for images of >= 8 Mpixel, 3 inside
                             the resolver (its idle waves shade ready batches; default), 4
                             inside it until its own work is over (k_finish: the rest)    */
  int split_shade;        /* 1: phase A's colours move beside the resolver (needs side)    */
  int resolve_shared;     /* 1: no one-resolver-workgroup-per-CU LDS reservation           */
  int resolve_lds_kb;     /* resolver LDS reservation in KiB, 0 = by path (96 / 56)        */
  int resolve_grid;       /* resolver workgroups, 0 = resident capacity (>= 8 otherwise)   */
  int team_blocks;        /* long-segment team workgroups, -1 = by path (128 / 3/8 grid)   */
  int helpers;            /* dense-run helper workgroups of a lone frame (0..64; pipeline lanes use none) */
  int hand_run;           /* changes in a row before a wave hands its run to a helper       */
  int long_len;           /* segments of >= long_len entries go to the team                 */
  int wave_k;             /* clean cooperative steps before a wave window returns to LANE   */
  int resolve_k;          /* the same for the team leader's block window                     */
  int coop;               /* 1: cooperative (lanes per entry) evaluator                      */
  int dep_fast;           /* 1: clean DEP entries take phase A's primary shade               */
  int o0;                 /* 1: primary rays through the origin-zero intersection forms      */
  int phase_c_finish;     /* 1: phase C after the resolver through k_finish's batch claims   */
  int single_res_cus;     /* lone frames: resolver sized for this many CUs, 0 = all          */
  int pipe_res_cus;       /* frames in flight: resolver partition CUs, 0 = by image size     */
  int pipe_resolvers;     /* frames in flight: resolver lanes (1..4)                          */
  int pipe_slots;         /* frames in flight: frame workspaces (lanes+1 .. 8)                */
  int pipe_timing;        /* 1: resolver timing events per pipelined frame                   */
  int pipe_slotstreams;   /* 1: one stream per slot (A, compaction, C in turn)               */
  int overlap_d2h;        /* 1: rc_render's copy overlaps the resolver (parity)              */
  int staged_d2h;         /* 1: pinned bounce buffers + host pool; 0: runtime pageable copy  */
  int prefault;           /* 1: fault the caller's pixmap in while the GPU renders           */
  int copy_threads;       /* host copy pool threads (1..32; fixed at the pool's first use)   */
  int side_blocks;        /* lone parity frames: at most this many k_side workgroups (phase C
                             beside the resolver), 0 = one per CU                            */
  int comp_stream;        /* frames in flight: compaction on an unmasked top-priority stream
                             (0 never, 1 always, 2 for images of >= 32 Mpixel)              */
  int block_min;          /* regular carry segments of >= block_min entries are resolved by a
                             whole resolver workgroup (block windows) when the grid has a
                             workgroup for each of them, 0 = never (default 3000)            */
  int pipe_inres;         /* frames in flight: phase C inside the resolver lanes (their idle
                             waves shade ready batches) instead of on the pixel partition:
                             0 never (default), 1 until the queue is drained, 2 until the
                             lane's own resolver work is over (k_finish shades the rest)     */
  int x0;                 /* 1: quadrics whose d, e, f are all zero are tested without their
                             cross terms (bit-identical, rc_device.hpp quad_abc; default 1) */
  int resolve_clean;      /* clean 256-entry windows in a row before the team leader hands a
                             RESOLVE round back to the team's SCAN (1..64)                   */
  int shard_lone;         /* 1: a one-rank group renders its image as a lone frame (default);
                             0: through the sharded exchange (wire records, gathers, the
                             root's resolver) like a multi-rank group — test and measurement */
  int team_cscan;         /* 1: the team leader hands a RESOLVE round back after resolve_k clean
                             cooperative steps and the team's next SCAN round is one
                             cooperative step of every team wave (default); 0: the leader's
                             LANE passes and LANE-only SCAN rounds                            */
  int pipe_order;         /* frames in flight: creation order of the CU-masked streams (the
                             runtime maps streams onto hardware queues in creation order): 0
                             lane by lane (resolver, phase C), then the pixel streams; 1
                             resolvers, pixel streams, phase C; 2 pixel streams, phase C,
                             resolvers; 3 each resolver lane on a hardware queue of its own
                             (placeholder streams fill the others; needs two lanes and the
                             default stream layout, else order 2 with a warning); 4 one phase
                             C stream for both lanes and each resolver lane beside an idle
                             placeholder (same conditions as 3)                           */
  int pipe_helpers;       /* frames in flight: dense-run helper workgroups per resolver lane
                             (default 4; 0 = none)                                            */
  int patch_host;         /* rc_render (parity, overlap_d2h): phase C writes the DEP entries'
                             packed colours straight into pinned host memory (zero-copy), so
                             nothing is left to copy when the frame ends, and the host
                             scatters each entry as it arrives, during the frame (default 2);
                             1: scattered after the frame; 0: a device buffer copied after
                             phase C                                                          */
  int share_device;       /* rc_render / raycast() with num_gpus > 1: 0 one device per rank
                             (devices device .. device+num_gpus-1, RCCL; fewer if the box has
                             fewer, with a warning); 1 every rank on `device` with device
                             copies between the ranks (the multi-GPU path on one GPU: tests) */
  int headb_first;        /* one frame at a time: resolver workgroups that skip the whole-
                             workgroup queue of long regular segments and start at once on the
                             per-wave queue, whose front holds the runs that can be dense    */
  int pipe_last_whole;    /* rc_frames_wait runs the window's last frame's phase C on every CU
                             instead of the pixel partition (1, default; 0 = the partition)   */
} rc_tuning;
void rc_default_tuning(rc_tuning *t);
int rc_set_tuning(const rc_tuning *t);
void rc_get_tuning(rc_tuning *t);

/* ---- multi-GPU row shards ----------------------------------------------
 * Rows are dealt cyclically (image row y -> rank y % G).  Every rank renders its rows; the
 * root (rank 0) gathers the row blocks over RCCL (ncclGather over xGMI) and undoes the
 * interleave on its device.  Parity mode adds the carry chain's exchange: every rank runs
 * phase A on its rows, the root receives the other ranks' DEP entries and row blocks
 * (ncclSend/ncclRecv; its own are read in place), rebuilds the scan-order DEP list, and its
 * resolver resolves the carry chain and shades every DEP entry (phase C) straight into the
 * image: nothing returns to the ranks.  The output is byte-identical to rc_render on one
 * device. */
#define RC_GROUP_ID_BYTES 128          /* == sizeof(ncclUniqueId) */
enum { RC_XFER_AUTO = 0,   /* RCCL when every rank has its own device, else RC_XFER_COPY */
       RC_XFER_RCCL = 1,   /* RCCL communicators (xGMI)                                 */
       RC_XFER_COPY = 2    /* device copies between the ranks' buffers (one process)    */ };
typedef struct rc_group rc_group;

/* A fresh RCCL unique id: rank 0 of a multi-process job makes one and shares it. */
int rc_group_unique_id(unsigned char id[RC_GROUP_ID_BYTES]);
/* One rank of a multi-process job (one process per GPU) on `device`; collective over the
 * nranks processes (ncclCommInitRank).  NULL on failure. */
rc_group *rc_group_create_rank(int nranks, int rank, const unsigned char id[RC_GROUP_ID_BYTES],
                               int device);
/* All nranks ranks in this process, rank i on devices[i] (ranks may share a device only with
 * RC_XFER_COPY; RC_XFER_AUTO picks).  NULL on failure. */
rc_group *rc_group_create_local(int nranks, const int *devices, int transport);
void rc_group_destroy(rc_group *group);
int rc_group_size(const rc_group *group);
int rc_group_transport(const rc_group *group);   /* RC_XFER_RCCL or RC_XFER_COPY */

/* Render W x H row-sharded over the group: collective (every rank's process calls it with
 * the same arguments).  The image lands in d_image (W*H*3 bytes, device memory of rank 0's
 * device; NULL = a buffer of the group's own) on the root; other ranks ignore d_image.
 * Synchronous.  timing (may be NULL): total_ms (host), kernel_ms (root's device span),
 * resolve_ms, dep_pixels and zero_normalize of the whole image (root).  Returns 0 on
 * success. */
int rc_render_sharded(rc_group *group, const rc_scene *scene, int width, int height,
                      const rc_options *opt, uint8_t *d_image, rc_timing *timing);

typedef struct rc_shard_stats {   /* the last rc_render_sharded, on the root */
  int ranks;
  double total_ms;        /* host wall clock of the call                                   */
  double device_ms;       /* root's stream: first kernel to the de-interleaved image        */
  double local_ms;        /* root's own rows: fast: render; parity: phase A + packing       */
  double exchange_in_ms;  /* parity: end of the root's phase A to the resolver's start (entry
                             and row-block gathers, de-interleave, scan-order rebuild)       */
  double resolve_ms;      /* parity: image-wide carry resolver on the root                  */
  double phase_c_ms;      /* parity: the phase C tail after the root's resolver (phase C runs
                             inside the resolver on the root)                                */
  double image_ms;        /* fast: row-block gather + de-interleave; parity: the image's copy
                             into the caller's buffer (the row blocks are gathered before the
                             resolver, inside exchange_in_ms)                                */
  int64_t dep_pixels;
  int64_t zero_normalize;
  int64_t entry_bytes;    /* DEP entries moved to the root                                  */
  int64_t carry_bytes;    /* carry-ins moved back (0: phase C runs on the root)              */
  int64_t image_bytes;    /* row blocks moved to the root (padded to ceil(H/G) rows)        */
} rc_shard_stats;
int rc_group_last_stats(const rc_group *group, rc_shard_stats *out);
/* One rank's own timeline of the last rc_render_sharded (every rank, root or not; -1 if this
 * process does not drive `rank`): local_ms = its rows (fast: render; parity: phase A + wire
 * records), exchange_ms = from there until its row blocks (and parity entries) have left,
 * total_ms = the whole frame on its stream. */
typedef struct rc_rank_stats {
  int rank;
  int rows;
  double local_ms;
  double exchange_ms;
  double total_ms;
  int64_t dep_pixels;     /* parity: the rank's own DEP entries */
} rc_rank_stats;
int rc_group_rank_stats(const rc_group *group, int rank, rc_rank_stats *out);
/* Parity frames exchange the DEP entries in fixed-size per-rank blocks (no host
 * synchronisation inside the frame) once a frame of the same scene and size has given the
 * per-rank count; a frame that exceeds it is rendered again with exact sizes.  Test aid: set
 * that bound (entries per rank; -1 forgets it). */
int rc_group_debug_bound(rc_group *group, long long per_rank);

/* Library version / build string. */
const char *rc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RAYCAST_HIP_H */
