/* gsplat.h — C ABI of the MI355X Gaussian-splat forward renderer (libgsplat.so).
 *
 * Drop-in boundary for the WebGPU path of Lontoone/gaussian-splatting-web (reference @ 2024-12-20,
 * paths relative to /root/reference).  The reference binds its GPU work through WebGPU objects
 * owned by `GpuContext` and `Renderer`; this ABI is what the Node N-API addon
 * (gaussian-splatting-web_amd/addon/gsplat_napi.cc) binds in their place:
 *
 *   gs_ctx_create / gs_ctx_destroy  <- GpuContext.create / GpuContext.destroy  (src/gpu_context.ts:12-32)
 *                                      Renderer.requestContext                (src/renderer.ts:79-100)
 *   gs_scene_upload / gs_scene_free <- Renderer ctor's pointDataBuffer upload (src/renderer.ts:139-146)
 *                                      and destroyImpl's buffer destroys      (src/renderer.ts:281-292)
 *   gs_render / gs_render_device    <- Renderer.draw: init-sort pass + radix sort + SimpleRender.draw
 *                                      (src/renderer.ts:301-319, src/shaders.ts:42-73,
 *                                       src/simple_render.ts:217-332, :169-200, :509-537)
 *   gs_pack_uniforms                <- uniformLayout.pack in Renderer.animate  (src/renderer.ts:24-33, :349-384)
 *   gs_look_at / gs_perspective /
 *   gs_camera_position              <- wgpu-matrix lookAt/perspective/inverse+getTranslation as used by
 *                                      src/camera.ts:101-138 (f32 storage semantics)
 *   gs_present / gs_present_device  <- PostProcessRenderer.draw               (src/post_process_render.ts:54-77)
 *   gs_encode_png                   <- (new: PNG dumps of the presented image for visual diffs)
 *
 * Conventions: every function returns 0 on success and a negative gs_status on failure; no C++
 * exception crosses the ABI; gs_last_error() returns a thread-local message for the last failure.
 * One gs_ctx per host thread; calls on a ctx are serialised by the caller.
 *
 * Scene input = the reference's AoS record (PackedGaussians.gaussiansBuffer, src/ply.ts:249-257):
 *   position f32x3 @0, scale f32x3 @16 (already |exp(s)|), rot f32x4 @32 (= (-x,-y,-z,w) of the
 *   normalised PLY quaternion), opacityLogit f32 @48, sh[n_sh] f32x3 @64 + 16k; record size
 *   64 + 16*n_sh bytes, n_sh in {1,4,9,16}.  The host buffer is borrowed for the call only.
 * Uniforms = the reference's 160-byte block (view mat4 @0, proj mat4 @64, camPos vec3 @128,
 *   tanHalfFovX/Y @140/144, focalX/Y @148/152, scaleModifier @156; matrices column-major).
 * Output = W*H premultiplied RGBA in framebuffer row order (row 0 = top), i.e. the contents of
 *   SimpleRender.framebuffer (src/simple_render.ts:499-505), as f32x4 (or f16x4) per pixel.
 */
#ifndef GSPLAT_H
#define GSPLAT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 5

typedef struct gs_ctx gs_ctx;
typedef struct gs_scene gs_scene;

typedef enum gs_status {
    GS_OK = 0,
    GS_ERR_INVALID = -1,     /* bad argument */
    GS_ERR_NO_DEVICE = -2,   /* no HIP device (GpuContext.create rejects) */
    GS_ERR_HIP = -3,         /* HIP runtime error */
    GS_ERR_OOM = -4,         /* device allocation failed */
    GS_ERR_UNSUPPORTED = -5, /* e.g. SH coefficient count not in {1,4,9,16} */
    GS_ERR_DEVICE_FAULT = -6,/* a kernel reported a protocol failure (bounded spin expired) */
    GS_ERR_INTERNAL = -7
} gs_status;

typedef enum gs_accum {
    GS_ACCUM_FP32 = 0,        /* fp32 accumulation (default) */
    GS_ACCUM_FP16_TARGET = 1  /* round dst to fp16 after every blend, as the rgba16float target does */
} gs_accum;

typedef enum gs_out_format {
    GS_OUT_RGBA_F32 = 0,
    GS_OUT_RGBA_F16 = 1
} gs_out_format;

typedef struct gs_opts {
    uint32_t struct_size; /* sizeof(gs_opts); set by gs_opts_default */
    int32_t accum;        /* gs_accum */
    int32_t out_format;   /* gs_out_format */
    float t_min;          /* a pixel stops compositing once (1 - alpha) < t_min; 0 = never (default 1e-4) */
    int32_t ref_quirks;   /* 1: reproduce the reference's init-sort grid truncation (src/renderer.ts:306):
                             only trunc(max(N/8,8))*8 slots are keyed per frame, the rest keep the previous
                             frame's sorted (key,value) (zero on the first frame), so a Gaussian may be drawn
                             twice or not at all.  The state lives in the scene and advances once per call
                             (one call = one reference frame; strips of one frame belong on separate scenes,
                             one per rank).  N <= 524280 (above it the reference's dispatch is invalid:
                             GS_ERR_UNSUPPORTED).  Waits for the frames in flight (a compatibility mode). */
    int32_t strip_index;  /* row strip rendered by this call, 0 <= strip_index < strip_count */
    int32_t strip_count;  /* number of equal row strips (16-px tile rows, see gs_strip_rows); 1 = whole image */
    int32_t timing;       /* 1: record per-stage hipEvent timings (gs_timings); 2: the composite's only
                             (each event costs the stream a few microseconds) */
    float chunk_fraction; /* depth split between the two chunks (the image never depends on it):
                             0 = adaptive (from the depth at which tiles saturated last frame),
                             >= 1 = one chunk, (0,1) = fixed split at the depth 2^-t <=
                             chunk_fraction of the way from the last frame's nearest to its
                             farthest visible splat (tests/diagnostics) */
    /* (ABI 3) an explicit strip: with tile_row_end > 0, render only tile rows [tile_row_begin,
       tile_row_end) of the image (16-px rows, 0 <= begin < end <= ceil(H/16); strip_count must be
       1; not on a device group, which chooses its own strips).  The output holds image rows
       [16*tile_row_begin, min(16*tile_row_end, H)), no padding.  K-balanced strips: gs_balance_strips. */
    int32_t tile_row_begin;
    int32_t tile_row_end;
    /* (ABI 5) list split: 0 (default) = every tile's depth-ordered list is one serial chain of
       blends; the image is then bit-identical whatever the chunk split, the strips or the device
       group.  1 = in frames with fewer tiles than the device holds at once (row strips, chunk 1's
       unsaturated tiles under a moving camera) a long tile list is cut into up to 4 contiguous
       segments blended by separate wave pairs and merged in list order (C += T C_s, T *= T_s):
       within the fp32 oracle bar and run-to-run deterministic, not bit-identical to 0 (a
       segment may add contributions below t_min x colour after the tile's saturation point).
       accum = GS_ACCUM_FP16_TARGET ignores it. */
    int32_t list_split;
} gs_opts;

typedef struct gs_stats {
    uint64_t n;           /* Gaussians in the scene */
    uint64_t n_vis;       /* visible splats in this strip; exact for a one-chunk frame (with a chunk
                             split, Gaussians past the split that survive the conservative cull
                             are counted, and partitions wholly past it are skipped) */
    uint64_t k_entries;   /* (tile, splat) pairs binned (both chunks) */
    uint64_t k_total;     /* sum of the box tile counts of the binned splats (SURVEY's K for a
                             one-chunk frame) */
    uint32_t tiles_unsaturated;  /* tiles chunk 0 left unsaturated */
    float chunk_fraction; /* fraction of the visible splats sorted in chunk 0 (last frame) */
    int32_t tile_row_begin, tile_row_end;  /* tile rows rendered by the last call */
    int32_t tiles_x;
    int32_t frames;       /* timed frames since gs_timings_reset; ms_composite averages all of them, the
                             other stage times the frames timed with opts.timing = 1 */
    float ms_total;       /* mean HIP-event times per timed frame: whole frame and per stage: */
    float ms_project, ms_sort, ms_bin, ms_tile_sort, ms_ranges, ms_composite, ms_other;
                          /* project = partition cull + cull + projection/colour; ms_sort = chunk 1
                             (one launch; ~0 when chunk 0 saturated every tile); bin = count,
                             column scan, tile scan, emission; tile_sort = per-tile sort; ranges
                             = 0 (kept for the ABI); composite = chunk 0's composite */
    uint32_t k_chunk0, k_chunk1;  /* pairs binned per chunk (last frame) */
    uint32_t wide_chunk0, wide_chunk1;  /* splats of >= 32 tiles emitted row-wise, per chunk */
    /* frame counts since gs_timings_reset (every frame, timed or not): */
    uint32_t frames_rendered;  /* frames enqueued */
    uint32_t frames_chunked;   /* ... rendered with a depth split (two chunks) */
    uint32_t frames_unsat;     /* ... whose chunk 0 left tiles unsaturated (chunk 1 composited them;
                                  counted when the frame's statistics arrive) */
    uint32_t frames_seeded;    /* ... whose split depth came from the frame's own coarse depth
                                  estimate (no usable history: a first frame or a camera cut) */
    float chunk_depth;         /* |view depth| of the last frame's chunk split (0: one chunk) */
    /* ABI 5: */
    uint32_t list_max;         /* longest tile list of the last frame, either chunk (0 when none is
                                  longer than 1024 entries) */
    uint32_t tiles_long;       /* tiles whose list outgrew the 1024-thread sort shape's one LDS
                                  round (8192 entries) and went to the linear long-list sort */
} gs_stats;

/* ---- library / device ---------------------------------------------------------------------- */
int gs_abi_version(void);
const char* gs_last_error(void);
int gs_device_count(int* out_count);

/* GpuContext.create: rejects (GS_ERR_NO_DEVICE) when no HIP device exists.  devices = NULL with
 * ndev = 0: device 0.  ndev > 1 (<= 64) makes a device group: one context drives every listed
 * device from this thread.  A scene uploaded to it is replicated on each device; a frame is split
 * into ndev row strips, strip g rendered on devices[g], and the strips are gathered into
 * devices[0] over RCCL (ncclCommInitAll; xGMI on MI355X) -- or, when the list repeats a device
 * (tests on one GPU), with peer copies.  The image is delivered on devices[0] (gs_render_device's out_dev and hip_stream
 * belong to it).  gs_opts.strip_count must be 1 on a group. */
int gs_ctx_create(const int* devices, int ndev, gs_ctx** out_ctx);
/* (A group's strips are K-balanced (gs_balance_strips on the members' binned entries, every 8
 * frames) and each member's strip goes to devices[0] only: RCCL send/receive pairs on per-member
 * gather streams, double-buffered, so frame f + 1 renders while frame f's strips travel.) */
typedef enum { GS_GATHER_NONE = 0, GS_GATHER_RCCL = 1, GS_GATHER_PEER_COPY = 2 } gs_gather_kind;
/* Devices driven by the context and how a group gathers its strips (gs_gather_kind). */
int gs_ctx_info(const gs_ctx* ctx, int* out_ndev, int* out_gather);
/* A device group's current strip boundaries in tile rows (G + 1 values; strip g = [b[g], b[g+1]))
 * for the last frame size; *out_n = G + 1 (0 before the first frame or on a single device).
 * out_bounds may be NULL (count only). */
int gs_ctx_strips(const gs_ctx* ctx, int* out_bounds, int capacity, int* out_n);
/* Also frees every scene still attached to the context (do not free those scenes afterwards). */
void gs_ctx_destroy(gs_ctx* ctx);

/* Copies the AoS scene once into device memory as SoA planes (AoS -> SoA transpose on device). */
int gs_scene_upload(gs_ctx* ctx, const void* aos, uint64_t n, int n_sh_coeffs, gs_scene** out_scene);
void gs_scene_free(gs_scene* scene);
uint64_t gs_scene_count(const gs_scene* scene);

void gs_opts_default(gs_opts* opts);

/* K-balanced row strips: new tile-row boundaries out_bounds[0..G] (0 = first, TR =
 * last) that equalise the strips' costs, given the current boundaries bounds[0..G] and each
 * strip's measured cost under them (e.g. its binned entries, gs_stats k_entries, plus a per-tile
 * term), the cost of a strip taken as spread evenly over its rows; each boundary moves half way
 * to that model's cut (damped: fed back frame after frame it converges).  Every strip keeps >= 1 tile
 * row when TR >= G.  Deterministic host arithmetic: ranks that feed it the same (all-gathered)
 * costs get the same boundaries.  A device group rebalances itself every 8 frames this way. */
int gs_balance_strips(int G, int tile_rows, const int* bounds, const double* cost, int* out_bounds);

/* Rows of image covered by strip `strip_index` of `strip_count`: tile rows
 * [s*ceil(TR/G), min((s+1)*ceil(TR/G), TR)), TR = ceil(H/16).  *row0 = first image row,
 * *rows_padded = ceil(TR/G)*16 (every strip's output buffer has this many rows, so an
 * all-gather of the G strip buffers is the image followed by padding rows; a render writes its
 * padding rows as zero). */
int gs_strip_rows(int H, int strip_index, int strip_count, int* row0, int* rows_padded);

/* Render one frame.  out_host_or_null: W*H pixels (strip_count == 1) or rows_padded*W pixels
 * (strip mode) of the chosen out_format, or NULL to keep the frame on the device.  Synchronous. */
int gs_render(gs_ctx* ctx, gs_scene* scene, const void* uniforms160, int W, int H,
              const gs_opts* opts, void* out_host_or_null);

/* Same, writing into device memory `out_dev` (>= out_bytes) on `hip_stream` (NULL = the ctx's
 * stream).  Returns when the work is enqueued; the caller synchronises the stream.  The frame's
 * culling, projection, binning and per-tile sort run on the scene's own streams (up to three
 * frames in flight); the composite (which writes out_dev) and the frame's end run on
 * `hip_stream` in call order, so work enqueued on it afterwards sees the finished frame.
 * Device-side frame errors (tile-entry overflow, a chunk-1 barrier timeout) come back with the
 * frame's statistics, asynchronously: an error of frame t is reported (GS_ERR_DEVICE_FAULT) by a
 * later gs_render_device or gs_sync call, never lost (the bits of every frame are kept
 * until reported).  gs_render, being synchronous, reports its own frame's errors. */
int gs_render_device(gs_ctx* ctx, gs_scene* scene, const void* uniforms160, int W, int H,
                     const gs_opts* opts, void* out_dev, uint64_t out_bytes, void* hip_stream);

/* Device framebuffers for gs_render_device / gs_present_device: the GPU-resident render target
 * of the reference (SimpleRender's rgba16float `framebuffer` texture, src/simple_render.ts:499-505,
 * read by the present pass) -- frames stay in HBM and are read back only on request.
 * gs_framebuffer_alloc: `bytes` of device memory on the context's device (a group's first).
 * gs_framebuffer_read: waits for the context's frames (gs_sync semantics, frame errors included),
 * then copies `bytes` to host memory; `dev` must lie inside a buffer gs_framebuffer_alloc made on
 * this context and the read must end inside it (else GS_ERR_INVALID). */
int gs_framebuffer_alloc(gs_ctx* ctx, uint64_t bytes, void** out_dev);
int gs_framebuffer_free(gs_ctx* ctx, void* dev);
int gs_framebuffer_read(gs_ctx* ctx, const void* dev, void* host, uint64_t bytes);

/* Asynchronous readback (ABI 4): the host side of the reference's frame loop, which submits a
 * frame and requests the next animation frame without waiting for it (src/renderer.ts:301-330,
 * :345-348), with the frame copied out to host memory.
 * gs_host_register / gs_host_unregister: page-lock a caller's host buffer (hipHostRegister) so
 * that copies into it run as DMA at the link's rate, asynchronously; unregister waits for the
 * readbacks in flight.  A buffer must be unregistered before it is freed.
 * gs_readback_start: enqueue a copy of `bytes` from a gs_framebuffer_alloc buffer (the same bounds
 * as gs_framebuffer_read) to `host`, ordered after every frame enqueued so far on the context's
 * own stream (gs_render_device with stream NULL), on a copy stream of its own, so the next frames
 * render meanwhile; returns a ticket.  It does not wait: the framebuffer must not be rendered into
 * again before the ticket's wait returns.
 * gs_readback_wait: blocks until the ticket's copy (and every earlier one) has landed.  Safe to
 * call from another thread than the one enqueuing frames. */
int gs_host_register(gs_ctx* ctx, void* host, uint64_t bytes);
int gs_host_unregister(gs_ctx* ctx, void* host);
int gs_readback_start(gs_ctx* ctx, const void* dev, void* host, uint64_t bytes, uint32_t* out_ticket);
int gs_readback_wait(gs_ctx* ctx, uint32_t ticket);

int gs_timings(gs_ctx* ctx, gs_stats* out_stats);
int gs_timings_reset(gs_ctx* ctx);
int gs_sync(gs_ctx* ctx);

/* PostProcessRenderer (src/post_process_render.ts:54-77) on the host-visible image: y flip,
 * a' = sat(1.5a), a' = a'^4 (computed as (a'^2)^2) if a' < 0.99.  rgba_in/out: W*H f32x4 host
 * buffers. */
int gs_present(const float* rgba_in, int W, int H, float* rgba_out);

typedef enum {
    GS_PRESENT_RGBA_F32 = 0,  /* f32x4 */
    GS_PRESENT_RGBA_F16 = 1,  /* f16x4: the reference's rgba16float canvas (src/post_process_render.ts:24) */
    GS_PRESENT_RGBA8 = 2      /* unorm8x4 = round(sat(v) * 255), for PNG dumps */
} gs_present_format;

/* The same transform on the device, from a framebuffer gs_render_device wrote (fb_format =
 * GS_OUT_RGBA_F32 or GS_OUT_RGBA_F16, W*H pixels, row 0 = top) into out_dev (>= out_bytes) in
 * out_format, on hip_stream (NULL = the ctx's stream); returns when the work is enqueued.  For
 * the same input it equals gs_present bit for bit (f32), or that result rounded (f16, unorm8). */
int gs_present_device(gs_ctx* ctx, const void* fb_dev, int fb_format, int W, int H, int out_format,
                      void* out_dev, uint64_t out_bytes, void* hip_stream);

/* PNG (RGBA, 8 bits, stored deflate blocks, no external library) of a W*H RGBA8 image, row 0 =
 * top.  out == NULL: *out_len = bytes needed.  GS_ERR_INVALID when cap is too small. */
int gs_encode_png(const uint8_t* rgba8, int W, int H, uint8_t* out, uint64_t cap, uint64_t* out_len);

/* ---- camera / uniforms (headless producer; wgpu-matrix 2.9.1 semantics, f32 storage) ------- */
int gs_look_at(const double eye[3], const double target[3], const double up[3], float out_view[16]);
int gs_perspective(double fovy_radians, double aspect, double z_near, double z_far, float out_proj[16]);
int gs_camera_position(const float view[16], float out_pos[3]);
/* cameraFromJSON (src/camera.ts:476-503) for one INRIA cameras.json entry: position[3],
 * rotation[9] (the JSON's 3x3 as given, rows flattened, handed to WM mat3.create), fx, fy, and the
 * canvas size.  view = worldToCamFromRT (src/camera.ts:467-473), proj = getProjectionMatrix(0.2,
 * 100, focal2fov(fx, W), focal2fov(fy, H)) (src/camera.ts:19-42, :463-465; +z forward).
 * out_focal (optional) = the Camera's focalX/focalY, which the reference sets to (H, W). */
int gs_camera_from_json(const double position[3], const double rotation[9], double fx, double fy,
                        int canvas_w, int canvas_h, float out_view[16], float out_proj[16],
                        float out_focal[2]);
int gs_pack_uniforms(const float view[16], const float proj[16], const float cam_pos[3],
                     float tan_half_fov_x, float tan_half_fov_y, float focal_x, float focal_y,
                     float scale_modifier, void* out160);

/* ---- synthetic scenes (seeded splitmix64) -------------------------------------- */
/* Writes n records of 320 bytes (SH degree 3) in the reference AoS layout. */
int gs_synth_aos(uint64_t n, uint64_t seed, int W, int H, void* out_aos);

/* ---- PLY ingest (src/ply.ts:54-355, PackedGaussians) --------------------------------------- */
typedef struct gs_ply_info {
    uint64_t num_gaussians;   /* PackedGaussians.numGaussians */
    int32_t sh_degree;        /* sphericalHarmonicsDegree (0..3) */
    int32_t n_sh_coeffs;      /* nShCoeffs: 1, 4, 9 or 16 */
    uint64_t record_bytes;    /* 64 + 16 * n_sh_coeffs: the AoS record of gs_scene_upload */
    uint64_t data_offset;     /* first vertex byte in the file */
    uint64_t vertex_stride;   /* bytes per vertex in the file (float 4, uchar 1, others unread) */
    float min_pos[3], max_pos[3];        /* PackedGaussians.min_pos / max_pos (f32) */
    double min_pos_d[3], max_pos_d[3];   /* the same as the reference holds them (JS numbers) */
} gs_ply_info;
/* Parses a binary-little-endian .ply with the reference's exact semantics (header chunks, property
 * order, float/uchar only, rotation normalise + swizzle, |exp(scale)|, SH order, f32 packing).
 * out_aos NULL: fills `info` only (size the buffer as num_gaussians * record_bytes).  Returns
 * GS_ERR_INVALID on a truncated file, GS_ERR_UNSUPPORTED when the f_rest count is not 0/9/24/45
 * (the reference throws "Unsupported SH degree"). */
int gs_ply_parse(const void* ply, uint64_t bytes, gs_ply_info* info, void* out_aos, uint64_t out_bytes);

/* ---- checks used by tests ------------------------------------------------------------------ */
/* Chunk 1's single-launch form (k_chunk1) separates its phases with grid barriers, so its whole
 * grid must be resident at once: the grid is min(64, CUs, occupancy x CUs) with the occupancy of
 * k_chunk1 queried at context creation (gs_ctx_create fails with GS_ERR_UNSUPPORTED when it is 0).
 * ctx != NULL: that context's grid and measured occupancy; ctx == NULL: the grid for the given
 * occupancy (workgroups per CU) and CU count (GS_ERR_UNSUPPORTED when nothing fits). */
int gs_debug_chunk1_grid(const gs_ctx* ctx, int occupancy, int cus, int* out_grid, int* out_occupancy);
/* The per-tile chunk-0 cut: margin 0 = default (a still camera's chunked frames bin
 * each tile's splats only up to its last saturation depth x 1.01), < 0 = off, > 0 = that depth
 * margin -- below 1 every tile is cut short of its saturation point, so chunk 1 must finish the
 * tiles with the entries chunk 0 left out (a test of that path; the image never changes). */
int gs_debug_cut_margin(gs_ctx* ctx, float margin);
/* Stable ascending GPU radix sort of (key,value) on bits [begin_bit,end_bit): host in/out. */
int gs_debug_sort_pairs(gs_ctx* ctx, uint32_t* keys, uint32_t* vals, uint64_t n, int begin_bit,
                        int end_bit);
/* The last frame's visible set: depth key and reference index of every composite slot, sorted on
 * the host by (key, index) (under ref_quirks: (draw rank, Gaussian)).  The order the composite
 * used is what gs_debug_tile_lists exports. */
int gs_debug_last_order(gs_ctx* ctx, gs_scene* scene, uint32_t* out_keys, uint32_t* out_index,
                        uint64_t capacity, uint64_t* out_n);
/* Projected record of every Gaussian in the last frame, 16 floats each: centre cx, cy (pixels);
 * quad axes e1/|e1|^2 and e2/|e2|^2 scaled by sqrt(log2 e) (2 floats each); log2(opacity);
 * pixel box x [x0|x1<<16] (u32 bits); colour r, g, b; 0; depth key; tile count; pixel box x, y
 * (u32 bits).  The colour is evaluated only for splats that received a tile entry this frame;
 * rows of culled Gaussians and the colour of unbinned splats are undefined. */
int gs_debug_last_records(gs_ctx* ctx, gs_scene* scene, float* out16, uint64_t capacity);
/* Every composite slot of the last frame, as k_project (chunk 0) / k_chunk1 (chunk 1) wrote it:
 * 16 words per slot: depth key, reference index (ref_quirks: draw rank, Gaussian), chunk, packed
 * tile rect, record r0 (4 f32: centre x, y, axis 1 / |e1|^2 * sqrt(log2 e)), r1 (4 f32: axis 2 likewise,
 * log2 opacity, pixel box x bits), colour r, g, b (f32) and the depth key bits.  out16 NULL: count only. */
int gs_debug_last_slots(gs_ctx* ctx, gs_scene* scene, uint32_t* out16, uint64_t capacity, uint64_t* out_n);
/* The per-tile lists the last frame's composite consumed (one-chunk frames only; else
 * GS_ERR_UNSUPPORTED): out_ranges[2t], [2t+1] = [begin, end) of tile t (row-major in the frame's
 * strip) in out_entries, whose entries are (depth key, reference index) pairs -- (draw rank,
 * Gaussian) under ref_quirks -- in composite order.  NULL outputs: counts only. */
int gs_debug_tile_lists(gs_ctx* ctx, gs_scene* scene, uint32_t* out_ranges, uint64_t ranges_capacity,
                        uint32_t* out_entries, uint64_t entries_capacity, uint64_t* out_tiles,
                        uint64_t* out_entries_n);
/* Structural check of the last frame's tile lists (one-chunk frames only), on the host, at any
 * frame size: out[0] = entries, out[1] = (tile, Gaussian) pairs listed more than once, out[2] =
 * adjacent entries of a tile not in strictly ascending (depth key, reference index) order, out[3]
 * = tiles whose list does not begin where the previous tile's ends, out[4] = entries holding a
 * slot that is not a visible splat of the frame (a hole or past the slot space).  A correct
 * frame has out[1..4] == 0; the reference draws every Gaussian at most once per frame
 * (drawIndexed(6, N), src/simple_render.ts:525-534) and blends in stable depth order. */
int gs_debug_tile_list_check(gs_ctx* ctx, gs_scene* scene, uint64_t out[5]);

#ifdef __cplusplus
}
#endif
#endif /* GSPLAT_H */
