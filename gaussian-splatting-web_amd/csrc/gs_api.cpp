// gs_api.cpp — C ABI (include/gsplat.h): contexts, scenes and the per-frame pipeline.
//
// A frame (render_frame) is a fixed sequence of launches with no host round trip; data-
// dependent sizes live in FrameCtl on the device:
//   k_part_list -> k_cull -> k_project -> k_bin_count -> k_bin_colscan -> k_bin_emit ->
//   k_tile_sort -> k_composite (a still camera: k_composite_ts, the sort inside it) ->
//   k_chunk1 (chunk 1 when chunk 0 left tiles unsaturated, then the frame's end; or chunk 1's
//   separate launches and k_frame_end)
// Chunk 0 = the visible splats nearer than a depth key T; chunk 1 = the rest, binned only into
// tiles chunk 0 left unsaturated.  T adapts from earlier frames' statistics (read back
// asynchronously); the image does not depend on T.  Frames rotate over kFrameSets sets of
// per-frame buffers, each with its own stream, so consecutive frames overlap on the GPU.
// Reference call stack replaced: Renderer.animate/draw (src/renderer.ts:332-387, :301-330).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <chrono>
#include <utility>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gsplat.h"
#include "gs_device.h"

using namespace gs;

namespace {

thread_local std::string g_last_error;

struct GsError : std::runtime_error {
    int code;
    GsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            throw GsError(e_ == hipErrorOutOfMemory ? GS_ERR_OOM : GS_ERR_HIP,           \
                          std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const GsError& e) {
        return fail(e.code, e.what());
    } catch (const std::bad_alloc&) {
        return fail(GS_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(GS_ERR_INTERNAL, e.what());
    } catch (...) {
        return fail(GS_ERR_INTERNAL, "unknown exception");
    }
}

template <class T>
void dev_alloc(T*& p, size_t count) {
    p = nullptr;
    if (count == 0) count = 1;
    HIPCHK(hipMalloc((void**)&p, count * sizeof(T)));
}
template <class T>
void dev_free(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}


// Per-frame timing events (opts.timing): kernel groups are bracketed directly.
enum {
    EV_BEGIN, EV_PROJ0, EV_PROJ1,
    EV_DSORT_0, EV_BIN_0, EV_TSORT_0, EV_RANGES_0, EV_COMP_0,
    EV_DSORT_1, EV_BIN_1, EV_TSORT_1, EV_RANGES_1, EV_COMP_1, EV_END, EV_COUNT
};
enum { ST_TOTAL, ST_PROJECT, ST_SORT, ST_BIN, ST_TSORT, ST_RANGES, ST_COMPOSITE, ST_COUNT };

#ifndef GS_FRAME_SETS
#define GS_FRAME_SETS 3
#endif
// Frames in flight: per-frame buffers (FrameSet), statistics slots and timing events rotate over
// this many frames; frame f reuses frame f - kFrameSets's set once that frame has ended.
constexpr int kFrameSets = GS_FRAME_SETS;
// Frame statistics and timing events rotate over more slots than there are frame sets: the host
// reads a frame's statistics (and its events) whenever they have arrived and never waits for the
// frame kFrameSets back to enqueue the next one (the sets' reuse is ordered on the device).  With
// kFrameSets slots the host blocked every third row-strip frame for the one three back
// (G = 8 strip: enqueue p50 34 us, p90 280 us, so at most ~1.5 frames ran on the GPU at once).
#ifndef GS_SET_STREAMS
#define GS_SET_STREAMS kFrameSets
#endif
constexpr int kSetStreams = GS_SET_STREAMS;  // distinct streams of the frame sets
constexpr int kStatSlots = 8;
static_assert(kStatSlots >= kFrameSets && kStatSlots * 4 <= 64, "statistics slots (h_seq: 64 B)");
#ifndef GS_DEEP_TILES
#define GS_DEEP_TILES 1536
#endif
constexpr int kDeepTiles = GS_DEEP_TILES;  // frames of at most this many tiles keep kFrameSets in flight

struct FrameEvents {
    hipEvent_t ev[EV_COUNT] = {};
    bool pending = false;
    int level = 0;        // opts.timing of the frame: 1 every stage, 2 the composite only
    bool chunk1 = false;  // chunk 1 ran (its composite events were recorded)
};

constexpr uint32_t kNoSplit = 0xFFFFFFFFu;  // chunk threshold: every visible splat in chunk 0

// Depth keys <-> the float they encode (src/shaders.ts:36-40; monotone in distance along the
// view axis for both camera conventions).
float key_to_float(uint32_t k) {
    const uint32_t fu = (k & 0x80000000u) ? (k ^ 0x80000000u) : (k ^ 0x80000001u);
    float f;
    std::memcpy(&f, &fu, 4);
    return f;
}
uint32_t float_to_key(float f) {
    uint32_t fu;
    std::memcpy(&fu, &f, 4);
    return fu ^ ((fu >> 31) ? 0x80000001u : 0x80000000u);
}
// Threshold just past key k with its depth scaled by `factor` (> 1: farther).
uint32_t scaled_threshold(uint32_t k, float factor) {
    const float v = key_to_float(k) * factor;
    if (!std::isfinite(v)) return kNoSplit;
    const uint32_t t = float_to_key(v);
    return t >= kNoSplit - 1 ? kNoSplit : t + 1;
}

// A device group's member g >= 1 enqueues its strip from a host thread of its own, so a group
// frame costs the caller about one strip's enqueue instead of G of them (G = 8
// members enqueued one after another took ~270-400 us of host time, more than one GPU's frame).
// Hand-off: the caller posts a job number; the worker spins on it for up to kSpinNs after its last
// job (a frame loop never sleeps) and then blocks on a condition variable; the caller spins until
// every worker has finished enqueueing (its own strip runs meanwhile), then enqueues the gather.
struct GroupWorker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint32_t> posted{0};    // jobs posted by the caller
    std::atomic<uint32_t> finished{0};  // jobs the worker finished (rc / msg valid)
    std::atomic<bool> sleeping{false};
    std::atomic<bool> quit{false};
    void (*fn)(void*, int) = nullptr;   // the job: fn(arg, member), set before `posted` moves
    void* arg = nullptr;
    int member = 0;
    int rc = 0;
    std::string msg;
    int64_t t_start = 0, t_end = 0;  // the last job's start and end (steady clock, ns; GS_GROUP_TRACE)
    int64_t t_post_last = 0;         // when the last job was posted (steady clock, ns)
    std::atomic<int64_t> gap_ns{kSpinNs};  // running mean of the time between posts
    // After a job the worker waits for the next post: it pause-spins for kPauseNs, then yields its
    // core while it polls (another runnable thread, e.g. Node's event loop, gets the core), up to
    // min(kSpinNs, 2 x the mean time between posts) -- a frame loop's next post arrives well within
    // it -- and then sleeps on the condition variable.  (Round 4 pause-spun the full 2 ms: a G = 8
    // group above ~500 fps kept seven host cores at 100 %)
    static constexpr int64_t kSpinNs = 2000000;   // 2 ms
    static constexpr int64_t kPauseNs = 20000;    // 20 us
};

static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct gs_ctx {
    int device = 0;
    int num_cus = 256;
    int c1_occ = 0;               // k_chunk1 workgroups resident per CU (occupancy query)
    int c1_grid = 0;              // k_chunk1's grid: chunk1_grid(c1_occ, num_cus), co-resident
    uint64_t spin_ticks = 20000000;  // grid-barrier timeout: 200 ms of the device's wall clock
    float cut_margin = 0.0f;      // gs_debug_cut_margin: 0 default, < 0 no per-tile cut, > 0 the depth margin
    hipStream_t stream = nullptr;
    void* d_out = nullptr;
    size_t d_out_bytes = 0;
    FrameEvents fe[kStatSlots];  // rotating: frame t's events are read once frame t + kStatSlots needs the slot
    int fe_cur = 0;
    double acc_ms[ST_COUNT] = {};
    uint32_t acc_frames = 0;    // frames timed at level 1 (every stage)
    double acc_comp_ms = 0.0;   // composite time of every timed frame (levels 1 and 2)
    uint32_t comp_frames = 0;
    gs_stats stats{};
    // frame counts since gs_timings_reset (gs_stats::frames_*)
    uint32_t n_rendered = 0, n_chunked = 0, n_unsat = 0, n_seeded = 0;
    std::vector<std::pair<void*, uint64_t>> fbufs;  // gs_framebuffer_alloc'd buffers and their sizes
    // asynchronous readback (gs_readback_start/wait): a copy stream and a ring of events
    static constexpr int kReadbacks = 8;
    hipStream_t copy_stream = nullptr;
    hipEvent_t rb_src[kReadbacks] = {};   // the context stream's frames so far (the copy's source)
    hipEvent_t rb_done[kReadbacks] = {};  // the copy landed
    std::atomic<uint32_t> rb_next{0};     // tickets issued
    std::vector<void*> host_regs;         // gs_host_register'd buffers
    gs_scene* last_scene = nullptr;
    std::vector<gs_scene*> scenes;  // attached scenes; gs_ctx_destroy frees the survivors
    // A device group (gs_ctx_create with ndev > 1): one single-device member context per entry;
    // member g renders row strip g of G into its slice of a G-strip buffer on its device, then one
    // RCCL all-gather (ncclCommInitAll over distinct devices; in place) fills every member's
    // buffer.  A device list with repeats (tests on one GPU) gathers with peer copies instead.
    std::vector<gs_ctx*> members;
    std::vector<ncclComm_t> comms;
    // member g >= 1 renders into one of two strip buffers on its device (double-buffered: frame
    // f + 1 renders while frame f's strip is sent); member 0 renders straight into the image
    std::vector<std::array<void*, 2>> gbuf;
    std::vector<size_t> gbuf_bytes;
    std::vector<hipStream_t> gstream;  // [member] the gather's stream (sends; member 0: receives)
    std::vector<hipEvent_t> gev_rendered;             // [member] strip rendered (on the member's stream)
    std::vector<std::array<hipEvent_t, 2>> gev_sent;  // [member][buffer] strip sent (buffer free again)
    hipEvent_t gev_entry = nullptr, gev_gathered = nullptr;  // device 0: the caller's stream at entry, image complete
    std::vector<int> gbounds;          // tile-row boundaries of the members' strips (G + 1), K-balanced
    int gH = 0;                        // the image height gbounds were made for
    uint32_t gframe = 0;               // frames since gbounds were (re)made
    std::vector<std::unique_ptr<GroupWorker>> workers;  // [member] (g >= 1): its enqueue thread
    bool group_peer_copy = false;      // GS_GROUP_PEER_COPY=1 at creation: members on device 0 peer-copy
                                       // their strips too (tests of that path on a one-GPU box)
};

// Everything one frame writes.  kFrameSets sets, used by frames in turn, each with its own stream
// for the frame's culling, projection, binning and per-tile sort; the composite and the frame's
// end run on the caller's stream (its buffer, in call order) once those are done.  So the next
// frames' early kernels run while this frame composites, with one cross-stream wait per frame.
struct FrameSet {
    hipStream_t stream = nullptr;
    hipEvent_t ev_early = nullptr;      // the frame's culling .. per-tile sort done (set stream)
    hipEvent_t ev_out = nullptr;        // the frame's end (on the caller's stream)
    float4* r2 = nullptr;               // per-Gaussian box of rects wider than 16 tiles
    // composite slots (slot_c0 / slot_c1): records (3 float4), (depth key, index), packed rect
    float4* crec = nullptr;
    uint32_t* wlist = nullptr;          // [slots] wide splats of both chunks (ProjParams::wlist)
    uint2* skey = nullptr;
    uint32_t* srect = nullptr;
    uint32_t *c0 = nullptr, *c1 = nullptr;  // [parts]: slots per projection partition and chunk
    uint16_t* cand = nullptr;           // chunk-0 candidates per partition (k_cull): offsets
    uint32_t* units = nullptr;          // the frame's non-empty chunk-0 work units (k_cull)
    uint32_t* plist = nullptr;          // chunk 1: partitions that may hold chunk-1 splats (k_chunk1)
    uint32_t* plist0 = nullptr;         // chunk 0: partitions that may hold candidates (k_part_list)
    uint32_t* order = nullptr;          // [tiles] the composite's tile order (k_tile_sort)
    uint32_t* sidx = nullptr;           // [slots] storage index of each composite slot
    FrameCtl* ctl = nullptr;            // zero at a frame's start (the frame's end clears it)
    StatShard* stats = nullptr;         // [kStatShards], zero at a frame's start (likewise)
    uint32_t* bar = nullptr;            // k_chunk1's grid barrier: arrival count (zero between barriers), generation
    bool meta_clean = false;            // the set's last frame zeroed FrameCtl (see render_frame)
    // tile lists
    uint64_t kcap = 0;
    uint32_t *tvA = nullptr, *tvB = nullptr;  // tile lists: unordered (binning), sorted
    uint2* ranges = nullptr;
    uint32_t* bmat = nullptr;           // [kBinParts][n_tiles] binning partition counts / offsets
    uint32_t* tbase = nullptr;          // [n_tiles] tile totals, then list begins
    uint2* bchk = nullptr;              // [bin_chk_words(n_tiles)] binning's count checksums
    uint16_t* cut = nullptr;            // [n_tiles] the frame's per-tile cut bounds (k_part_list)
    uint32_t* cutb = nullptr;           // [kCutMaxBlocks] their minimum / maximum per block
    uint8_t* done = nullptr;
    uint32_t* c1tiles = nullptr;  // chunk 1: the tiles chunk 0 left unsaturated, compact
    uint32_t* umask = nullptr;          // chunk 1: the unsaturated tiles' bits, strip rows x umask_words
    size_t umask_cap = 0;
    int tiles_cap = 0;
    float4* state = nullptr;
    uint64_t state_cap = 0;
    float* seedh = nullptr;             // seeded frames: alpha mass by coarse cell and depth bucket (zero between frames)
    size_t seed_cap = 0;
};

struct gs_scene {
    gs_ctx* ctx = nullptr;
    uint64_t n = 0;
    int n_sh = 0;
    float4* geo = nullptr;              // geometry records (3 float4 per Gaussian)
    float4* shade = nullptr;            // packed SH coefficients (sh_quads float4 per Gaussian)
    float4* dbg = nullptr;              // per-Gaussian debug records (3 float4), allocated on demand
    float4* cull = nullptr;             // cull planes (two-phase projection)
    FrameSet fs[kFrameSets];            // per-frame buffers, rotating frame to frame
    int cur_fs = 0;                     // the set the next frame uses
    int last_fs = 0;                    // the set of the last frame
    uint32_t* orig = nullptr;           // [n] reference index of each storage slot (Morton order)
    PartBound* bounds = nullptr;        // [parts] partition bounds (upload)
    PartBound* bbounds = nullptr;       // [ceil(n / kCullBlock)] block bounds (upload)
    ProjParams last_pp{};               // the last frame's projection (k_records for the debug dump)
    int last_tiles = 0;                 // tiles of the last frame's strip
    // asynchronous frame statistics (chunk controller, capacity): the frame's end (k_chunk1) stores FrameCtl into
    // a pinned slot and then publishes a sequence number there; kStatSlots slots
    FrameCtl* h_ctl = nullptr;    // pinned, coherent, device-mapped (d_ctl_slot): kStatSlots slots
    uint32_t* h_seq = nullptr;    // pinned, coherent, device-mapped (d_seq): per slot
    FrameCtl* d_ctl_slot = nullptr;
    uint32_t* d_seq = nullptr;
    uint32_t seq_next = 1;
    uint32_t stat_want[kStatSlots] = {};   // sequence number that completes the slot's frame
    uint32_t stat_base[kStatSlots] = {};   // the slot's frame's saturation-histogram base (sat_bucket)
    bool stat_pending[kStatSlots] = {};
    int stat_cur = 0;
    FrameCtl last{};            // latest harvested statistics
    uint32_t pending_err = 0;   // error bits of every harvested frame not yet reported (sticky)
    uint64_t overflow_k = 0;    // largest k_total of a harvested frame that overflowed the tile lists
    bool have_last = false;
    uint32_t chunk_T = kNoSplit;        // adaptive chunk threshold for the next frame
    float last_view[16] = {};           // the last frame's view matrix (a moving camera widens T)
    float last_campos[3] = {};          // ... and camera position (camera cuts)
    bool have_view = false;
    uint32_t cut_seq = 0;               // statistics of frames before this sequence number (the
                                        // last camera cut) do not steer the chunk controller
    bool hist_ok = false;               // the controller has statistics of this view (since the last cut)
    uint32_t key_lo = 0, key_hi = 0;    // depth-key range of the last frame's visible splats
    bool have_krange = false;
    bool have_frame = false;
    // ref_quirks (src/renderer.ts:306): the init-sort slots' state and the draw-ordered copy,
    // allocated by the first ref_quirks frame (quirk_prepare)
    uint32_t *qk = nullptr, *qv = nullptr;        // [n] state: (key, value) of slots >= nk after the last sort
    uint32_t *qK = nullptr, *qV = nullptr, *qK2 = nullptr, *qV2 = nullptr;  // [n] slots, sort ping-pong
    uint32_t* qinv = nullptr;                     // [n] storage slot of each reference index
    float4 *qgeo = nullptr, *qshade = nullptr, *qcull = nullptr;  // the scene in draw order
    uint32_t* qorig = nullptr;                    // [n] = draw rank
    PartBound* qbounds = nullptr;
    const uint32_t* qdraw = nullptr;              // [n] Gaussian of each draw rank, last ref_quirks frame
    bool last_quirk = false;                      // the last frame ran with ref_quirks
    std::vector<gs_scene*> members;               // a device group's scene: one replica per member
    // per-tile cut (kCutMaxTiles): [tiles of the W x H frame] the depth key at which each tile last
    // saturated (kSentinel: unknown), written by the composites, read by the next frames
    uint32_t* tile_sat = nullptr;
    int sat_W = 0, sat_H = 0;
};

static constexpr size_t kHistWords = kHistShards * 256;

// Largest scene for which the reference's init-sort dispatch is valid: max(N/8, 8) workgroups
// <= 65535 (src/renderer.ts:306; beyond it WebGPU rejects the dispatch and no key is written).
static constexpr uint64_t kQuirkMaxN = 65535ull * 8;
static constexpr int kMaxGroup = 64;  // devices per context
// radix partition sizes (items per thread x 256): small partitions keep every CU busy on the
// short depth sorts; the tile-id sort is long enough for 4096-element partitions
// radix partition size of gs_debug_sort_pairs (items per thread x 256)
static constexpr int kDepthSortIpt = 8;
// chunk-0 threshold: the farthest saturation key of the last frame, its depth scaled by this
// (bench scene: 1.15 -> 1.05 was 2766 -> 2915 fps static, 1.05 -> 1.01 3262 -> 3318 and at
// 50 M / 4K 1511 -> 1655; a moving camera multiplies in kMovingMargin, and the tiles that
// saturate later than the margin finish in chunk 1)
#ifndef GS_CHUNK_MARGIN
#define GS_CHUNK_MARGIN 1.01f
#endif
static constexpr float kChunkMargin = GS_CHUNK_MARGIN;
#ifndef GS_MOVING_MARGIN
#define GS_MOVING_MARGIN 1.09f
#endif
static constexpr float kMovingMargin = GS_MOVING_MARGIN;  // extra depth margin while the view changes
// split the visible splats into two chunks when at least this share of the tiles saturated in the
// last frame; chunk 1 then visits only the partitions that can reach an unsaturated tile
#ifndef GS_SPLIT_SAT_FRAC
#define GS_SPLIT_SAT_FRAC 0.2
#endif
static constexpr double kSplitSatFrac = GS_SPLIT_SAT_FRAC;
// ... at this quantile of the saturated tiles' saturation depths (GS_SAT_QUANTILE overrides),
// when the deepest saturation is more than kQuantileGain times deeper
#ifndef GS_QUANTILE_GAIN
#define GS_QUANTILE_GAIN 1.5f
#endif
static constexpr float kQuantileGain = GS_QUANTILE_GAIN;
static double sat_quantile() {
    static const double q = [] {
        const char* e = std::getenv("GS_SAT_QUANTILE");
        const double v = e ? std::atof(e) : 0.95;
        return v > 0.0 && v <= 1.0 ? v : 0.95;
    }();
    return q;
}
static_assert(sizeof(FrameCtl) <= 256, "FrameCtl too large");

static Records records(gs_scene* s, const FrameSet& F) {
    return Records{s->dbg, F.r2, 3u, 0u};
}

static void ensure_tile_capacity(FrameSet& F, uint64_t k) {
    if (k <= F.kcap && F.tvA) return;
    if (k >= 0xFFFFFFFFull) throw GsError(GS_ERR_UNSUPPORTED, "more than 2^32 tile entries");
    const uint64_t cap = std::min<uint64_t>(0xFFFFFFFEull, std::max<uint64_t>(k + k / 2, 1u << 20));
    dev_free(F.tvA); dev_free(F.tvB);
    dev_alloc(F.tvA, cap); dev_alloc(F.tvB, cap);
    F.kcap = cap;
}

static void ensure_tiles(FrameSet& F, int n_tiles) {
    if (n_tiles <= F.tiles_cap && F.ranges) return;
    dev_free(F.ranges);
    dev_free(F.done);
    dev_free(F.c1tiles);
    dev_free(F.bmat);
    dev_free(F.tbase);
    dev_free(F.bchk);
    dev_free(F.cut);
    dev_free(F.cutb);
    dev_free(F.order);
    dev_alloc(F.ranges, (size_t)n_tiles);
    dev_alloc(F.cut, (size_t)n_tiles);
    dev_alloc(F.cutb, (size_t)kCutMaxBlocks);
    dev_alloc(F.bchk, (size_t)bin_chk_words((uint32_t)n_tiles));
    dev_alloc(F.order, (size_t)n_tiles);
    dev_alloc(F.done, (size_t)n_tiles);
    dev_alloc(F.c1tiles, (size_t)n_tiles);
    dev_alloc(F.bmat, (size_t)kBmatRows * n_tiles);
    dev_alloc(F.tbase, (size_t)n_tiles);
    F.tiles_cap = n_tiles;
    F.meta_clean = false;  // (the new checksum array is zeroed with FrameCtl)
}

static void ensure_umask(FrameSet& F, size_t words) {
    if (words <= F.umask_cap && F.umask) return;
    dev_free(F.umask);
    dev_alloc(F.umask, words);
    F.umask_cap = words;
}

static void ensure_seed(FrameSet& F, size_t words) {
    if (words <= F.seed_cap && F.seedh) return;
    dev_free(F.seedh);
    dev_alloc(F.seedh, words);
    // zeroed on the set's stream, ahead of the k_seed_hist that reads it (a plain hipMemset runs
    // on the null stream, which does not order against the non-blocking set streams);
    // k_seed_pick re-zeroes what it read
    HIPCHK(hipMemsetAsync(F.seedh, 0, words * sizeof(float), F.stream));
    F.seed_cap = words;
}

static void ensure_state(FrameSet& F, uint64_t pixels) {
    if (pixels <= F.state_cap && F.state) return;
    dev_free(F.state);
    dev_alloc(F.state, pixels);
    F.state_cap = pixels;
}

static void ensure_out(gs_ctx* c, size_t bytes) {
    if (bytes <= c->d_out_bytes && c->d_out) return;
    if (c->d_out) (void)hipFree(c->d_out);
    c->d_out = nullptr;
    HIPCHK(hipMalloc(&c->d_out, bytes));
    c->d_out_bytes = bytes;
}

// (P*V) in the reference's evaluation order (src/simple_render.ts:228, WGSL mat4 product).
static void mat4_mul_ref(const float* A, const float* B, float* R) {
#pragma clang fp contract(off)
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i)
            R[4 * j + i] = ((A[i] * B[4 * j + 0] + A[4 + i] * B[4 * j + 1]) + A[8 + i] * B[4 * j + 2]) +
                           A[12 + i] * B[4 * j + 3];
}

static void strip_geometry(int H, int si, int sc, int& tr_begin, int& tr_end, int& rows_padded) {
    const int TR = (H + kTile - 1) / kTile;
    const int per = (TR + sc - 1) / sc;
    tr_begin = std::min(si * per, TR);
    tr_end = std::min((si + 1) * per, TR);
    rows_padded = per * kTile;
}

// The rows a frame renders and its output buffer: tile rows [tb, te); the buffer holds `rows`
// image rows from image row `row0` (`pad` of them past the image: zero padding of the last
// equal strip).  Explicit tile-row ranges (gs_opts.tile_row_end > 0) have no padding.
struct FrameRows {
    int tb, te, row0, rows, pad;
};
static FrameRows frame_rows(int H, const gs_opts& o) {
    FrameRows r{};
    if (o.tile_row_end > 0) {
        r.tb = o.tile_row_begin;
        r.te = o.tile_row_end;
        r.row0 = r.tb * kTile;
        r.rows = std::min(r.te * kTile, H) - r.row0;
        return r;
    }
    const int sc = std::max(1, o.strip_count);
    int rp;
    strip_geometry(H, o.strip_index, sc, r.tb, r.te, rp);
    r.row0 = sc > 1 ? r.tb * kTile : 0;
    r.rows = sc > 1 ? rp : H;
    r.pad = sc > 1 ? std::min(rp, std::max(0, r.row0 + rp - H)) : 0;
    return r;
}

// gs_opts of the caller, read up to its struct_size (callers built against an older header pass a
// shorter struct; the fields past it keep their defaults).
static gs_opts read_opts(const gs_opts* opts) {
    gs_opts o;
    gs_opts_default(&o);
    if (opts) {
        const size_t n = std::min<size_t>(sizeof(gs_opts), opts->struct_size ? opts->struct_size : sizeof(gs_opts));
        std::memcpy(&o, opts, n);
        o.struct_size = sizeof(gs_opts);
    }
    return o;
}

// K-balanced strips: new tile-row boundaries that equalise the strips' costs, the cost of each
// current strip taken as spread evenly over its rows, each boundary moved half way to that
// model's cut (every strip keeps >= 1 row when TR >= G).
static void balance_bounds(int G, int TR, const int* b, const double* cost, int* nb) {
    double total = 0.0;
    for (int g = 0; g < G; ++g) total += std::max(0.0, cost[g]);
    nb[0] = 0;
    nb[G] = TR;
    if (!(total > 0.0) || TR < G) {
        for (int g = 1; g < G; ++g) nb[g] = b[g];
        return;
    }
    int seg = 0;
    double cum = 0.0;  // cost of rows [0, b[seg])
    for (int k = 1; k < G; ++k) {
        const double want = total * k / G;
        while (seg < G - 1 && cum + std::max(0.0, cost[seg]) < want) cum += std::max(0.0, cost[seg++]);
        const int rows = b[seg + 1] - b[seg];
        const double c = std::max(0.0, cost[seg]);
        const double x = b[seg] + (c > 0.0 && rows > 0 ? (want - cum) / c * rows : 0.0);
        // half way from the old boundary: the even-spread model over- or undershoots where the
        // cost is concentrated (a dense band of rows); damped, the feedback converges
        int r = (int)std::lround(0.5 * (x + b[k]));
        if (r == b[k] && std::fabs(x - b[k]) >= 0.5) r += x > b[k] ? 1 : -1;  // at least one row toward it
        r = std::max(r, nb[k - 1] + 1);
        r = std::min(r, TR - (G - k));
        nb[k] = r;
    }
}

static void harvest(gs_ctx* c, FrameEvents& f) {
    if (!f.pending) return;
    auto el = [&](int a, int b) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, f.ev[a], f.ev[b]));
        return (double)ms;
    };
    HIPCHK(hipEventSynchronize(f.ev[f.level == 1 ? EV_END : EV_COMP_0]));
    c->acc_comp_ms += el(EV_RANGES_0, EV_COMP_0);
    c->comp_frames++;
    if (f.level != 1) {
        f.pending = false;
        return;
    }
    c->acc_ms[ST_TOTAL] += el(EV_BEGIN, EV_END);
    c->acc_ms[ST_PROJECT] += el(EV_PROJ0, EV_PROJ1);
    c->acc_ms[ST_SORT] += f.chunk1 ? el(EV_COMP_0, EV_COMP_1) : 0.0;  // chunk 1 (k_chunk1)
    c->acc_ms[ST_BIN] += el(EV_DSORT_0, EV_BIN_0);
    c->acc_ms[ST_TSORT] += el(EV_BIN_0, EV_TSORT_0);
    c->acc_ms[ST_RANGES] += el(EV_TSORT_0, EV_RANGES_0);
    c->acc_frames++;
    f.pending = false;
}

static bool seq_arrived(const gs_scene* s, int slot) {
    return __atomic_load_n(&s->h_seq[slot], __ATOMIC_ACQUIRE) == s->stat_want[slot];
}

// Spin until the frame's end (k_chunk1) published `slot`'s sequence number.  `st` (nullable) is a stream the
// signal is queued on: polled now and then, so a fault surfaces as an error, not a hang.
// Without a stream: a device synchronize if the signal is late.  False: it never came.
static bool wait_slot(gs_scene* s, int slot, hipStream_t st) {
    for (uint32_t it = 1;; ++it) {
        if (seq_arrived(s, slot)) return true;
        if ((it & 255u) == 0) {
            if (st) {
                const hipError_t e = hipStreamQuery(st);
                if (e == hipSuccess) return seq_arrived(s, slot);
                if (e != hipErrorNotReady) HIPCHK(e);
            } else {
                HIPCHK(hipDeviceSynchronize());
                return seq_arrived(s, slot);
            }
        }
        __builtin_ia32_pause();
    }
}

// Latest frame statistics that have arrived on the host; `wait` blocks for the newest frame.
static void collect_stats(gs_scene* s, bool wait) {
    for (int k = 0; k < kStatSlots; ++k) {
        const int slot = (s->stat_cur + k) % kStatSlots;  // oldest slot first
        if (!s->stat_pending[slot]) continue;
        if (!seq_arrived(s, slot)) {
            if (!wait) continue;
            if (!wait_slot(s, slot, nullptr)) {  // the frame never completed (an error mid-frame)
                s->stat_pending[slot] = false;
                continue;
            }
        }
        s->last = s->h_ctl[slot];
        s->pending_err |= s->last.err;  // an older frame's error is not overwritten by a newer clean frame
        if (s->last.err & kErrOverflow) s->overflow_k = std::max<uint64_t>(s->overflow_k, s->last.k_total);
        if (s->last.not_done > 0) s->ctx->n_unsat++;
        s->have_last = true;
        s->stat_pending[slot] = false;
        if (s->stat_want[slot] < s->cut_seq) continue;  // a view before the last camera cut
        s->hist_ok = true;
        // chunk controller: chunk 0 = the splats nearer than 1.15x the depth at which the last
        // tile saturated (measured by the composite), rising at once, decaying slowly (3 % of
        // depth per frame); frames where most tiles never saturate use one chunk
        const FrameCtl& l = s->last;
        if (l.n_vis > 0 && ~l.key_min_inv <= l.key_max) {  // depth range (fixed-fraction chunking)
            s->key_lo = ~l.key_min_inv;
            s->key_hi = l.key_max;
            s->have_krange = true;
        }
        // the threshold sits past the depth at which all but a (1 - q) share of the saturated
        // tiles saturated (the upper edge of that histogram bucket, then the margin); the
        // later-saturating tiles complete in chunk 1
        uint32_t sat_tiles = 0;
        for (int k = 0; k < kSatBuckets; ++k) sat_tiles += l.sat_hist[k];
        uint32_t target = kNoSplit;
        if (l.n_vis > 0 && l.sat_key != 0 && sat_tiles >= kSplitSatFrac * std::max(1, s->last_tiles)) {
            const double want = sat_quantile() * sat_tiles;
            uint32_t cum = 0;
            int b = 0;
            for (; b < kSatBuckets - 1; ++b) {
                cum += l.sat_hist[b];
                if (cum >= want) break;
            }
            uint32_t edge = l.sat_key;
            if (b < kSatBuckets - 1) {
                const uint64_t e = ((uint64_t)s->stat_base[slot] + (uint64_t)b + 1) << kSatShift;
                const uint32_t eq = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(e, 0xFFFFFFFEull), l.sat_key);
                // the quantile only when the last tiles saturate much deeper than the rest (a
                // moving camera, sparse regions): otherwise chunk 1's launches cost more than the
                // smaller chunk 0 saves
                const float dq = std::fabs(key_to_float(eq)), dm = std::fabs(key_to_float(l.sat_key));
                if (dm > kQuantileGain * dq) edge = eq;
            }
            target = scaled_threshold(edge, kChunkMargin);
        }
        if (target >= s->chunk_T || s->chunk_T == kNoSplit)
            s->chunk_T = target;
        else
            s->chunk_T = std::max(target, scaled_threshold(s->chunk_T, 0.97f));
    }
}

static void quirk_prepare(gs_scene* s, const float* uni, hipStream_t st);

// Seeded frames (k_seed_*): the alpha mass per pixel taken as saturation (sum of alpha >=
// -ln(1e-4) = 9.21 leaves T < 1e-4), GS_SEED_TAU overrides; GS_SEED=0 disables seeding (a cold
// frame is then one chunk).
static double seed_tau() {
    static const double v = [] {
        const char* e = std::getenv("GS_SEED_TAU");
        const double x = e ? std::atof(e) : 9.21;
        return x > 0.0 ? x : 9.21;
    }();
    return v;
}
static uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = std::getenv(name);
    return e ? (uint32_t)std::atoi(e) : dflt;
}
// Binning partitions (A/B runs: GS_NPARTS_MOVE, GS_NPARTS_C1 = 128 or 256)
static uint32_t env_nparts(const char* name, uint32_t dflt) {
    const char* e = std::getenv(name);
    const uint32_t v = e ? (uint32_t)std::atoi(e) : dflt;
    return v == kBinPartsSmall || v == (uint32_t)kBinParts ? v : dflt;
}
// ... each partition holding at most kBinMaxUnits of the frame's units (else kBinParts)
static uint32_t fit_nparts(uint32_t parts, uint32_t want) {
    return (uint64_t)parts * kProjRounds <= (uint64_t)kBinMaxUnits * want ? want : (uint32_t)kBinParts;
}
// Per-tile chunk-0 cut (kCutMaxTiles; GS_TILE_CUT=0 turns it off, for A/B runs)
static bool tile_cut_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("GS_TILE_CUT");
        return !(e && e[0] == '0');
    }();
    return v;
}
static bool seed_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("GS_SEED");
        return !(e && e[0] == '0');
    }();
    return v;
}
// Depth bucket 0 of the seed histogram: the near plane's key (clip z = 0 on the view axis:
// vz = -P[14] / P[10]); the buckets are sat_bucket's quarter octaves of depth from there.
static uint32_t seed_base(const float* uni) {
    const float p10 = uni[16 + 10], p14 = uni[16 + 14];
    const float vz = p10 != 0.0f ? -p14 / p10 : 0.0f;
    if (!std::isfinite(vz) || vz == 0.0f) return 0u;
    return float_to_key(vz) >> kSatShift;
}

// A camera cut: the view turned by more than kCutAngle against the last frame, or the camera moved
// by more than kCutShift of the depth at which the last frame's tiles saturated.  The chunk
// controller's history (saturation depths of earlier frames) then describes another view.
constexpr float kCutCos = 0.98480775f;  // cos 10 deg
constexpr float kCutShift = 0.1f;
static bool camera_cut(const gs_scene* s, const float* uni) {
    if (!s->have_view) return false;
    const float* a = s->last_view;  // view row 2 (column-major): the camera's depth axis in world space
    const double da = std::sqrt((double)a[2] * a[2] + (double)a[6] * a[6] + (double)a[10] * a[10]);
    const double db = std::sqrt((double)uni[2] * uni[2] + (double)uni[6] * uni[6] + (double)uni[10] * uni[10]);
    const double dot = (double)a[2] * uni[2] + (double)a[6] * uni[6] + (double)a[10] * uni[10];
    if (!(da > 0.0 && db > 0.0) || !(dot >= kCutCos * da * db)) return true;
    if (!s->have_last) return false;
    const uint32_t ref = s->last.sat_key ? s->last.sat_key : s->key_hi;
    const double dref = std::fabs((double)key_to_float(ref)) / da;  // world units (the view's scale is da)
    double d2 = 0.0;
    for (int k = 0; k < 3; ++k) d2 += ((double)uni[32 + k] - s->last_campos[k]) * ((double)uni[32 + k] - s->last_campos[k]);
    return std::isfinite(dref) && dref > 0.0 && std::sqrt(d2) > kCutShift * dref;
}

// The per-frame pipeline.  `out` is device memory of rows_padded*W (strip) or H*W pixels.
static void render_frame(gs_ctx* c, gs_scene* s, const float* uni, int W, int H, const gs_opts& o,
                         void* out, hipStream_t st) {
    const FrameRows fr = frame_rows(H, o);
    const int tr_begin = fr.tb, tr_end = fr.te;
    const int TX = (W + kTile - 1) / kTile;
    const int n_tiles = TX * (tr_end - tr_begin);
    FrameSet& F = s->fs[s->cur_fs];
    {  // frames in flight: three for small frames (row strips: latency-bound kernels, so a third
       // frame's early kernels fill the GPU; measured G=8 strip 0.156 -> 0.144 ms), two for large
       // ones (a third only adds contention: 448 -> 461 us at the bench configuration)
        const int depth = n_tiles <= kDeepTiles ? kFrameSets : 2;
        if (depth < kFrameSets) HIPCHK(hipEventSynchronize(s->fs[(s->cur_fs + kFrameSets - depth) % kFrameSets].ev_out));
    }
    // culling .. per-tile sort run on the set's stream, the composite and the frame's end on the
    // caller's stream `st`.  Stage timing (level 1) serialises the frames so that each stage's
    // events measure that stage alone.
    const hipStream_t cst = st;
    st = F.stream;
    {  // the set's last frame ended (normally long ago: then the host skips the wait, ~3 us of enqueue)
        const hipError_t q = hipEventQuery(F.ev_out);
        if (q == hipErrorNotReady) HIPCHK(hipStreamWaitEvent(st, F.ev_out, 0));
        else HIPCHK(q);
    }
    if (o.timing == 1) HIPCHK(hipStreamWaitEvent(st, s->fs[s->last_fs].ev_out, 0));
    collect_stats(s, false);
    const int slot = s->stat_cur;  // this frame's statistics slot
    if (s->stat_pending[slot]) {  // the slot's last frame (kStatSlots ago): its statistics first
        wait_slot(s, slot, nullptr);
        collect_stats(s, false);
        s->stat_pending[slot] = false;
    }
    if (s->have_last && s->last.k_total > F.kcap) ensure_tile_capacity(F, s->last.k_total);
    ensure_tiles(F, std::max(n_tiles, 1));
    s->last_tiles = n_tiles;
    // chunk threshold: adaptive, one chunk (chunk_fraction >= 1), or a fixed split for tests and
    // diagnostics (chunk_fraction in (0,1): the depth 2^-t <= chunk_fraction of the way from the
    // last frame's nearest to its farthest visible splat; one chunk until a frame was seen)
    if (camera_cut(s, uni)) {  // the earlier frames' saturation depths say nothing about this view
        s->cut_seq = s->seq_next;
        s->chunk_T = kNoSplit;
        s->hist_ok = false;
    }
    uint32_t T = s->chunk_T;
    bool moving = false;
    {  // the statistics are a few frames old: while the camera moves, the depth at which tiles
       // saturate moves too, so the threshold gets a wider margin (kChunkMargin x kMovingMargin
       // ~ 1.10 measured best over 1080p and 4K orbits, tools/gpu_margin_sweep.sh); a still camera
       // keeps the tight one
        moving = std::memcmp(s->last_view, uni, sizeof(s->last_view)) != 0;
        std::memcpy(s->last_view, uni, sizeof(s->last_view));
        std::memcpy(s->last_campos, uni + 32, sizeof(s->last_campos));
        s->have_view = true;
        if (moving && T != kNoSplit) T = scaled_threshold(T, kMovingMargin);
    }
    const bool cold = !s->hist_ok && o.chunk_fraction == 0.0f && !o.ref_quirks;  // no usable history
    if (o.chunk_fraction >= 1.0f) {
        T = kNoSplit;
    } else if (o.chunk_fraction > 0.0f) {
        const int t = std::min(7, std::max(0, (int)std::ceil(-std::log2((double)o.chunk_fraction))));
        T = kNoSplit;
        if (s->have_krange) {
            const float v0 = key_to_float(s->key_lo), v1 = key_to_float(s->key_hi);
            const float v = v0 + (v1 - v0) * std::ldexp(1.0f, -t);
            const uint32_t k = float_to_key(v);
            if (std::isfinite(v) && k < kNoSplit - 1) T = k + 1;
        }
    }
    const bool quirk = o.ref_quirks != 0;
    if (quirk) {
        T = kNoSplit;  // one chunk: the slot keys are draw ranks
        quirk_prepare(s, uni, F.stream);
    }
    s->last_quirk = quirk;
    // no usable history: the frame estimates its own threshold on the device (k_seed_*)
    const bool seeded = cold && n_tiles > 0 && s->n > 0 && seed_enabled();
    const bool two_chunks = T != kNoSplit || seeded;
    if (s->sat_W != W || s->sat_H != H || !s->tile_sat) {  // the per-tile saturation keys of this frame size
        const size_t tiles = (size_t)TX * (size_t)((H + kTile - 1) / kTile);
        if (s->tile_sat) {
            HIPCHK(hipDeviceSynchronize());  // (earlier frames' composites may still write the old table)
            dev_free(s->tile_sat);
        }
        dev_alloc(s->tile_sat, tiles);
        HIPCHK(hipMemsetAsync(s->tile_sat, 0xFF, tiles * 4, st));  // kSentinel: no cut yet (before k_part_list reads it)
        s->sat_W = W;
        s->sat_H = H;
    }
    // the per-tile cut: chunked frames with history (not seeded: a cut's view has none), when the
    // band's bounds fit the binning's LDS; under ref_quirks the slot keys are draw ranks (one chunk)
    // and a still camera: under a moving one each tile's content (and saturation depth) shifts
    // between frames, the last frame's per-tile bounds leave tiles unsaturated and chunk 1 then
    // re-walks chunk 0 (bench orbit 2372 -> 1433 fps with the cut on moving frames)
    // and whole frames (a row strip's chunk 0 is a few hundred entries per tile after a G-fold
    // shorter chain: the cut's classification and bound reads cost more than they save there,
    // 50 M / 4K G = 8 strip 0.140 -> 0.153 ms, 1080p G = 8 equal)
    const bool cut_on = two_chunks && !seeded && !quirk && !moving && fr.tb == 0 && fr.te * kTile >= H &&
                        n_tiles > 0 && n_tiles <= kCutMaxTiles &&
                        cut_blocks(TX, tr_end - tr_begin) <= (uint32_t)kCutMaxBlocks && tile_cut_enabled() &&
                        c->cut_margin >= 0.0f;
    c->n_rendered++;
    c->n_chunked += two_chunks ? 1u : 0u;
    c->n_seeded += seeded ? 1u : 0u;
    const int seed_cx = (W + kSeedCell - 1) / kSeedCell;
    const int seed_cy = ((std::min(tr_end * kTile, H) - tr_begin * kTile) + kSeedCell - 1) / kSeedCell;
    if (seeded) ensure_seed(F, (size_t)seed_cx * std::max(seed_cy, 1) * kSeedBuckets);
    if (two_chunks) {
        ensure_state(F, (uint64_t)W * H);
        ensure_umask(F, (size_t)(tr_end - tr_begin) * umask_words(TX));
    }

    // timing 1: events between every stage; 2: around the composite only (each event record costs
    // the stream a few microseconds, so a frame timed at level 1 runs slower)
    const bool timed = o.timing != 0;
    FrameEvents& fe = c->fe[c->fe_cur];
    auto mark = [&](int e) {
        if (!timed) return;
        if (o.timing != 1 && e != EV_RANGES_0 && e != EV_COMP_0 && e != EV_RANGES_1 && e != EV_COMP_1) return;
        HIPCHK(hipEventRecord(fe.ev[e], st));
    };
    if (timed) {
        harvest(c, fe);  // slot reuse: its frame completed long ago (or wait for it)
        fe.level = o.timing;
        fe.chunk1 = two_chunks;
    }
    mark(EV_BEGIN);

    // FrameCtl is zero at a frame's start: the end of the set's last frame cleared it, unless that
    // frame never ended (first frame, an error mid-frame)
    if (!F.meta_clean) {  // (and the binning checksums: k_bin_emit zeroes them only when it ran)
        HIPCHK(hipMemsetAsync(F.bchk, 0, (size_t)bin_chk_words((uint32_t)F.tiles_cap) * sizeof(uint2), st));
        HIPCHK(hipMemsetAsync(F.ctl, 0, sizeof(FrameCtl), st));
        HIPCHK(hipMemsetAsync(F.stats, 0, kStatShards * sizeof(StatShard), st));
        HIPCHK(hipMemsetAsync(F.bar, 0, 16, st));
    }
    F.meta_clean = false;
    ProjParams pp{};
    pp.geo = s->geo;
    pp.cull = s->cull;
    pp.n = n_tiles > 0 ? (uint32_t)s->n : 0u;
    std::memcpy(pp.V, uni + 0, 64);
    mat4_mul_ref(uni + 16, uni + 0, pp.PV);
    pp.scale_mod = uni[39];
    std::memcpy(pp.cam, uni + 32, 12);
    pp.P00 = uni[16];
    pp.P11 = uni[21];
    pp.focal = (float)W * pp.P00 / 2.0f;
    {  // lambda_max of the 2x2 Gram matrix of W3's rows 0 and 1 (row r = V[r], V[4 + r], V[8 + r])
        double g[2][2];
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 2; ++q)
                g[r][q] = (double)uni[r] * uni[q] + (double)uni[4 + r] * uni[4 + q] + (double)uni[8 + r] * uni[8 + q];
        const double m = 0.5 * (g[0][0] + g[1][1]), h = 0.5 * (g[0][0] - g[1][1]);
        const double lmax = m + std::sqrt(h * h + g[0][1] * g[0][1]);
        pp.w01_spec2 = std::isfinite(lmax) ? (float)(lmax * 1.0001 + 1e-30) : INFINITY;  // NaN view: never cull
    }
    pp.W = W;
    pp.H = H;
    pp.tile_row_begin = tr_begin;
    pp.tile_row_end = tr_end;
    pp.tiles_x = TX;
    pp.rec = records(s, F);
    pp.sh = s->shade;
    pp.shq = sh_quads(s->n_sh);
    pp.ctl = F.ctl;
    pp.stats = F.stats;
    pp.thresh = T;
    pp.crec = F.crec;
    pp.skey = F.skey;
    pp.srect = F.srect;
    pp.c0 = F.c0;
    pp.c1 = F.c1;
    pp.cand = F.cand;
    pp.units = F.units;
    pp.plist0 = F.plist0;
    pp.bounds = s->bounds;
    pp.bbounds = s->bbounds;
    pp.orig = s->orig;
    pp.sidx = F.sidx;
    pp.wlist = F.wlist;
    pp.wide_tiles = wide_tiles(n_tiles);
    pp.tile_sat = s->tile_sat;
    pp.cut = cut_on ? F.cut : nullptr;
    pp.cutb = F.cutb;
    pp.cut_margin = c->cut_margin > 0.0f ? c->cut_margin : kChunkMargin;
    pp.umask = two_chunks ? F.umask : nullptr;  // (chunk 1's rectangle tests; zeroed by k_part_list)
    pp.umask_w = umask_words(TX);
    // Grids of the frame's culling and projection, which run beside the previous frame's composite
    // (tools/ab_env.sh, two runs each): k_cull on 1024 workgroups for a still camera, 512 when it
    // moves (2048 before: bench 3485-3506 -> 3625-3628 fps, 1536: 3502, 768: 3614-3625, the
    // composite beside it 175.5 -> 171 us; cold frames 2690-2696 -> 2767-2779 with 512, 1024:
    // 2755; orbit unchanged); k_project on 1280 for a still camera (1536 before: bench 3625 -> 3640;
    // 1024: 3464; 768 under a moving camera made the orbit slower, 2526-2530 against 2538-2545).
    // GS_CULL_GRID_STILL, GS_CULL_GRID_MOVE, GS_PROJ_GRID_STILL override (A/B runs).
    static const uint32_t cull_grid_move = env_u32("GS_CULL_GRID_MOVE", 512u);
    static const uint32_t cull_grid_still = env_u32("GS_CULL_GRID_STILL", 1024u);
    static const uint32_t proj_grid_still = env_u32("GS_PROJ_GRID_STILL", 1280u);
    pp.cull_grid = moving ? cull_grid_move : cull_grid_still;
    pp.proj_grid = moving ? 0u : proj_grid_still;
    if (seeded) {
        pp.thresh = kNoSplit;
        pp.thresh_dev = &F.ctl->seed_T;
        pp.seedh = F.seedh;
        const uint64_t runs = (s->n + kSeedRun - 1) / kSeedRun, want = (uint64_t)kSeedRunsPerCell * seed_cx * seed_cy;
        pp.seed_stride = (uint32_t)std::max<uint64_t>(1u, runs / std::max<uint64_t>(want, 1));
        pp.seed_base = seed_base(uni);
        pp.seed_cx = seed_cx;
        pp.seed_cy = seed_cy;
        pp.seed_tau = seed_tau();
    }
    if (quirk) {  // the frame runs on the draw-ordered copy; each slot's sort key = (0, draw rank)
        pp.geo = s->qgeo;
        pp.cull = s->qcull;
        pp.sh = s->qshade;
        pp.bounds = s->qbounds;
        pp.bbounds = nullptr;  // (the draw-ordered copy has partition bounds only)
        pp.orig = s->qorig;
        pp.key_zero = 1;
    }
    mark(EV_PROJ0);
    if (seeded) launch_seed(pp, st);
    launch_project(pp, st);
    mark(EV_PROJ1);

    // ---- chunk 0: bin -> per-tile sort -> composite.  Chunk 1 (the splats at or past T that
    // touch a tile chunk 0 left unsaturated) is one launch enqueued behind it (64 workgroups,
    // grid barriers) that returns at once when chunk 0 saturated every tile (k_chunk1), or
    // separate launches when a recent frame left tiles unsaturated.
    BinParams bp{};
    bp.skey = F.skey;
    bp.sidx = F.sidx;
    bp.srect = F.srect;
    bp.cnt = F.c0;
    bp.parts = proj_parts(pp.n);
    bp.units = F.units;
    bp.rec = records(s, F);
    bp.crec = F.crec;
    bp.wlist = F.wlist;
    bp.wide_tiles = pp.wide_tiles;
    bp.done = F.done;
    bp.ctl = F.ctl;
    bp.chunk = 0;
    bp.tile_row_begin = tr_begin;
    bp.tiles_x = TX;
    bp.capacity = (uint32_t)F.kcap;
    bp.ranges = F.ranges;
    bp.n_tiles = (uint32_t)n_tiles;
    bp.bmat = F.bmat;
    bp.tbase = F.tbase;
    bp.bchk = F.bchk;
    // binning partitions: fewer under a moving camera and in chunk 1.  A moving frame is bound by
    // the caller's stream (chunk 0's composite, then chunk 1's chain); its chunk-0 binning runs
    // beside the previous frame's, and 128 workgroups of it leave that more of the device, while
    // chunk 1's few entries cost the per-partition work over every tile, not the walk.  Orbit
    // (tools/ab_env.sh, two runs each): 256 / 256 2431-2434 fps, 128 / 256 2460-2463, 256 / 128
    // 2414-2420, 128 / 128 2528-2533.  A still frame's chunk-0 binning is slower with 128 (85 ->
    // 111 us, bench 3507 -> 3434-3456 fps), so it keeps 256.
    // (frames of up to 16384 tiles: at 3840 x 2160 the moving frame's chunk 0 is bound by its own
    // binning, orbit 741 fps with 128 against 765 with 256)
    bp.nparts = fit_nparts(bp.parts, moving && n_tiles <= 16384 ? env_nparts("GS_NPARTS_MOVE", kBinPartsSmall)
                                                                 : (uint32_t)kBinParts);
    bp.cut = cut_on ? F.cut : nullptr;
    bp.cutb = F.cutb;
    bp.tvals = F.tvA;
    bp.rows = tr_end - tr_begin;
    bp.order = F.order;
    bp.stats = F.stats;
    {  // twice the last frame's mean chunk-0 list length (a frame with no history: no long lists)
        const uint64_t k0 = s->have_last ? s->last.k_chunk[0] : 0;
        bp.heavy_len = k0 ? (uint32_t)std::min<uint64_t>(2 * k0 / (uint64_t)std::max(1, n_tiles), 0xFFFFFFFFull)
                          : 0xFFFFFFFFu;
    }
    TileSortParams tsp{};  // each tile's list into (depth key, index) order
    tsp.ranges = F.ranges;
    tsp.in = F.tvA;
    tsp.out = F.tvB;
    tsp.skey = F.skey;
    tsp.done = nullptr;
    tsp.scratch = F.bmat;  // kBmatRows (>= 256) words per tile, dead once the emission has read them
    tsp.n_tiles = n_tiles;
    {  // lists of more than kTsBigMean entries on average (last frame; the 128-thread shape sorts rounds of 1024): most
       // tiles would take the multi-round path (each round re-reads the whole list), so the
       // 256-thread shape with rounds of 2048 (a moving camera at 4K: 1200 entries per tile)
        const uint64_t k0 = s->have_last ? s->last.k_chunk[0] : 0;
        tsp.big = n_tiles <= 0                                       ? 0
                  : k0 > (uint64_t)kTsHugeMean * (uint64_t)n_tiles ? 2
                  : k0 > (uint64_t)kTsBigMean * (uint64_t)n_tiles  ? 1
                                                                   : 0;
    }
    tsp.stats = F.stats;
    if (tsp.big == 2) {  // lists past one 7168-entry LDS round: the linear long-list path (256 threads);
                         // c1tiles is free until the composite appends chunk 1's tiles to it
        tsp.long_tiles = F.c1tiles;
        tsp.long_n = &F.ctl->long_n;
        tsp.long_grid = (uint32_t)std::min(n_tiles, 2 * c->num_cus);
    }
    CompositeParams cp{};
    cp.ranges = F.ranges;
    cp.tvals = F.tvB;
    cp.rec = F.crec;
    cp.order = F.order;
    cp.W = W;
    cp.H = H;
    cp.tiles_x = TX;
    cp.tile_row_begin = tr_begin;
    cp.row0 = fr.row0;
    cp.n_tiles = n_tiles;
    cp.t_min = o.t_min;
    cp.mode = two_chunks ? kCompFirst : kCompSingle;
    cp.state = F.state;
    cp.done = F.done;
    cp.c1tiles = two_chunks ? F.c1tiles : nullptr;
    cp.ctl = F.ctl;
    cp.stats = F.stats;
    cp.sat_base = s->have_krange ? (s->key_lo >> kSatShift) : 0u;
    s->stat_base[slot] = cp.sat_base;
    cp.out = out;
    cp.out_f16 = o.out_format == GS_OUT_RGBA_F16;
    cp.tile_sat = s->tile_sat;
    cp.umask = pp.umask;
    cp.umask_w = pp.umask_w;
    const bool split = o.list_split != 0 && o.accum != GS_ACCUM_FP16_TARGET;
    // chunk 0: as many wave pairs per tile as keep every tile resident (a function of the frame's
    // size only, so a view renders the same whatever came before it)
    cp.seg = split ? composite_seg(n_tiles, c->num_cus) : 1;
    {  // row bands (image-invariant): 4 when the last frame left most tiles unsaturated
        uint32_t sat_tiles = 0;
        for (int k = 0; k < kSatBuckets; ++k) sat_tiles += s->last.sat_hist[k];
        cp.bands = s->have_last && 2u * sat_tiles < (uint32_t)n_tiles ? 4 : 2;
    }
    mark(EV_DSORT_0);
    launch_bin(bp, st);
    mark(EV_BIN_0);
    // A still camera's chunk-0 per-tile sort in the composite's launch (composite_sorts): the set
    // stream's chain then ends with the emission, and a still frame waits for the end of that chain
    // (bench 3626-3640 -> 3683-3695 fps).  Not under a moving camera, whose frames are bound by the
    // caller's stream (chunk 0's composite, then chunk 1): orbit 2528 -> 2416 with it.
    // GS_FUSE_SORT=0 keeps the separate sort (A/B runs).
    static const uint32_t fuse_sort = env_u32("GS_FUSE_SORT", 1u);
    // (nor for frames of at most kDeepTiles tiles: 1080p G = 8 strips 0.088-0.090 -> 0.090-0.094 ms with it)
    const bool sort_in_composite = fuse_sort && !moving && n_tiles > kDeepTiles && composite_sorts(tsp, cp);
    if (!sort_in_composite) launch_tile_sort(tsp, st);
    mark(EV_TSORT_0);
    HIPCHK(hipEventRecord(F.ev_early, st));
    HIPCHK(hipStreamWaitEvent(cst, F.ev_early, 0));
    st = cst;  // the composite (the caller's buffer) and the frame's end, in call order
    mark(EV_RANGES_0);
    if (fr.pad > 0) {  // the last equal strip's rows past the image are padding (gs_strip_rows):
        // defined as zero (transparent black); no kernel writes them
        const size_t px = cp.out_f16 ? 8 : 16;
        HIPCHK(hipMemsetAsync((char*)out + (size_t)(fr.rows - fr.pad) * (size_t)W * px, 0,
                              (size_t)fr.pad * (size_t)W * px, st));
    }
    launch_composite(cp, o.accum == GS_ACCUM_FP16_TARGET, st, sort_in_composite ? &tsp : nullptr);
    mark(EV_COMP_0);
    {  // chunk 1 (when chunk 0 left tiles unsaturated), then the frame's end: statistics into the
       // slot, FrameCtl zeroed for the next frame; one launch
        Chunk1Params c1{};
        c1.pp = pp;
        c1.pp.plist = F.plist;
        c1.pp.rec_all = 0;
        c1.bp = bp;
        c1.bp.cnt = F.c1;
        c1.bp.units = nullptr;  // chunk 1: every unit
        c1.bp.cut_units = cut_on ? F.units : nullptr;  // ... and chunk 0's again for the entries the cut left out
        c1.bp.chunk = 1;
        c1.bp.nparts = fit_nparts(c1.bp.parts, env_nparts("GS_NPARTS_C1", kBinPartsSmall));
        c1.bp.order = nullptr;
        c1.tp = tsp;
        c1.tp.done = F.done;
        c1.tp.c1tiles = cp.c1tiles;
        c1.tp.c1_n = &F.ctl->not_done;
        c1.cp = cp;
        c1.cp.mode = kCompSecond;
        c1.cp.order = nullptr;
        c1.cp.seg = split ? 4 : 1;  // chunk 1: a few tiles with long lists (launch_chunk1_split)
        c1.bar = F.bar;
        c1.spin_ticks = c->spin_ticks;
        c1.cus = c->num_cus;
        c1.two_chunks = two_chunks ? 1 : 0;
        const uint32_t q = s->seq_next++;
        s->stat_want[slot] = q;
        c1.stats = F.stats;
        c1.host_ctl = s->d_ctl_slot + slot;
        c1.host_seq = s->d_seq + slot;
        c1.seq = q;
        // While chunk 0 saturates every tile: k_chunk1 on 64 workgroups (the launch then only ends
        // the frame; it is LDS-heavy and starts beside the next frame's kernels).  Its grid fits the
        // device at once (one 256-thread workgroup per CU), so every workgroup becomes resident
        // while the others wait at a grid barrier: the kernels beside it never wait for k_chunk1
        // and finish.  Once a recent frame left tiles unsaturated: chunk 1 as separate launches
        // at full occupancy (a kernel boundary costs less than a grid barrier), then the frame's end.
        // (a moving camera takes the launches too: its first frame that leaves tiles unsaturated
        // after saturated ones ran chunk 1 on k_chunk1's 64 workgroups, 5.4 ms at 4K)
        if (two_chunks && (seeded || moving || (s->have_last && s->last.not_done > 0)))
            launch_chunk1_split(c1, o.accum == GS_ACCUM_FP16_TARGET, st);
        else
            launch_chunk1(c1, c->c1_grid, o.accum == GS_ACCUM_FP16_TARGET, st);
        if (two_chunks && o.timing == 1) mark(EV_COMP_1);
    }
    F.meta_clean = true;
    mark(EV_END);
    HIPCHK(hipEventRecord(F.ev_out, st));
    s->last_fs = s->cur_fs;
    s->cur_fs = (s->cur_fs + 1) % kFrameSets;
    s->last_pp = pp;
    HIPCHK(hipGetLastError());
    if (timed) {
        fe.pending = true;
        c->fe_cur = (c->fe_cur + 1) % kStatSlots;
    }
    s->stat_pending[slot] = true;  // frame statistics arrive asynchronously (k_chunk1)
    s->stat_cur = (s->stat_cur + 1) % kStatSlots;
    s->have_frame = true;
    c->last_scene = s;
    c->stats.n = s->n;
    c->stats.tile_row_begin = tr_begin;
    c->stats.tile_row_end = tr_end;
    c->stats.tiles_x = TX;
}

static void validate_render_args(gs_ctx* c, gs_scene* s, const void* uni, int W, int H,
                                 const gs_opts* o) {
    if (!c || !s || !uni) throw GsError(GS_ERR_INVALID, "null ctx/scene/uniforms");
    if (s->ctx != c) throw GsError(GS_ERR_INVALID, "scene belongs to another context");
    if (!c->members.empty() && o && o->strip_count != 1)
        throw GsError(GS_ERR_INVALID, "a device group renders its row strips itself (strip_count must be 1)");
    if (W <= 0 || H <= 0 || W > 65535 || H > 65535) throw GsError(GS_ERR_INVALID, "bad image size");
    if (o) {
        const gs_opts oo = read_opts(o);
        if (oo.strip_count < 1 || oo.strip_index < 0 || oo.strip_index >= oo.strip_count)
            throw GsError(GS_ERR_INVALID, "bad strip index/count");
        if (oo.tile_row_end != 0 || oo.tile_row_begin != 0) {
            const int TR = (H + kTile - 1) / kTile;
            if (oo.strip_count != 1) throw GsError(GS_ERR_INVALID, "an explicit tile-row range takes strip_count 1");
            if (!c->members.empty())
                throw GsError(GS_ERR_INVALID, "a device group chooses its strips itself (no explicit tile-row range)");
            if (oo.tile_row_begin < 0 || oo.tile_row_end <= oo.tile_row_begin || oo.tile_row_end > TR)
                throw GsError(GS_ERR_INVALID, "bad tile-row range");
        }
        if (o->accum != GS_ACCUM_FP32 && o->accum != GS_ACCUM_FP16_TARGET)
            throw GsError(GS_ERR_INVALID, "bad accum mode");
        if (o->out_format != GS_OUT_RGBA_F32 && o->out_format != GS_OUT_RGBA_F16)
            throw GsError(GS_ERR_INVALID, "bad out_format");
        if (!(o->t_min >= 0.0f && o->t_min < 1.0f)) throw GsError(GS_ERR_INVALID, "t_min must be in [0,1)");
        if (o->timing < 0 || o->timing > 2) throw GsError(GS_ERR_INVALID, "timing must be 0, 1 or 2");
        if (!(o->chunk_fraction >= 0.0f)) throw GsError(GS_ERR_INVALID, "chunk_fraction must be >= 0");
        if (o->ref_quirks && s->n > kQuirkMaxN)
            throw GsError(GS_ERR_UNSUPPORTED, "ref_quirks: the reference's init-sort dispatch is invalid above 524280 "
                                              "Gaussians (max(N/8,8) > 65535 workgroups)");
    }
}

static size_t out_bytes_for(int W, int H, const gs_opts& o) {
    return (size_t)frame_rows(H, o).rows * (size_t)W * (o.out_format == GS_OUT_RGBA_F16 ? 8 : 16);
}

// After a tile-list overflow: every frame set grows to the largest total of the frames that
// overflowed (a later, smaller frame's total would grow them too little).
static void grow_after_overflow(gs_scene* s) {
    const uint64_t k = std::max<uint64_t>(s->overflow_k, s->last.k_total);
    for (FrameSet& F : s->fs) ensure_tile_capacity(F, k);
    s->overflow_k = 0;
}

// Frame errors surface here: every frame's FrameCtl comes back asynchronously, so an error of a
// frame rendered with gs_render_device is reported by a later call (gsplat.h).  The error bits of
// every harvested frame accumulate in pending_err until reported.
static void check_frame_errors(gs_scene* s) {
    HIPCHK(hipSetDevice(s->ctx->device));  // a device group's member: its own device
    collect_stats(s, true);
    const uint32_t e = s->pending_err;
    s->pending_err = 0;
    if (e & kErrBarrier) {  // a timed-out barrier leaves its arrival count behind: zero every set's
        HIPCHK(hipDeviceSynchronize());
        for (FrameSet& F : s->fs) HIPCHK(hipMemset(F.bar, 0, 16));
        throw GsError(GS_ERR_DEVICE_FAULT, "chunk-1 grid barrier timed out (workgroups not co-resident)");
    }
    if (e & kErrState) {  // frame state the frame did not write: every set starts clean again
        for (FrameSet& F : s->fs) F.meta_clean = false;
        throw GsError(GS_ERR_DEVICE_FAULT, "frame state out of range (a unit, partition or wide-splat count past its list)");
    }
    if (e & kErrBinning)  // a wrong tile list (count and emission disagreed): never a valid image
        throw GsError(GS_ERR_DEVICE_FAULT, "binning invariant violated: a tile's emitted entries differ from its count");
    if (e & kErrOverflow) {
        grow_after_overflow(s);
        throw GsError(GS_ERR_DEVICE_FAULT, "tile-entry capacity exceeded; capacity grown, render again");
    }
}

// Stable LSD radix sort of (key, value) pairs on bits [b0, b1) on the device: (ka, va) in, ping-pong
// with (kb, vb); returns the buffers holding the result.
static std::pair<uint32_t*, uint32_t*> device_sort_pairs(uint32_t* ka, uint32_t* va, uint32_t* kb, uint32_t* vb,
                                                         uint64_t n, int b0, int b1, hipStream_t st) {
    if (n == 0) return {ka, va};
    const int npass = (b1 - b0 + 7) / 8;
    uint32_t *hist = nullptr, *offs = nullptr, *gsum = nullptr;
    const size_t region = 256 * ((sort_parts(n, kDepthSortIpt) + kGroupParts - 1) / kGroupParts + 1);
    try {
        dev_alloc(hist, (size_t)npass * kHistWords);
        dev_alloc(offs, (size_t)256 * sort_parts(n, kDepthSortIpt));
        dev_alloc(gsum, (size_t)npass * region);
        HIPCHK(hipMemsetAsync(hist, 0, (size_t)npass * kHistWords * 4, st));
        HIPCHK(hipMemsetAsync(gsum, 0, (size_t)npass * region * 4, st));
        for (int ps = 0; ps < npass; ++ps) {
            SortPass sp{};
            sp.keys_in = ka; sp.vals_in = va; sp.keys_out = kb; sp.vals_out = vb;
            sp.n = (uint32_t)n;
            sp.ipt = kDepthSortIpt;
            sp.parts_max = sort_parts(n, sp.ipt);
            sp.shift = b0 + 8 * ps;
            const int bits = std::min(8, b1 - sp.shift);
            sp.mask = (1u << bits) - 1u;
            sp.hist = hist + ps * kHistWords;
            sp.offsets = offs;
            sp.gsum = gsum + (size_t)ps * region;
            launch_sort_pass(sp, st);
            std::swap(ka, kb);
            std::swap(va, vb);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(st));
    } catch (...) {
        dev_free(hist); dev_free(offs); dev_free(gsum);
        throw;
    }
    dev_free(hist); dev_free(offs); dev_free(gsum);
    return {ka, va};
}

// Slots the reference's init-sort pass keys: trunc(max(N/8, 8)) * 8 (WebIDL [EnforceRange]
// truncation of dispatchWorkgroups' argument; the shader skips idx >= N).
static uint64_t quirk_keyed_slots(uint64_t n) {
    const uint64_t keyed = (uint64_t)std::trunc(std::max((double)n / 8.0, 8.0)) * 8;
    return std::min(keyed, n);
}

// ref_quirks: this frame's N init-sort slots -> stable sort -> the draw-ordered copy of the scene
// (and the next frame's state).  Runs on `st` ahead of the frame's culling; waits for every frame
// in flight first (they read the copy).
static void quirk_prepare(gs_scene* s, const float* uni, hipStream_t st) {
    const uint32_t n = (uint32_t)s->n;
    HIPCHK(hipDeviceSynchronize());
    if (!s->qk) {
        const size_t m = std::max<size_t>(n, 1);
        dev_alloc(s->qk, m); dev_alloc(s->qv, m);
        dev_alloc(s->qK, m); dev_alloc(s->qV, m); dev_alloc(s->qK2, m); dev_alloc(s->qV2, m);
        dev_alloc(s->qinv, m);
        dev_alloc(s->qgeo, 3 * m);
        dev_alloc(s->qshade, (size_t)sh_quads(s->n_sh) * m);
        dev_alloc(s->qcull, m);
        dev_alloc(s->qorig, m);
        dev_alloc(s->qbounds, (size_t)proj_parts(n) + 1);
        HIPCHK(hipMemsetAsync(s->qk, 0, m * 4, st));  // WebGPU buffers start zeroed
        HIPCHK(hipMemsetAsync(s->qv, 0, m * 4, st));
        launch_inverse(s->orig, n, s->qinv, st);
    }
    if (!n) return;
    const uint32_t nk = (uint32_t)quirk_keyed_slots(n);
    const float4 vrow = make_float4(uni[2], uni[6], uni[10], uni[14]);  // view row 2 (column-major)
    launch_quirk_keys(s->cull, s->orig, n, nk, vrow, s->qk, s->qv, s->qK, s->qV, st);
    const auto r = device_sort_pairs(s->qK, s->qV, s->qK2, s->qV2, n, 0, 32, st);
    launch_quirk_gather(r.first, r.second, s->qinv, n, nk, sh_quads(s->n_sh), s->geo, s->shade, s->cull, s->qgeo,
                        s->qshade, s->qcull, s->qorig, s->qk, s->qv, st);
    launch_part_bounds(s->qcull, n, s->qbounds, st);
    HIPCHK(hipGetLastError());
    s->qdraw = r.second;
}

// Group strips are K-balanced (render_group): every kRebalanceFrames frames the boundaries move.
constexpr uint32_t kRebalanceFrames = 8;
constexpr double kTileCost = 32.0;  // a tile's fixed cost in binned-entry units (its scan, sort and composite start)

static void rebalance_group(gs_ctx* c, gs_scene* s, int W, int TR) {
    const int G = (int)c->members.size();
    const int TX = (W + kTile - 1) / kTile;
    std::vector<double> cost(G, 0.0);
    for (int g = 0; g < G; ++g) {
        gs_scene* m = s->members[g];
        if (!m->have_last) return;  // no statistics yet
        const int rows = c->gbounds[g + 1] - c->gbounds[g];
        cost[g] = (double)m->last.k_chunk[0] + (double)m->last.k_chunk[1] + kTileCost * TX * rows;
    }
    std::vector<int> nb(G + 1);
    balance_bounds(G, TR, c->gbounds.data(), cost.data(), nb.data());
    // a member whose strip grows may bin more entries than its tile lists hold: grow them ahead
    // (each old strip's entries spread evenly over its rows; 1.5x headroom), instead of letting the
    // first frame on the new strips overflow and fail
    for (int g = 0; g < G; ++g) {
        double est = 0.0;
        for (int j = 0; j < G; ++j) {
            const int r0 = std::max(nb[g], c->gbounds[j]), r1 = std::min(nb[g + 1], c->gbounds[j + 1]);
            const int rows = c->gbounds[j + 1] - c->gbounds[j];
            if (r1 > r0 && rows > 0) est += (double)s->members[j]->last.k_total * (r1 - r0) / rows;
        }
        gs_scene* m = s->members[g];
        const uint64_t want = (uint64_t)(1.5 * est);
        bool grow = false;
        for (const FrameSet& F : m->fs) grow = grow || want > F.kcap;
        if (!grow) continue;
        HIPCHK(hipSetDevice(c->members[g]->device));
        for (FrameSet& F : m->fs) ensure_tile_capacity(F, want);  // (hipFree waits for the frames using them)
    }
    c->gbounds = nb;
}

// ---- the group's enqueue threads
static void worker_loop(GroupWorker* w, int device) {
    (void)hipSetDevice(device);
    uint32_t seen = 0;
    for (;;) {
        uint32_t p = w->posted.load(std::memory_order_acquire);
        if (p == seen) {  // spin a while (pause, then yield), then sleep until the next post
            const int64_t t0 = now_ns();
            const int64_t window = std::min<int64_t>(GroupWorker::kSpinNs, 2 * w->gap_ns.load(std::memory_order_relaxed));
            while ((p = w->posted.load(std::memory_order_acquire)) == seen) {
                const int64_t dt = now_ns() - t0;
                if (dt > window) break;
                if (dt < GroupWorker::kPauseNs)
                    __builtin_ia32_pause();
                else
                    std::this_thread::yield();
            }
            if (p == seen) {
                std::unique_lock<std::mutex> lk(w->mu);
                w->sleeping.store(true);  // (seq_cst, paired with post_job's load: no lost wake-up)
                w->cv.wait(lk, [&] { return w->quit.load() || w->posted.load() != seen; });
                w->sleeping.store(false);
                p = w->posted.load(std::memory_order_acquire);
            }
        }
        if (w->quit.load()) return;
        seen = p;
        w->rc = GS_OK;
        w->msg.clear();
        w->t_start = now_ns();
        try {
            w->fn(w->arg, w->member);
        } catch (const GsError& e) {
            w->rc = e.code;
            w->msg = e.what();
        } catch (const std::bad_alloc&) {
            w->rc = GS_ERR_OOM;
            w->msg = "host allocation failed";
        } catch (const std::exception& e) {
            w->rc = GS_ERR_INTERNAL;
            w->msg = e.what();
        } catch (...) {
            w->rc = GS_ERR_INTERNAL;
            w->msg = "unknown exception";
        }
        w->t_end = now_ns();
        w->finished.store(p, std::memory_order_release);
    }
}

static void post_job(GroupWorker* w, void (*fn)(void*, int), void* arg, int member) {
    const int64_t t = now_ns();
    if (w->t_post_last) {  // running mean of the time between posts (the worker's spin window)
        const int64_t g = std::min<int64_t>(t - w->t_post_last, GroupWorker::kSpinNs);
        w->gap_ns.store((w->gap_ns.load(std::memory_order_relaxed) * 7 + g) / 8, std::memory_order_relaxed);
    }
    w->t_post_last = t;
    w->fn = fn;
    w->arg = arg;
    w->member = member;
    w->posted.fetch_add(1);  // seq_cst: ordered against the worker's `sleeping` store
    if (w->sleeping.load()) {
        { std::lock_guard<std::mutex> lk(w->mu); }  // the worker is inside cv.wait (or has left it)
        w->cv.notify_one();
    }
}

// Wait for the worker's last posted job; its error, if any, as (code, message).
static void join_job(GroupWorker* w, int& rc, std::string& msg) {
    const uint32_t want = w->posted.load();
    const int64_t t0 = now_ns();
    while (w->finished.load(std::memory_order_acquire) != want) {
        if (now_ns() - t0 < GroupWorker::kPauseNs)
            __builtin_ia32_pause();
        else
            std::this_thread::yield();
    }
    if (w->rc != GS_OK && rc == GS_OK) {
        rc = w->rc;
        msg = w->msg;
    }
}

static void start_workers(gs_ctx* c) {
    c->workers.resize(c->members.size());
    for (size_t g = 1; g < c->members.size(); ++g) {
        c->workers[g].reset(new GroupWorker());
        GroupWorker* w = c->workers[g].get();
        c->workers[g]->th = std::thread(worker_loop, w, c->members[g]->device);
    }
}

static void stop_workers(gs_ctx* c) {
    for (auto& w : c->workers) {
        if (!w) continue;
        {
            std::lock_guard<std::mutex> lk(w->mu);
            w->quit.store(true);
            w->posted.fetch_add(1);  // a spinning worker sees a post, then quit
        }
        w->cv.notify_one();
        if (w->th.joinable()) w->th.join();
    }
    c->workers.clear();
}

// One group frame as the members see it (on the caller's stack while render_group runs).
struct GroupFrame {
    gs_ctx* c;
    gs_scene* s;
    const float* uni;
    int W, H;
    gs_opts o;
    void* out;
    hipStream_t st0;
    size_t row_bytes;
    int buf;
    std::atomic<bool> m0_enqueued{false};  // member 0's frame is on st0: the members' strips may be waited for there
};

// How member g's strip reaches the image on device 0.
enum GroupPath {
    kGroupDirect = 0,  // member 0, or a member on device 0: it renders straight into its rows of the image
    kGroupRccl = 1,    // distinct devices: an RCCL send of the strip buffer to member 0
    kGroupPeer = 2     // another device without RCCL (a list that repeats devices), or forced: a peer copy
};
static int group_path(const gs_ctx* c, int g) {
    if (g == 0) return kGroupDirect;
    if (!c->comms.empty()) return kGroupRccl;
    return c->members[g]->device == c->members[0]->device && !c->group_peer_copy ? kGroupDirect : kGroupPeer;
}

// Member g's two strip buffers on its device, at least `need` bytes each (any strip fits: the
// bounds move).
static void ensure_group_buffers(gs_ctx* c, int g, size_t need) {
    if (c->gbuf_bytes[g] >= need) return;
    gs_ctx* m = c->members[g];
    HIPCHK(hipSetDevice(m->device));
    HIPCHK(hipDeviceSynchronize());
    for (void*& p : c->gbuf[g]) {
        if (p) HIPCHK(hipFree(p));
        p = nullptr;
    }
    c->gbuf_bytes[g] = 0;
    for (void*& p : c->gbuf[g]) HIPCHK(hipMalloc(&p, need));
    c->gbuf_bytes[g] = need;
}

// Member g's part of a group frame, enqueued from its own thread: render its strip -- into its
// rows of the image (direct), or into its strip buffer `buf` -- and start the strip's way to
// device 0: an RCCL send or a peer copy on its gather stream, each recording gev_sent[g][buf]
// ("the strip is in the image / the buffer is free again").
static void group_member(void* arg, int g) {
    const GroupFrame& f = *(const GroupFrame*)arg;
    gs_ctx* c = f.c;
    const int tb = c->gbounds[g], te = c->gbounds[g + 1];
    if (tb >= te) return;
    gs_ctx* m = c->members[g];
    HIPCHK(hipSetDevice(m->device));
    gs_opts og = f.o;
    og.strip_index = 0;
    og.strip_count = 1;
    og.tile_row_begin = tb;
    og.tile_row_end = te;
    char* img = (char*)f.out + (size_t)tb * kTile * f.row_bytes;
    const int path = group_path(c, g);
    if (g == 0) {
        render_frame(m, f.s->members[0], f.uni, f.W, f.H, og, img, f.st0);
        return;
    }
    // st0 (the caller's stream) waits for this strip behind member 0's frame (so that member 0's
    // kernels do not wait for it); from this thread, so the caller does not issue G - 1 waits
    auto st0_waits = [&](hipEvent_t e) {
        while (!f.m0_enqueued.load(std::memory_order_acquire)) __builtin_ia32_pause();
        HIPCHK(hipSetDevice(c->members[0]->device));
        HIPCHK(hipStreamWaitEvent(f.st0, e, 0));
    };
    if (path == kGroupDirect) {  // device 0's rows, after the caller's earlier work on the image
        HIPCHK(hipStreamWaitEvent(m->stream, c->gev_entry, 0));
        render_frame(m, f.s->members[g], f.uni, f.W, f.H, og, img, m->stream);
        HIPCHK(hipEventRecord(c->gev_sent[g][f.buf], m->stream));
        st0_waits(c->gev_sent[g][f.buf]);
        return;
    }
    if (path == kGroupPeer) ensure_group_buffers(c, g, (size_t)f.H * f.row_bytes);  // (RCCL: by the caller)
    void* dst = c->gbuf[g][f.buf];
    const size_t bytes = (size_t)(std::min(te * kTile, f.H) - tb * kTile) * f.row_bytes;
    if (path == kGroupRccl) {
        // Member 0's receive of this strip is already queued (render_group): it must get its send
        // whatever happens here, or device 0's gather stream waits forever / pairs the next
        // frame's send with this frame's receive.  On a failed render the (stale)
        // strip buffer is still sent, then the error goes to the caller.
        std::string err;
        int code = GS_OK;
        try {
            HIPCHK(hipStreamWaitEvent(m->stream, c->gev_sent[g][f.buf], 0));  // frame f - 2's transfer of it
            render_frame(m, f.s->members[g], f.uni, f.W, f.H, og, dst, m->stream);
        } catch (const GsError& e) {
            code = e.code;
            err = e.what();
        }
        (void)hipEventRecord(c->gev_rendered[g], m->stream);
        (void)hipStreamWaitEvent(c->gstream[g], c->gev_rendered[g], 0);
        const ncclResult_t r = ncclSend(dst, bytes, ncclUint8, 0, c->comms[g], c->gstream[g]);
        HIPCHK(hipEventRecord(c->gev_sent[g][f.buf], c->gstream[g]));
        if (code != GS_OK) throw GsError(code, err);
        if (r != ncclSuccess) throw GsError(GS_ERR_HIP, std::string("ncclSend: ") + ncclGetErrorString(r));
        return;
    }
    HIPCHK(hipStreamWaitEvent(m->stream, c->gev_sent[g][f.buf], 0));  // frame f - 2's transfer of it
    render_frame(m, f.s->members[g], f.uni, f.W, f.H, og, dst, m->stream);
    HIPCHK(hipEventRecord(c->gev_rendered[g], m->stream));
    HIPCHK(hipStreamWaitEvent(c->gstream[g], c->gev_rendered[g], 0));
    {  // peer copy into the image, after the caller's earlier work on it (gev_entry)
        HIPCHK(hipStreamWaitEvent(c->gstream[g], c->gev_entry, 0));
        HIPCHK(hipMemcpyPeerAsync(img, c->members[0]->device, dst, m->device, bytes, c->gstream[g]));
    }
    HIPCHK(hipEventRecord(c->gev_sent[g][f.buf], c->gstream[g]));
    if (path == kGroupPeer) st0_waits(c->gev_sent[g][f.buf]);  // (RCCL: st0 waits for member 0's receives)
}

// A device group's frame (gs_ctx::members): member g renders tile rows [gbounds[g], gbounds[g+1])
// of the image, every member at once -- member 0 on the caller's thread, member g >= 1 from its own
// enqueue thread (GroupWorker).  Member 0, and members on device 0, render straight into their rows
// of `out`; a member on another device renders into one of two strip buffers there
// (double-buffered: its next frame renders into the other while this one travels) and sends it to
// device 0 on its gather stream -- RCCL send/receive pairs over the communicators of
// ncclCommInitAll (distinct devices, xGMI; the caller queues member 0's receives while the members
// render), or a peer copy (a list that repeats devices).  The strips are K-balanced: every
// kRebalanceFrames frames the boundaries move so that each member's binned entries (plus a
// per-tile cost) are equal (balance_bounds).  Enqueue only: the image is complete on device 0 in
// stream order of st0.
static void render_group(gs_ctx* c, gs_scene* s, const float* uni, int W, int H, const gs_opts& o, void* out,
                         hipStream_t st0) {
    const int G = (int)c->members.size();
    const int TR = (H + kTile - 1) / kTile;
    if (c->gH != H || (int)c->gbounds.size() != G + 1) {  // even strips until statistics arrive
        c->gbounds.assign(G + 1, 0);
        for (int g = 0; g <= G; ++g) c->gbounds[g] = (int)((int64_t)g * TR / G);
        c->gH = H;
        c->gframe = 0;
    } else if (++c->gframe % kRebalanceFrames == 0) {
        rebalance_group(c, s, W, TR);
    }
    if (c->workers.size() != (size_t)G) start_workers(c);
    GroupFrame f{c, s, uni, W, H, o, out, st0, (size_t)W * (o.out_format == GS_OUT_RGBA_F16 ? 8 : 16),
                 (int)(c->gframe & 1u), {false}};
    const int dev0 = c->members[0]->device;
    const bool rccl = !c->comms.empty();
    // the strips land in `out` after the caller's earlier work on it
    HIPCHK(hipSetDevice(dev0));
    HIPCHK(hipEventRecord(c->gev_entry, st0));
    static const bool serial_env = [] {  // GS_GROUP_SERIAL=1: every member from the caller's thread (A/B)
        const char* e = std::getenv("GS_GROUP_SERIAL");
        return e && e[0] == '1';
    }();
    // (not with RCCL: member 0's receives are queued before the sends, and one thread issuing both
    // could block in the first connection setup -- ADVICE r04)
    const bool serial = serial_env && !rccl;
    if (rccl) {  // every strip buffer exists before any receive is queued (each receive gets its send)
        for (int g = 1; g < G; ++g) ensure_group_buffers(c, g, (size_t)H * f.row_bytes);
        HIPCHK(hipSetDevice(dev0));
    }
    static const int trace = [] {  // GS_GROUP_TRACE=1: per-member enqueue times to stderr every 200 frames; 2: every frame
        const char* e = std::getenv("GS_GROUP_TRACE");
        return e ? std::atoi(e) : 0;
    }();
    const int64_t t_post = trace ? now_ns() : 0;
    if (!serial)
        for (int g = 1; g < G; ++g) post_job(c->workers[g].get(), group_member, &f, g);
    int rc = GS_OK;
    std::string msg;
    try {
        if (rccl) {  // member 0's receives, queued while the members render (ordered per peer by frame)
            HIPCHK(hipStreamWaitEvent(c->gstream[0], c->gev_entry, 0));
            ncclResult_t r = ncclGroupStart();
            for (int g = 1; g < G && r == ncclSuccess; ++g) {
                const int tb = c->gbounds[g], te = c->gbounds[g + 1];
                if (tb >= te) continue;
                const size_t bytes = (size_t)(std::min(te * kTile, H) - tb * kTile) * f.row_bytes;
                r = ncclRecv((char*)out + (size_t)tb * kTile * f.row_bytes, bytes, ncclUint8, g, c->comms[0], c->gstream[0]);
            }
            const ncclResult_t r2 = ncclGroupEnd();
            if (r != ncclSuccess || r2 != ncclSuccess)
                throw GsError(GS_ERR_HIP, std::string("ncclRecv: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
            HIPCHK(hipEventRecord(c->gev_gathered, c->gstream[0]));
        }
        group_member(&f, 0);
        f.m0_enqueued.store(true, std::memory_order_release);
        if (serial)
            for (int g = 1; g < G; ++g) group_member(&f, g);
    } catch (const GsError& e) {
        rc = e.code;
        msg = e.what();
    } catch (const std::exception& e) {
        rc = GS_ERR_INTERNAL;
        msg = e.what();
    } catch (...) {
        rc = GS_ERR_INTERNAL;
        msg = "unknown exception";
    }
    f.m0_enqueued.store(true, std::memory_order_release);  // (also after an error: the members finish)
    const int64_t t_m0 = trace ? now_ns() : 0;
    if (!serial)
        for (int g = 1; g < G; ++g) join_job(c->workers[g].get(), rc, msg);  // (every job ends before f does)
    HIPCHK(hipSetDevice(dev0));
    if (rc != GS_OK) throw GsError(rc, msg);
    if (rccl) HIPCHK(hipStreamWaitEvent(st0, c->gev_gathered, 0));
    if (trace && !serial) {
        static std::vector<double> acc;
        static int frames = 0;
        acc.resize(3 * G + 1, 0.0);
        acc[0] += (t_m0 - t_post) * 1e-3;
        for (int g = 1; g < G; ++g) {
            acc[3 * g] += (c->workers[g]->t_start - t_post) * 1e-3;
            acc[3 * g + 1] += (c->workers[g]->t_end - c->workers[g]->t_start) * 1e-3;
        }
        acc[3 * G] += (now_ns() - t_post) * 1e-3;
        if (++frames == (trace == 2 ? 1 : 200)) {
            std::fprintf(stderr, "group trace (mean us over %d frames): member 0 %.1f; call %.1f;", frames, acc[0] / frames,
                         acc[3 * G] / frames);
            for (int g = 1; g < G; ++g) std::fprintf(stderr, " m%d start +%.1f run %.1f;", g, acc[3 * g] / frames, acc[3 * g + 1] / frames);
            std::fprintf(stderr, "\n");
            std::fill(acc.begin(), acc.end(), 0.0);
            frames = 0;
        }
    }
    c->last_scene = s;
}

extern "C" {

int gs_abi_version(void) { return GS_ABI_VERSION; }
const char* gs_last_error(void) { return g_last_error.c_str(); }

int gs_device_count(int* out) {
    return guarded([&] {
        if (!out) throw GsError(GS_ERR_INVALID, "null out");
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        *out = n;
        return GS_OK;
    });
}

void gs_opts_default(gs_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->struct_size = sizeof(gs_opts);
    o->accum = GS_ACCUM_FP32;
    o->out_format = GS_OUT_RGBA_F32;
    o->t_min = 1e-4f;
    o->strip_index = 0;
    o->strip_count = 1;
    o->chunk_fraction = 0.0f;
}

static gs_ctx* create_single(int dev);

int gs_ctx_create(const int* devices, int ndev, gs_ctx** out) {
    return guarded([&] {
        if (!out) throw GsError(GS_ERR_INVALID, "null out");
        *out = nullptr;
        if (ndev < 0 || ndev > kMaxGroup || (ndev > 0 && !devices) || (ndev == 0 && devices))
            throw GsError(GS_ERR_INVALID, "bad device list");
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
            throw GsError(GS_ERR_NO_DEVICE, "no HIP device available");
        for (int g = 0; g < std::max(ndev, 1); ++g) {
            const int dev = devices ? devices[g] : 0;
            if (dev < 0 || dev >= count) throw GsError(GS_ERR_INVALID, "device index out of range");
        }
        if (ndev <= 1) {
            *out = create_single(devices ? devices[0] : 0);
            return GS_OK;
        }
        gs_ctx* c = new gs_ctx();
        c->device = devices[0];
        try {
            for (int g = 0; g < ndev; ++g) c->members.push_back(create_single(devices[g]));
            std::vector<int> d(devices, devices + ndev);
            std::sort(d.begin(), d.end());
            if (std::adjacent_find(d.begin(), d.end()) == d.end()) {  // distinct devices: RCCL
                c->comms.assign(ndev, nullptr);
                const ncclResult_t r = ncclCommInitAll(c->comms.data(), ndev, devices);
                if (r != ncclSuccess) {
                    c->comms.clear();
                    throw GsError(GS_ERR_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
                }
            }
            {
                const char* e = std::getenv("GS_GROUP_PEER_COPY");
                c->group_peer_copy = e && e[0] == '1';
            }
            c->gbuf.assign(ndev, {nullptr, nullptr});
            c->gbuf_bytes.assign(ndev, 0);
            c->gstream.assign(ndev, nullptr);
            c->gev_rendered.assign(ndev, nullptr);
            c->gev_sent.assign(ndev, {nullptr, nullptr});
            const bool rccl = !c->comms.empty();
            for (int g = 0; g < ndev; ++g) {
                HIPCHK(hipSetDevice(devices[g]));
                HIPCHK(hipStreamCreateWithFlags(&c->gstream[g], hipStreamNonBlocking));
                HIPCHK(hipEventCreateWithFlags(&c->gev_rendered[g], hipEventDisableTiming));
                if (g == 0) {
                    const bool one_dev = std::all_of(devices, devices + ndev, [&](int d) { return d == devices[0]; });
                    HIPCHK(hipEventCreateWithFlags(&c->gev_entry, one_dev ? hipEventDisableTiming | hipEventDisableSystemFence
                                                                          : hipEventDisableTiming));
                    HIPCHK(hipEventCreateWithFlags(&c->gev_gathered, hipEventDisableTiming));
                }
            }
            (void)rccl;
            // events that order work on device 0 only need no system-scope fence (its cache
            // write-back would delay the waiting stream); those waited on across devices keep it
            for (int g = 1; g < ndev; ++g)  // recorded where the strip is sent: member g's gather stream
                for (hipEvent_t& e : c->gev_sent[g]) {
                    HIPCHK(hipSetDevice(devices[g]));
                    const unsigned fl = devices[g] == devices[0] ? hipEventDisableTiming | hipEventDisableSystemFence
                                                                 : hipEventDisableTiming;
                    HIPCHK(hipEventCreateWithFlags(&e, fl));
                    HIPCHK(hipEventRecord(e, c->gstream[g]));  // "the buffer is free"
                }
            start_workers(c);
        } catch (...) {
            gs_ctx_destroy(c);
            throw;
        }
        *out = c;
        return GS_OK;
    });
}

static gs_ctx* create_single(int dev) {
    HIPCHK(hipSetDevice(dev));
    gs_ctx* c = new gs_ctx();
    c->device = dev;
    try {
        int cus = 0;
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (cus > 0) c->num_cus = cus;
        // k_chunk1's grid barrier needs every workgroup resident at once: its grid is sized from
        // the occupancy query, and a device that cannot hold it is refused here
        c->c1_occ = chunk1_occupancy();
        c->c1_grid = chunk1_grid(c->c1_occ, c->num_cus);
        if (c->c1_grid <= 0)
            throw GsError(GS_ERR_UNSUPPORTED, "k_chunk1 cannot be resident on this device (occupancy " +
                                                  std::to_string(c->c1_occ) + " per CU)");
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
            c->spin_ticks = (uint64_t)khz * 200u;  // 200 ms
        HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        for (auto& f : c->fe)
            for (auto& e : f.ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    } catch (...) {
        gs_ctx_destroy(c);
        throw;
    }
    return c;
}

void gs_ctx_destroy(gs_ctx* c) {
    if (!c) return;
    if (!c->members.empty()) {
        stop_workers(c);
        while (!c->scenes.empty()) gs_scene_free(c->scenes.back());
        for (size_t g = 0; g < c->members.size(); ++g) {
            (void)hipSetDevice(c->members[g]->device);
            (void)hipDeviceSynchronize();
            if (g < c->gbuf.size())
                for (void* p : c->gbuf[g])
                    if (p) (void)hipFree(p);
        }
        for (size_t g = 0; g < c->members.size(); ++g) {
            (void)hipSetDevice(c->members[g]->device);
            if (g < c->gev_rendered.size() && c->gev_rendered[g]) (void)hipEventDestroy(c->gev_rendered[g]);
            if (g < c->gstream.size() && c->gstream[g]) (void)hipStreamDestroy(c->gstream[g]);
        }
        for (size_t g = 0; g < c->gev_sent.size(); ++g)
            for (hipEvent_t e : c->gev_sent[g])
                if (e) (void)hipEventDestroy(e);
        if (!c->members.empty()) {
            (void)hipSetDevice(c->members[0]->device);
            if (c->gev_entry) (void)hipEventDestroy(c->gev_entry);
            if (c->gev_gathered) (void)hipEventDestroy(c->gev_gathered);
        }
        (void)hipSetDevice(c->members[0]->device);
        for (void* h : c->host_regs) (void)hipHostUnregister(h);
        for (ncclComm_t m : c->comms)
            if (m) (void)ncclCommDestroy(m);
        for (gs_ctx* m : c->members) gs_ctx_destroy(m);
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    while (!c->scenes.empty()) gs_scene_free(c->scenes.back());
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy_stream) {  // readbacks in flight land before their buffers are unpinned
        (void)hipStreamSynchronize(c->copy_stream);
        for (int k = 0; k < gs_ctx::kReadbacks; ++k) {
            if (c->rb_src[k]) (void)hipEventDestroy(c->rb_src[k]);
            if (c->rb_done[k]) (void)hipEventDestroy(c->rb_done[k]);
        }
        (void)hipStreamDestroy(c->copy_stream);
    }
    for (void* h : c->host_regs) (void)hipHostUnregister(h);
    for (auto& f : c->fe)
        for (auto& e : f.ev)
            if (e) (void)hipEventDestroy(e);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int gs_scene_upload(gs_ctx* c, const void* aos, uint64_t n, int n_sh, gs_scene** out) {
    return guarded([&] {
        if (!c || !out || (!aos && n)) throw GsError(GS_ERR_INVALID, "null argument");
        *out = nullptr;
        if (n_sh != 1 && n_sh != 4 && n_sh != 9 && n_sh != 16)
            throw GsError(GS_ERR_UNSUPPORTED, "n_sh_coeffs must be 1, 4, 9 or 16");
        if (n > (1ull << 28)) throw GsError(GS_ERR_UNSUPPORTED, "scene larger than 2^28 Gaussians");
        if (!c->members.empty()) {  // a device group: one replica per member, uploaded concurrently
            const size_t G = c->members.size();
            gs_scene* s = new gs_scene();
            s->ctx = c;
            s->n = n;
            s->n_sh = n_sh;
            s->members.assign(G, nullptr);
            std::vector<int> rc(G, GS_OK);
            std::vector<std::string> msg(G);
            std::vector<std::thread> th;
            for (size_t g = 0; g < G; ++g)
                th.emplace_back([&, g] {
                    rc[g] = gs_scene_upload(c->members[g], aos, n, n_sh, &s->members[g]);
                    if (rc[g] != GS_OK) msg[g] = gs_last_error();
                });
            for (auto& t : th) t.join();
            for (size_t g = 0; g < G; ++g)
                if (rc[g] != GS_OK) {
                    gs_scene_free(s);
                    throw GsError(rc[g], "device " + std::to_string(c->members[g]->device) + ": " + msg[g]);
                }
            c->scenes.push_back(s);
            *out = s;
            return GS_OK;
        }
        HIPCHK(hipSetDevice(c->device));
        gs_scene* s = new gs_scene();
        s->ctx = c;
        s->n = n;
        s->n_sh = n_sh;
        try {
            dev_alloc(s->geo, 3 * (size_t)std::max<uint64_t>(n, 1));
            dev_alloc(s->shade, (size_t)sh_quads(n_sh) * std::max<uint64_t>(n, 1));
            dev_alloc(s->cull, (size_t)std::max<uint64_t>(n, 1));
            dev_alloc(s->bounds, (size_t)proj_parts(n) + 1);
            dev_alloc(s->bbounds, (size_t)((n + kCullBlock - 1) / kCullBlock) + 1);
            dev_alloc(s->orig, (size_t)n + 1);
            for (int k = 0; k < kFrameSets; ++k) {
                FrameSet& F = s->fs[k];
                // (high-priority set streams, like more hardware queues, ran every kernel slower:
                // G = 8 strip 0.09 -> 0.20 ms)
                if (k < kSetStreams) HIPCHK(hipStreamCreateWithFlags(&F.stream, hipStreamNonBlocking));
                else  // sets share streams: set k runs on set k % kSetStreams's stream
                    F.stream = s->fs[k % kSetStreams].stream;
                // the set's events order work on this device only (the host paces on ev_out and
                // reads frame data through its own protocols): no system-scope fence when they
                // are recorded (the default writes back and invalidates the caches; the composite
                // then waited ~17 us on the set stream's per-tile sort, now ~13-15 us)
                HIPCHK(hipEventCreateWithFlags(&F.ev_early, hipEventDisableTiming | hipEventDisableSystemFence));
                HIPCHK(hipEventCreateWithFlags(&F.ev_out, hipEventDisableTiming | hipEventDisableSystemFence));
                HIPCHK(hipEventRecord(F.ev_out, F.stream));  // "the last frame on this set ended"
                dev_alloc(F.r2, (size_t)std::max<uint64_t>(n, 1));
                dev_alloc(F.crec, 3 * ((size_t)proj_parts(n) * kProjTile + 1));
                dev_alloc(F.wlist, (size_t)kWideShards * wide_shard_cap(proj_parts(n)) + 1);
                dev_alloc(F.ctl, 1);
                dev_alloc(F.stats, kStatShards);
                dev_alloc(F.bar, 4);
                HIPCHK(hipMemset(F.bar, 0, 16));
                // slots: part * kProjTile + q < proj_parts(n) * kProjTile
                const size_t nslots = (size_t)proj_parts(n) * kProjTile + 1;
                dev_alloc(F.skey, nslots);
                dev_alloc(F.srect, nslots);
                dev_alloc(F.c0, (size_t)proj_parts(n) + 1);
                dev_alloc(F.c1, (size_t)proj_parts(n) + 1);
                dev_alloc(F.units, (size_t)kUnitShards * unit_shard_cap(proj_parts(n)) + 1);
                dev_alloc(F.plist, (size_t)std::max<uint64_t>(proj_parts(n), (n + kCullBlock - 1) / kCullBlock) + 1);
                dev_alloc(F.plist0, (size_t)proj_parts(n) + 1);
                dev_alloc(F.cand, nslots);
                dev_alloc(F.sidx, nslots);
                ensure_tile_capacity(F, 4 * n + (1u << 20));
            }
            const unsigned hf = hipHostMallocCoherent | hipHostMallocMapped;
            HIPCHK(hipHostMalloc((void**)&s->h_ctl, kStatSlots * sizeof(FrameCtl), hf));
            HIPCHK(hipHostMalloc((void**)&s->h_seq, 64, hf));
            std::memset(s->h_seq, 0, 64);
            HIPCHK(hipHostGetDevicePointer((void**)&s->d_ctl_slot, s->h_ctl, 0));
            HIPCHK(hipHostGetDevicePointer((void**)&s->d_seq, s->h_seq, 0));
            // AoS -> SoA on device in spatial (Morton) order: codes, stable sort, gather-transpose,
            // then the partition bounds
            const uint64_t rb = 64 + 16 * (uint64_t)n_sh;
            if (n) {
                uint8_t* tmp = nullptr;
                uint32_t *bbox = nullptr, *kA = nullptr, *vA = nullptr, *kB = nullptr, *vB = nullptr;
                auto free_tmp = [&] {
                    dev_free(tmp); dev_free(bbox); dev_free(kA); dev_free(vA); dev_free(kB); dev_free(vB);
                };
                try {
                    hipStream_t st = c->stream;
                    dev_alloc(tmp, n * rb);
                    dev_alloc(bbox, 6);
                    dev_alloc(kA, n); dev_alloc(vA, n); dev_alloc(kB, n); dev_alloc(vB, n);
                    HIPCHK(hipMemcpyAsync(tmp, aos, n * rb, hipMemcpyHostToDevice, st));
                    const uint32_t b0[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
                    HIPCHK(hipMemcpyAsync(bbox, b0, sizeof(b0), hipMemcpyHostToDevice, st));
                    launch_bbox(tmp, n, (uint32_t)rb, bbox, st);
                    launch_morton(tmp, n, (uint32_t)rb, bbox, kA, vA, st);
                    const auto r = device_sort_pairs(kA, vA, kB, vB, n, 0, 32, st);
                    launch_transpose(tmp, n, n_sh, r.second, s->geo, s->shade, s->cull, s->orig, st);
                    launch_part_bounds(s->cull, n, s->bounds, st);
                    launch_block_bounds(s->cull, n, s->bbounds, st);
                    HIPCHK(hipGetLastError());
                    HIPCHK(hipStreamSynchronize(st));
                } catch (...) {
                    free_tmp();
                    throw;
                }
                free_tmp();
            }
        } catch (...) {
            gs_scene_free(s);
            throw;
        }
        c->scenes.push_back(s);
        *out = s;
        return GS_OK;
    });
}

void gs_scene_free(gs_scene* s) {
    if (!s) return;
    if (!s->members.empty()) {
        for (gs_scene* m : s->members)
            if (m) gs_scene_free(m);
        if (s->ctx) {
            auto& v = s->ctx->scenes;
            v.erase(std::remove(v.begin(), v.end(), s), v.end());
            if (s->ctx->last_scene == s) s->ctx->last_scene = nullptr;
        }
        delete s;
        return;
    }
    if (s->ctx) {
        (void)hipSetDevice(s->ctx->device);
        (void)hipStreamSynchronize(s->ctx->stream);
        for (FrameSet& F : s->fs)
            if (F.stream) (void)hipStreamSynchronize(F.stream);
        auto& v = s->ctx->scenes;
        v.erase(std::remove(v.begin(), v.end(), s), v.end());
        if (s->ctx->last_scene == s) s->ctx->last_scene = nullptr;
    }
    dev_free(s->geo);
    dev_free(s->shade);
    dev_free(s->dbg);
    dev_free(s->cull);
    for (FrameSet& F : s->fs) {
        if (F.stream) (void)hipStreamSynchronize(F.stream);
        dev_free(F.r2);
        dev_free(F.crec);
        dev_free(F.wlist);
        dev_free(F.ctl);
        dev_free(F.stats);
        dev_free(F.bar);
        dev_free(F.skey);
        dev_free(F.srect);
        dev_free(F.c0);
        dev_free(F.c1);
        dev_free(F.cand);
        dev_free(F.units);
        dev_free(F.plist);
        dev_free(F.plist0);
        dev_free(F.sidx);
        dev_free(F.tvA); dev_free(F.tvB);
        dev_free(F.ranges);
        dev_free(F.bmat);
        dev_free(F.tbase);
        dev_free(F.bchk);
        dev_free(F.cut);
        dev_free(F.cutb);
        dev_free(F.order);
        dev_free(F.done);
        dev_free(F.c1tiles);
        dev_free(F.umask);
        dev_free(F.state);
        dev_free(F.seedh);
        if (F.ev_early) (void)hipEventDestroy(F.ev_early);
        if (F.ev_out) (void)hipEventDestroy(F.ev_out);
    }
    for (int k = 0; k < kSetStreams; ++k)  // (sets past kSetStreams share these)
        if (s->fs[k].stream) (void)hipStreamDestroy(s->fs[k].stream);
    dev_free(s->bounds);
    dev_free(s->bbounds);
    dev_free(s->orig);
    dev_free(s->tile_sat);
    dev_free(s->qk); dev_free(s->qv); dev_free(s->qK); dev_free(s->qV); dev_free(s->qK2); dev_free(s->qV2);
    dev_free(s->qinv); dev_free(s->qgeo); dev_free(s->qshade); dev_free(s->qcull); dev_free(s->qorig);
    dev_free(s->qbounds);
    if (s->h_ctl) (void)hipHostFree(s->h_ctl);
    if (s->h_seq) (void)hipHostFree(s->h_seq);
    delete s;
}

uint64_t gs_scene_count(const gs_scene* s) { return s ? s->n : 0; }

int gs_ctx_info(const gs_ctx* c, int* out_ndev, int* out_gather) {
    return guarded([&] {
        if (!c) throw GsError(GS_ERR_INVALID, "null ctx");
        if (out_ndev) *out_ndev = c->members.empty() ? 1 : (int)c->members.size();
        if (out_gather) *out_gather = c->members.empty() ? GS_GATHER_NONE : !c->comms.empty() ? GS_GATHER_RCCL : GS_GATHER_PEER_COPY;
        return GS_OK;
    });
}

int gs_balance_strips(int G, int tile_rows, const int* bounds, const double* cost, int* out_bounds) {
    return guarded([&] {
        if (G < 1 || G > 4096 || tile_rows < 1 || !bounds || !cost || !out_bounds)
            throw GsError(GS_ERR_INVALID, "bad balance arguments");
        if (bounds[0] != 0 || bounds[G] != tile_rows) throw GsError(GS_ERR_INVALID, "bounds must span [0, tile_rows]");
        for (int g = 0; g < G; ++g)
            if (bounds[g + 1] < bounds[g]) throw GsError(GS_ERR_INVALID, "bounds must not decrease");
        for (int g = 0; g < G; ++g)
            if (!std::isfinite(cost[g])) throw GsError(GS_ERR_INVALID, "non-finite cost");
        std::vector<int> nb(G + 1);
        balance_bounds(G, tile_rows, bounds, cost, nb.data());
        std::copy(nb.begin(), nb.end(), out_bounds);
        return GS_OK;
    });
}

int gs_ctx_strips(const gs_ctx* c, int* out_bounds, int capacity, int* out_n) {
    return guarded([&] {
        if (!c || !out_n) throw GsError(GS_ERR_INVALID, "null argument");
        *out_n = c->members.empty() ? 0 : (int)c->gbounds.size();
        if (out_bounds)
            for (int k = 0; k < *out_n && k < capacity; ++k) out_bounds[k] = c->gbounds[k];
        return GS_OK;
    });
}

int gs_strip_rows(int H, int si, int sc, int* row0, int* rows_padded) {
    return guarded([&] {
        if (H <= 0 || sc < 1 || si < 0 || si >= sc || !row0 || !rows_padded)
            throw GsError(GS_ERR_INVALID, "bad strip arguments");
        int tb, te, rp;
        strip_geometry(H, si, sc, tb, te, rp);
        *row0 = tb * kTile;
        *rows_padded = rp;
        return GS_OK;
    });
}

int gs_render_device(gs_ctx* c, gs_scene* s, const void* uni, int W, int H, const gs_opts* opts,
                     void* out_dev, uint64_t out_bytes, void* stream) {
    return guarded([&] {
        validate_render_args(c, s, uni, W, H, opts);
        const gs_opts o = read_opts(opts);
        if (!out_dev) throw GsError(GS_ERR_INVALID, "null output");
        if (out_bytes < out_bytes_for(W, H, o)) throw GsError(GS_ERR_INVALID, "output buffer too small");
        if (!c->members.empty()) {  // the image (H rows) into out_dev on the first device
            // every member's pending error is handled (capacities grown) before the first is reported
            int rc = GS_OK;
            std::string msg;
            for (gs_scene* m : s->members)
                if (m->pending_err & (kErrOverflow | kErrBarrier | kErrBinning | kErrState)) {
                    const int r = guarded([&] { check_frame_errors(m); return GS_OK; });  // (sets m's device)
                    if (r != GS_OK && rc == GS_OK) {
                        rc = r;
                        msg = gs_last_error();
                    }
                }
            if (rc != GS_OK) throw GsError(rc, msg);
            gs_ctx* m0 = c->members[0];
            HIPCHK(hipSetDevice(m0->device));
            hipStream_t st0 = stream ? (hipStream_t)stream : m0->stream;
            render_group(c, s, (const float*)uni, W, H, o, out_dev, st0);
            return GS_OK;
        }
        HIPCHK(hipSetDevice(c->device));
        if (s->pending_err & (kErrOverflow | kErrBarrier | kErrBinning | kErrState)) check_frame_errors(s);
        hipStream_t st = stream ? (hipStream_t)stream : c->stream;
        render_frame(c, s, (const float*)uni, W, H, o, out_dev, st);
        return GS_OK;
    });
}

int gs_present_device(gs_ctx* c, const void* fb_dev, int fb_format, int W, int H, int out_format,
                      void* out_dev, uint64_t out_bytes, void* stream) {
    return guarded([&] {
        if (!c || !fb_dev || !out_dev) throw GsError(GS_ERR_INVALID, "null argument");
        if (W <= 0 || H <= 0 || W > 65535 || H > 65535) throw GsError(GS_ERR_INVALID, "bad image size");
        if (fb_format != GS_OUT_RGBA_F32 && fb_format != GS_OUT_RGBA_F16)
            throw GsError(GS_ERR_INVALID, "bad framebuffer format");
        uint64_t px_bytes;
        switch (out_format) {
            case GS_PRESENT_RGBA_F32: px_bytes = 16; break;
            case GS_PRESENT_RGBA_F16: px_bytes = 8; break;
            case GS_PRESENT_RGBA8: px_bytes = 4; break;
            default: throw GsError(GS_ERR_INVALID, "bad present format");
        }
        if (out_bytes < px_bytes * (uint64_t)W * (uint64_t)H) throw GsError(GS_ERR_INVALID, "output buffer too small");
        if (fb_dev == out_dev) throw GsError(GS_ERR_INVALID, "present cannot run in place");
        if (!c->members.empty()) c = c->members[0];  // a group's image lives on its first device
        HIPCHK(hipSetDevice(c->device));
        launch_present(fb_dev, fb_format == GS_OUT_RGBA_F16, W, H, out_format, out_dev,
                       stream ? (hipStream_t)stream : c->stream);
        HIPCHK(hipGetLastError());
        return GS_OK;
    });
}

int gs_render(gs_ctx* c, gs_scene* s, const void* uni, int W, int H, const gs_opts* opts, void* out_host) {
    return guarded([&] {
        validate_render_args(c, s, uni, W, H, opts);
        const gs_opts o = read_opts(opts);
        const size_t bytes = out_bytes_for(W, H, o);
        if (!c->members.empty()) {
            HIPCHK(hipSetDevice(c->members[0]->device));
            ensure_out(c->members[0], bytes);
            void* full = c->members[0]->d_out;
            for (int attempt = 0;; ++attempt) {
                render_group(c, s, (const float*)uni, W, H, o, full, c->members[0]->stream);
                bool overflow = false;
                for (size_t g = 0; g < c->members.size(); ++g) {
                    HIPCHK(hipSetDevice(c->members[g]->device));
                    HIPCHK(hipDeviceSynchronize());
                    gs_scene* m = s->members[g];
                    collect_stats(m, true);
                    if (m->pending_err & (kErrBarrier | kErrBinning | kErrState)) check_frame_errors(m);
                    if (m->pending_err & kErrOverflow) {
                        overflow = true;
                        m->pending_err = 0;
                        grow_after_overflow(m);
                    }
                }
                HIPCHK(hipSetDevice(c->members[0]->device));
                if (!overflow) {
                    if (out_host) HIPCHK(hipMemcpy(out_host, full, bytes, hipMemcpyDeviceToHost));
                    return GS_OK;
                }
                if (attempt >= 2) throw GsError(GS_ERR_DEVICE_FAULT, "tile-entry capacity exceeded");
            }
        }
        HIPCHK(hipSetDevice(c->device));
        ensure_out(c, bytes);
        for (int attempt = 0;; ++attempt) {
            render_frame(c, s, (const float*)uni, W, H, o, c->d_out, c->stream);
            HIPCHK(hipStreamSynchronize(c->stream));
            collect_stats(s, true);
            if (s->pending_err & (kErrBarrier | kErrBinning | kErrState)) check_frame_errors(s);
            if (!(s->pending_err & kErrOverflow)) break;
            s->pending_err = 0;
            if (attempt >= 2) throw GsError(GS_ERR_DEVICE_FAULT, "tile-entry capacity exceeded");
            grow_after_overflow(s);  // grow, render again
        }
        if (out_host) HIPCHK(hipMemcpy(out_host, c->d_out, bytes, hipMemcpyDeviceToHost));
        return GS_OK;
    });
}

int gs_framebuffer_alloc(gs_ctx* c, uint64_t bytes, void** out) {
    return guarded([&] {
        if (!c || !out || bytes == 0) throw GsError(GS_ERR_INVALID, "null ctx/out or zero bytes");
        *out = nullptr;
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        HIPCHK(hipSetDevice(d->device));
        if (hipMalloc(out, bytes) != hipSuccess) {
            (void)hipGetLastError();
            *out = nullptr;
            throw GsError(GS_ERR_OOM, "framebuffer allocation failed");
        }
        c->fbufs.emplace_back(*out, bytes);
        return GS_OK;
    });
}

int gs_framebuffer_free(gs_ctx* c, void* dev) {
    return guarded([&] {
        if (!c) throw GsError(GS_ERR_INVALID, "null ctx");
        if (!dev) return GS_OK;
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        HIPCHK(hipSetDevice(d->device));
        HIPCHK(hipDeviceSynchronize());  // no frame in flight may still write it
        HIPCHK(hipFree(dev));
        auto& v = c->fbufs;
        v.erase(std::remove_if(v.begin(), v.end(), [&](const std::pair<void*, uint64_t>& e) { return e.first == dev; }),
                v.end());
        return GS_OK;
    });
}

// `bytes` from `dev` stay inside one of this context's gs_framebuffer_alloc buffers.
static void check_fb_range(const gs_ctx* c, const void* dev, uint64_t bytes) {
    const char* p = (const char*)dev;
    for (const auto& e : c->fbufs) {
        const char* b = (const char*)e.first;
        if (p >= b && p < b + e.second) {
            if (bytes > e.second - (uint64_t)(p - b)) throw GsError(GS_ERR_INVALID, "read past the end of the framebuffer");
            return;
        }
    }
    throw GsError(GS_ERR_INVALID, "not a framebuffer of this context (gs_framebuffer_alloc)");
}

int gs_framebuffer_read(gs_ctx* c, const void* dev, void* host, uint64_t bytes) {
    return guarded([&] {
        if (!c || !dev || !host) throw GsError(GS_ERR_INVALID, "null argument");
        check_fb_range(c, dev, bytes);
        const int rc = gs_sync(c);
        if (rc != GS_OK) throw GsError(rc, gs_last_error());
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        HIPCHK(hipSetDevice(d->device));
        HIPCHK(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
        return GS_OK;
    });
}

int gs_host_register(gs_ctx* c, void* host, uint64_t bytes) {
    return guarded([&] {
        if (!c || !host || bytes == 0) throw GsError(GS_ERR_INVALID, "null ctx/host or zero bytes");
        if (std::find(c->host_regs.begin(), c->host_regs.end(), host) != c->host_regs.end()) return GS_OK;
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        HIPCHK(hipSetDevice(d->device));
        HIPCHK(hipHostRegister(host, bytes, hipHostRegisterDefault));
        c->host_regs.push_back(host);
        return GS_OK;
    });
}

int gs_host_unregister(gs_ctx* c, void* host) {
    return guarded([&] {
        if (!c || !host) throw GsError(GS_ERR_INVALID, "null argument");
        auto it = std::find(c->host_regs.begin(), c->host_regs.end(), host);
        if (it == c->host_regs.end()) throw GsError(GS_ERR_INVALID, "not registered (gs_host_register)");
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        HIPCHK(hipSetDevice(d->device));
        if (d->copy_stream) HIPCHK(hipStreamSynchronize(d->copy_stream));  // no copy still lands in it
        HIPCHK(hipHostUnregister(host));
        c->host_regs.erase(it);
        return GS_OK;
    });
}

int gs_readback_start(gs_ctx* c, const void* dev, void* host, uint64_t bytes, uint32_t* out_ticket) {
    return guarded([&] {
        if (!c || !dev || !host || !out_ticket) throw GsError(GS_ERR_INVALID, "null argument");
        check_fb_range(c, dev, bytes);
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        HIPCHK(hipSetDevice(d->device));
        if (!d->copy_stream) {
            HIPCHK(hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking));
            for (int k = 0; k < gs_ctx::kReadbacks; ++k) {
                HIPCHK(hipEventCreateWithFlags(&d->rb_src[k], hipEventDisableTiming));
                HIPCHK(hipEventCreateWithFlags(&d->rb_done[k], hipEventDisableTiming));
            }
        }
        const uint32_t t = d->rb_next.load();
        const int k = (int)(t % gs_ctx::kReadbacks);
        if (t >= (uint32_t)gs_ctx::kReadbacks) HIPCHK(hipEventSynchronize(d->rb_done[k]));  // ring full: the oldest first
        HIPCHK(hipEventRecord(d->rb_src[k], d->stream));
        HIPCHK(hipStreamWaitEvent(d->copy_stream, d->rb_src[k], 0));
        HIPCHK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, d->copy_stream));
        HIPCHK(hipEventRecord(d->rb_done[k], d->copy_stream));
        d->rb_next.store(t + 1);
        *out_ticket = t;
        return GS_OK;
    });
}

int gs_readback_wait(gs_ctx* c, uint32_t ticket) {
    return guarded([&] {
        if (!c) throw GsError(GS_ERR_INVALID, "null ctx");
        gs_ctx* d = c->members.empty() ? c : c->members[0];
        if (ticket >= d->rb_next.load()) throw GsError(GS_ERR_INVALID, "no such readback ticket");
        HIPCHK(hipSetDevice(d->device));
        // the slot may hold a later copy by now: it lands after this one (one stream, in order)
        HIPCHK(hipEventSynchronize(d->rb_done[ticket % gs_ctx::kReadbacks]));
        return GS_OK;
    });
}

int gs_sync(gs_ctx* c) {
    return guarded([&] {
        if (!c) throw GsError(GS_ERR_INVALID, "null ctx");
        if (!c->members.empty()) {  // every member synchronised and its errors handled; the first reported
            int rc = GS_OK;
            std::string msg;
            for (gs_ctx* m : c->members) {
                const int r = gs_sync(m);
                if (r != GS_OK && rc == GS_OK) {
                    rc = r;
                    msg = gs_last_error();
                }
            }
            if (rc != GS_OK) throw GsError(rc, msg);
            return GS_OK;
        }
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipDeviceSynchronize());
        for (gs_scene* s : c->scenes) check_frame_errors(s);
        return GS_OK;
    });
}

int gs_timings(gs_ctx* c, gs_stats* out) {
    return guarded([&] {
        if (!c || !out) throw GsError(GS_ERR_INVALID, "null argument");
        if (!c->members.empty()) {  // counts summed over the strips, stage times the slowest strip's
            gs_stats a{};
            for (size_t g = 0; g < c->members.size(); ++g) {
                gs_stats m{};
                const int rc = gs_timings(c->members[g], &m);
                if (rc != GS_OK) throw GsError(rc, gs_last_error());
                if (g == 0) {
                    a = m;
                    continue;
                }
                a.n_vis += m.n_vis;
                a.k_entries += m.k_entries;
                a.k_total += m.k_total;
                a.tiles_unsaturated += m.tiles_unsaturated;
                a.k_chunk0 += m.k_chunk0;
                a.k_chunk1 += m.k_chunk1;
                a.wide_chunk0 += m.wide_chunk0;
                a.wide_chunk1 += m.wide_chunk1;
                a.frames_unsat = std::max(a.frames_unsat, m.frames_unsat);  // frames, not strips (as below)
                a.frames_chunked = std::max(a.frames_chunked, m.frames_chunked);
                a.frames_seeded = std::max(a.frames_seeded, m.frames_seeded);
                a.tile_row_end = std::max(a.tile_row_end, m.tile_row_end);
                a.list_max = std::max(a.list_max, m.list_max);
                a.tiles_long += m.tiles_long;
                for (float* f : {&a.ms_total, &a.ms_project, &a.ms_sort, &a.ms_bin, &a.ms_tile_sort, &a.ms_ranges,
                                 &a.ms_composite, &a.ms_other}) {
                    const float v = *(const float*)((const char*)&m + ((const char*)f - (const char*)&a));
                    *f = std::max(*f, v);
                }
            }
            a.tile_row_begin = 0;
            *out = a;
            return GS_OK;
        }
        HIPCHK(hipSetDevice(c->device));
        for (int k = 1; k <= kStatSlots; ++k) harvest(c, c->fe[(c->fe_cur + k) % kStatSlots]);  // oldest first
        gs_stats st = c->stats;
        if (c->last_scene) {
            collect_stats(c->last_scene, true);
            const FrameCtl& l = c->last_scene->last;
            st.n_vis = l.n_vis;
            st.k_entries = (uint64_t)l.k_chunk[0] + l.k_chunk[1];
            st.k_total = l.k_total;
            st.tiles_unsaturated = l.not_done;
            st.k_chunk0 = l.k_chunk[0];
            st.k_chunk1 = l.k_chunk[1];
            st.wide_chunk0 = l.wide_n[0];
            st.wide_chunk1 = l.wide_n[1];
            st.chunk_fraction = l.n_vis ? (float)l.n_chunk[0] / (float)l.n_vis : 0.0f;
            st.chunk_depth = l.frame_T == kNoSplit ? 0.0f : std::fabs(key_to_float(l.frame_T));
            st.list_max = l.list_max;
            st.tiles_long = l.long_n;
        }
        st.frames = (int32_t)c->comp_frames;
        for (gs_scene* s : c->scenes) collect_stats(s, false);
        st.frames_rendered = c->n_rendered;
        st.frames_chunked = c->n_chunked;
        st.frames_unsat = c->n_unsat;
        st.frames_seeded = c->n_seeded;
        const double k = c->acc_frames ? 1.0 / c->acc_frames : 0.0;
        st.ms_total = (float)(c->acc_ms[ST_TOTAL] * k);
        st.ms_project = (float)(c->acc_ms[ST_PROJECT] * k);
        st.ms_sort = (float)(c->acc_ms[ST_SORT] * k);
        st.ms_bin = (float)(c->acc_ms[ST_BIN] * k);
        st.ms_tile_sort = (float)(c->acc_ms[ST_TSORT] * k);
        st.ms_ranges = (float)(c->acc_ms[ST_RANGES] * k);
        st.ms_composite = (float)(c->comp_frames ? c->acc_comp_ms / c->comp_frames : 0.0);
        st.ms_other = c->acc_frames ? st.ms_total - (st.ms_project + st.ms_sort + st.ms_bin + st.ms_tile_sort +
                                                     st.ms_ranges + st.ms_composite)
                                    : 0.0f;
        *out = st;
        return GS_OK;
    });
}

int gs_timings_reset(gs_ctx* c) {
    return guarded([&] {
        if (!c) throw GsError(GS_ERR_INVALID, "null ctx");
        for (gs_ctx* m : c->members) {
            const int rc = gs_timings_reset(m);
            if (rc != GS_OK) throw GsError(rc, gs_last_error());
        }
        if (!c->members.empty()) return GS_OK;
        HIPCHK(hipSetDevice(c->device));
        for (int k = 1; k <= kStatSlots; ++k) harvest(c, c->fe[(c->fe_cur + k) % kStatSlots]);  // every pending frame
        for (gs_scene* s : c->scenes) collect_stats(s, true);  // their frame counts before the reset
        c->n_rendered = c->n_chunked = c->n_unsat = c->n_seeded = 0;
        for (auto& v : c->acc_ms) v = 0.0;
        c->acc_frames = 0;
        c->acc_comp_ms = 0.0;
        c->comp_frames = 0;
        return GS_OK;
    });
}

int gs_debug_cut_margin(gs_ctx* c, float margin) {
    return guarded([&] {
        if (!c) throw GsError(GS_ERR_INVALID, "null context");
        if (!std::isfinite(margin)) throw GsError(GS_ERR_INVALID, "margin not finite");
        c->cut_margin = margin;
        for (gs_ctx* m : c->members) m->cut_margin = margin;
        return GS_OK;
    });
}

int gs_debug_chunk1_grid(const gs_ctx* c, int occupancy, int cus, int* out_grid, int* out_occupancy) {
    return guarded([&] {
        if (!out_grid) throw GsError(GS_ERR_INVALID, "null out_grid");
        if (c && !c->members.empty()) c = c->members[0];
        const int occ = c ? c->c1_occ : occupancy;
        const int g = c ? c->c1_grid : chunk1_grid(occupancy, cus);
        *out_grid = g;
        if (out_occupancy) *out_occupancy = occ;
        if (g <= 0) throw GsError(GS_ERR_UNSUPPORTED, "k_chunk1's grid cannot be resident");
        return GS_OK;
    });
}

int gs_debug_sort_pairs(gs_ctx* c, uint32_t* keys, uint32_t* vals, uint64_t n, int begin_bit, int end_bit) {
    return guarded([&] {
        if (c && !c->members.empty()) throw GsError(GS_ERR_UNSUPPORTED, "debug exports take a single-device context");
        if (!c || (!keys && n) || (!vals && n)) throw GsError(GS_ERR_INVALID, "null argument");
        if (begin_bit < 0 || end_bit > 32 || begin_bit >= end_bit) throw GsError(GS_ERR_INVALID, "bad bit range");
        if (n >= 0xFFFFFFFFull) throw GsError(GS_ERR_UNSUPPORTED, "n too large");
        if (n == 0) return GS_OK;
        HIPCHK(hipSetDevice(c->device));
        uint32_t *kA = nullptr, *vA = nullptr, *kB = nullptr, *vB = nullptr;
        try {
            dev_alloc(kA, n); dev_alloc(vA, n); dev_alloc(kB, n); dev_alloc(vB, n);
            hipStream_t st = c->stream;
            HIPCHK(hipMemcpyAsync(kA, keys, n * 4, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(vA, vals, n * 4, hipMemcpyHostToDevice, st));
            const auto r = device_sort_pairs(kA, vA, kB, vB, n, begin_bit, end_bit, st);
            HIPCHK(hipMemcpy(keys, r.first, n * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(vals, r.second, n * 4, hipMemcpyDeviceToHost));
        } catch (...) {
            dev_free(kA); dev_free(vA); dev_free(kB); dev_free(vB);
            throw;
        }
        dev_free(kA); dev_free(vA); dev_free(kB); dev_free(vB);
        return GS_OK;
    });
}

// Reference index of each draw rank of the last ref_quirks frame (empty otherwise).
static std::vector<uint32_t> quirk_draw(gs_scene* s) {
    std::vector<uint32_t> d;
    if (!s->last_quirk || !s->qdraw) return d;
    d.resize(s->n);
    HIPCHK(hipMemcpy(d.data(), s->qdraw, s->n * 4, hipMemcpyDeviceToHost));
    return d;
}

// The last frame's visible splats' composite slots as (slot, depth key, reference index, chunk),
// chunk 0 then chunk 1.  Under ref_quirks the slot key is (0, draw rank): reported as (draw rank,
// the Gaussian drawn at that rank).
static std::vector<std::array<uint32_t, 4>> frame_slots(gs_scene* s) {
    collect_stats(s, true);
    const FrameSet& F = s->fs[s->last_fs];
    const uint32_t parts = proj_parts(s->n);
    std::vector<std::array<uint32_t, 4>> out;
    if (!parts) return out;
    const std::vector<uint32_t> qd = quirk_draw(s);
    std::vector<uint32_t> c0(parts), c1(parts);
    std::vector<uint2> sk((size_t)parts * kProjTile);
    std::vector<uint32_t> rect((size_t)parts * kProjTile);
    HIPCHK(hipMemcpy(rect.data(), F.srect, rect.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c0.data(), F.c0, parts * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c1.data(), F.c1, parts * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sk.data(), F.skey, sk.size() * sizeof(uint2), hipMemcpyDeviceToHost));
    const bool chunk1 = s->last.n_chunk[1] > 0;
    for (int ch = 0; ch < (chunk1 ? 2 : 1); ++ch)
        for (uint32_t p = 0; p < parts; ++p)
            for (uint32_t q = 0; q < (ch ? c1[p] : c0[p]); ++q) {
                const uint32_t g = ch ? slot_c1(p, q) : slot_c0(p, q);
                if (rect[g] == kRectHole) continue;  // an invisible chunk-0 candidate
                out.push_back({g, qd.empty() ? sk[g].x : sk[g].y, qd.empty() ? sk[g].y : qd[sk[g].y], (uint32_t)ch});
            }
    return out;
}

int gs_debug_last_order(gs_ctx* c, gs_scene* s, uint32_t* out_keys, uint32_t* out_index, uint64_t cap,
                        uint64_t* out_n) {
    return guarded([&] {
        if (c && !c->members.empty()) throw GsError(GS_ERR_UNSUPPORTED, "debug exports take a single-device context");
        if (!c || !s || !out_n) throw GsError(GS_ERR_INVALID, "null argument");
        if (!s->have_frame) throw GsError(GS_ERR_INVALID, "no frame rendered yet");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipDeviceSynchronize());  // both frame sets' streams
        auto sl = frame_slots(s);  // every composite slot, sorted here by (key, index): the visible set
        std::sort(sl.begin(), sl.end(), [](const std::array<uint32_t, 4>& a, const std::array<uint32_t, 4>& b) {
            return a[1] != b[1] ? a[1] < b[1] : a[2] < b[2];
        });
        *out_n = sl.size();
        const uint64_t m = std::min<uint64_t>(cap, sl.size());
        for (uint64_t k = 0; k < m; ++k) {
            if (out_keys) out_keys[k] = sl[k][1];
            if (out_index) out_index[k] = sl[k][2];
        }
        return GS_OK;
    });
}

int gs_debug_last_records(gs_ctx* c, gs_scene* s, float* out16, uint64_t cap) {
    return guarded([&] {
        if (c && !c->members.empty()) throw GsError(GS_ERR_UNSUPPORTED, "debug exports take a single-device context");
        if (!c || !s || !out16) throw GsError(GS_ERR_INVALID, "null argument");
        if (!s->have_frame) throw GsError(GS_ERR_INVALID, "no frame rendered yet");
        if (s->last_quirk) throw GsError(GS_ERR_UNSUPPORTED, "per-Gaussian records of a ref_quirks frame "
                                                             "(a Gaussian may be drawn twice): use gs_debug_last_slots");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipDeviceSynchronize());  // both frame sets' streams
        const uint64_t m = std::min(cap, s->n);
        const auto sl = frame_slots(s);
        const FrameSet& F = s->fs[s->last_fs];
        if (m) {  // r01 -> words [0, 8); r2 -> words [12, 16); colour below
            if (!s->dbg) dev_alloc(s->dbg, 3 * (size_t)std::max<uint64_t>(s->n, 1));
            ProjParams rp = s->last_pp;  // records of every visible Gaussian (a frame stores fewer)
            rp.rec = records(s, F);
            rp.rec_all = 1;
            launch_records(rp, c->stream);
            HIPCHK(hipDeviceSynchronize());  // both frame sets' streams
            const Records rc = records(s, F);
            const uint64_t n = s->n;           // storage slot j holds reference record orig[j]
            std::vector<float> a((size_t)n * 8), b((size_t)n * 4);
            std::vector<uint32_t> orig(n);
            HIPCHK(hipMemcpy2D(a.data(), 32, rc.r01, (size_t)rc.stride * 16, 32, n, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(b.data(), F.r2, b.size() * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(orig.data(), s->orig, n * 4, hipMemcpyDeviceToHost));
            for (uint64_t j = 0; j < n; ++j) {
                const uint64_t o = orig[j];
                if (o >= m) continue;
                std::memcpy(out16 + 16 * o, &a[8 * j], 32);
                std::memset(out16 + 16 * o + 8, 0, 16);
                std::memcpy(out16 + 16 * o + 12, &b[4 * j], 16);
            }
        }
        // colour words [8, 11): from the composite record of each slot of the frame
        if (!sl.empty()) {
            const size_t ns = (size_t)proj_parts(s->n) * kProjTile;
            std::vector<float> cr(ns * 12);
            HIPCHK(hipMemcpy(cr.data(), F.crec, ns * 48, hipMemcpyDeviceToHost));
            for (const auto& e : sl)
                if (e[2] < m) std::memcpy(out16 + 16 * (uint64_t)e[2] + 8, &cr[12 * (size_t)e[0] + 8], 12);
        }
        return GS_OK;
    });
}

int gs_debug_last_slots(gs_ctx* c, gs_scene* s, uint32_t* out16, uint64_t cap, uint64_t* out_n) {
    return guarded([&] {
        if (c && !c->members.empty()) throw GsError(GS_ERR_UNSUPPORTED, "debug exports take a single-device context");
        if (!c || !s || !out_n) throw GsError(GS_ERR_INVALID, "null argument");
        if (!s->have_frame) throw GsError(GS_ERR_INVALID, "no frame rendered yet");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipDeviceSynchronize());
        const auto sl = frame_slots(s);
        *out_n = sl.size();
        const uint64_t m = out16 ? std::min<uint64_t>(cap, sl.size()) : 0;
        if (!m) return GS_OK;
        const FrameSet& F = s->fs[s->last_fs];
        const size_t ns = (size_t)proj_parts(s->n) * kProjTile;
        std::vector<uint32_t> cr(ns * 12), rect(ns);
        HIPCHK(hipMemcpy(cr.data(), F.crec, ns * 48, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(rect.data(), F.srect, ns * 4, hipMemcpyDeviceToHost));
        for (uint64_t k = 0; k < m; ++k) {
            const auto& e = sl[k];
            uint32_t* o = out16 + 16 * k;
            o[0] = e[1];
            o[1] = e[2];
            o[2] = e[3];
            o[3] = rect[e[0]];
            std::memcpy(o + 4, &cr[12 * (size_t)e[0]], 48);
        }
        return GS_OK;
    });
}

int gs_debug_tile_lists(gs_ctx* c, gs_scene* s, uint32_t* out_ranges, uint64_t ranges_cap, uint32_t* out_entries,
                        uint64_t entries_cap, uint64_t* out_tiles, uint64_t* out_entries_n) {
    return guarded([&] {
        if (c && !c->members.empty()) throw GsError(GS_ERR_UNSUPPORTED, "debug exports take a single-device context");
        if (!c || !s || !out_tiles || !out_entries_n) throw GsError(GS_ERR_INVALID, "null argument");
        if (!s->have_frame) throw GsError(GS_ERR_INVALID, "no frame rendered yet");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipDeviceSynchronize());
        collect_stats(s, true);
        if (s->last.n_chunk[1] > 0)
            throw GsError(GS_ERR_UNSUPPORTED, "tile lists of a two-chunk frame (render with chunk_fraction >= 1)");
        const FrameSet& F = s->fs[s->last_fs];
        const int nt = s->last_tiles;
        *out_tiles = (uint64_t)std::max(nt, 0);
        std::vector<uint2> rg((size_t)std::max(nt, 1));
        if (nt > 0) HIPCHK(hipMemcpy(rg.data(), F.ranges, (size_t)nt * sizeof(uint2), hipMemcpyDeviceToHost));
        uint64_t total = 0;
        for (int t = 0; t < nt; ++t) total = std::max<uint64_t>(total, rg[t].y);
        *out_entries_n = total;
        if (out_ranges)
            for (int t = 0; t < nt && (uint64_t)t < ranges_cap; ++t) {
                out_ranges[2 * t] = rg[t].x;
                out_ranges[2 * t + 1] = rg[t].y;
            }
        const uint64_t m = out_entries ? std::min(entries_cap, total) : 0;
        if (!m) return GS_OK;
        std::vector<uint32_t> tv(m);
        HIPCHK(hipMemcpy(tv.data(), F.tvB, m * 4, hipMemcpyDeviceToHost));
        const size_t ns = (size_t)proj_parts(s->n) * kProjTile;
        std::vector<uint2> sk(ns);
        HIPCHK(hipMemcpy(sk.data(), F.skey, ns * sizeof(uint2), hipMemcpyDeviceToHost));
        const std::vector<uint32_t> qd = quirk_draw(s);
        for (uint64_t e = 0; e < m; ++e) {
            const uint32_t g = tv[e];
            if (g >= ns) throw GsError(GS_ERR_INTERNAL, "tile list entry out of range");
            out_entries[2 * e] = qd.empty() ? sk[g].x : sk[g].y;
            out_entries[2 * e + 1] = qd.empty() ? sk[g].y : qd[sk[g].y];
        }
        return GS_OK;
    });
}

int gs_debug_tile_list_check(gs_ctx* c, gs_scene* s, uint64_t out[5]) {
    return guarded([&] {
        if (c && !c->members.empty()) throw GsError(GS_ERR_UNSUPPORTED, "debug exports take a single-device context");
        if (!c || !s || !out) throw GsError(GS_ERR_INVALID, "null argument");
        if (!s->have_frame) throw GsError(GS_ERR_INVALID, "no frame rendered yet");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipDeviceSynchronize());
        collect_stats(s, true);
        if (s->last.n_chunk[1] > 0)
            throw GsError(GS_ERR_UNSUPPORTED, "tile lists of a two-chunk frame (render with chunk_fraction >= 1)");
        const FrameSet& F = s->fs[s->last_fs];
        const int nt = std::max(s->last_tiles, 0);
        std::vector<uint2> rg((size_t)std::max(nt, 1));
        if (nt > 0) HIPCHK(hipMemcpy(rg.data(), F.ranges, (size_t)nt * sizeof(uint2), hipMemcpyDeviceToHost));
        uint64_t total = 0;
        for (int t = 0; t < nt; ++t) total = std::max<uint64_t>(total, rg[t].y);
        std::vector<uint32_t> tv(total);
        if (total) HIPCHK(hipMemcpy(tv.data(), F.tvB, total * 4, hipMemcpyDeviceToHost));
        const size_t ns = (size_t)proj_parts(s->n) * kProjTile;
        std::vector<uint2> sk(std::max<size_t>(ns, 1));
        std::vector<uint32_t> sr(std::max<size_t>(ns, 1));
        if (ns) {
            HIPCHK(hipMemcpy(sk.data(), F.skey, ns * sizeof(uint2), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(sr.data(), F.srect, ns * 4, hipMemcpyDeviceToHost));
        }
        uint64_t dup = 0, order = 0, gaps = 0, bad = 0, prev_end = 0;
        std::vector<uint32_t> idx;
        for (int t = 0; t < nt; ++t) {
            const uint64_t b = rg[t].x, e = rg[t].y;
            if (b != prev_end || e < b) ++gaps;
            prev_end = e;
            idx.clear();
            uint64_t last = 0;
            for (uint64_t j = b; j < e && j < total; ++j) {
                const uint32_t g = tv[j];
                if (g >= ns || sr[g] == kRectHole || sr[g] == kRectEmpty) {
                    ++bad;
                    continue;
                }
                const uint64_t k = ((uint64_t)sk[g].x << 32) | sk[g].y;
                if (j > b && k <= last) ++order;
                last = k;
                idx.push_back(sk[g].y);
            }
            std::sort(idx.begin(), idx.end());
            for (size_t j = 1; j < idx.size(); ++j) dup += idx[j] == idx[j - 1] ? 1u : 0u;
        }
        out[0] = total;
        out[1] = dup;
        out[2] = order;
        out[3] = gaps;
        out[4] = bad;
        return GS_OK;
    });
}

}  // extern "C"
