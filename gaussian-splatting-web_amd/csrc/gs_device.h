// gs_device.h — shared constants, the device-side frame control block, kernel parameter blocks
// and launchers (host side of gs_kernels.hip).
//
// A frame is a fixed sequence of launches with no host round trip: every count that depends on
// the data (visible splats, entries per chunk, unsaturated tiles) lives in FrameCtl on the device
// and every kernel sizes its work from it (grid-stride loops over a worst-case grid).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/gsplat.h"

namespace gs {

constexpr int kTile = 16;             // 16x16-pixel composite tile
constexpr int kProjThreads = 256;  // = kSortThreads: k_project works on radix partitions
constexpr int kSortThreads = 256;     // 4 waves
constexpr int kSortIPT = 16;          // items per thread
constexpr int kProjTile = 1024;       // projection partition: bounds, candidates, slot block
constexpr int kProjRounds = kProjTile / kProjThreads;  // work units (rounds of kProjThreads) per partition
constexpr int kCullBlock = 64;        // storage slots per block bound (one wave's cull planes)
constexpr float kCullFaint = -1.0f;   // cull plane w of a Gaussian whose opacity is below 1/255
constexpr int kUnitShards = 8;        // the frame's work-unit list, sharded (FrameCtl::unit_n)
constexpr int kSortTile = kSortThreads * kSortIPT;  // 4096 elements per radix partition
constexpr int kBinThreads = 1024;     // binning workgroup (one partition of the chunk's ranks)
#ifndef GS_BIN_PARTS
#define GS_BIN_PARTS 256
#endif
constexpr int kBinParts = GS_BIN_PARTS;  // binning partitions per chunk (rows of BinParams::bmat)
constexpr uint32_t kBinPartsSmall = 128;  // moving frames' and chunk 1's binning partitions (BinParams::nparts)
constexpr uint32_t kBinMaxUnits = 4096;   // units per binning partition (scenes up to 2^28 Gaussians at kBinParts)
constexpr int kBmatRows = kBinParts > 256 ? kBinParts : 256;  // bmat rows: binning partitions, and the
                                                              // per-tile sort's long-list scratch (256 per tile)
constexpr int kBandTiles = 8192;      // tiles per binning band inside k_chunk1 (static LDS)
constexpr int kBandTilesMax = 36000;  // largest band of the binning launches (dynamic LDS)
constexpr int kHistShards = 8;        // global histograms sharded by blockIdx % 8 (XCD group)
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // key of a culled Gaussian (no visible splat has it)
constexpr int kRecFloats = 16;        // 64-B projected record
constexpr int kMaxGrid = 2048;        // persistent grids: 8 workgroups per CU
// Splats of at least wide_tiles(n_tiles) box tiles are "wide": listed at projection and walked in
// binning by whole waves or workgroups (wide_listed).  64 at 1080p (the few workgroups whose
// partitions met the near splats walked them all), up to 256 at 4K (there the many medium splats
// walk faster one per thread: 4K binning 170 us at 256, 225 us at 64).
__host__ __device__ inline uint32_t wide_tiles(int n_tiles) {
    const int t = n_tiles / 128;
    return (uint32_t)(t < 64 ? 64 : (t > 256 ? 256 : t));
}
constexpr int kMaxMerge = 16;           // compacted radix input: partitions per downsweep workgroup
constexpr uint32_t kGroupParts = 32;    // radix partitions per group sum (the downsweep's offsets)

// Packed tile rectangle carried through the depth sort (32 bits): tx0[0:12) ty0[12:24)
// (w-1)[24:28) (h-1)[28:32).  Rectangles wider or taller than 16 tiles use kRectLarge (the
// binning reads the full rectangle from the record); kRectEmpty = visible but binds no tile.
constexpr uint32_t kRectLarge = 0xFFFFFFFFu;
constexpr uint32_t kRectEmpty = 0xFFFFFFFEu;
constexpr uint32_t kRectHole = 0xFFFFFFFDu;   // a composite slot whose candidate was not visible

// Device-side error bits (FrameCtl::err); a nonzero word fails the frame.
constexpr uint32_t kErrOverflow = 1u;
constexpr uint32_t kErrBarrier = 2u;   // a grid barrier of k_chunk1 timed out
constexpr uint32_t kErrBinning = 4u;   // a binning workgroup emitted other entries than it counted
                                       // (k_bin_emit's check of BinParams::bchk): a tile list is wrong
constexpr uint32_t kErrState = 8u;     // a frame-state count read from FrameCtl / StatShard exceeded the
                                       // buffer it indexes (a unit list, the partition list, the wide
                                       // list): the kernels skip the work instead of reading past it

// Saturation-depth histogram: tile saturated at depth key k -> bucket (k >> 21) - base, clamped to
// [0, kSatBuckets): quarter-octave buckets of depth from the last frame's nearest visible splat
// (the base, set by the host).  The chunk controller places the threshold at a quantile of it.
constexpr int kSatBuckets = 32;
constexpr int kSatShift = 21;
__host__ __device__ inline uint32_t sat_bucket(uint32_t key, uint32_t base) {
    const int b = (int)(key >> kSatShift) - (int)base;
    return (uint32_t)(b < 0 ? 0 : (b >= kSatBuckets ? kSatBuckets - 1 : b));
}

struct FrameCtl {                 // zeroed at the start of every frame
    unsigned long long k_total;   // sum of tile counts over visible splats (project)
    uint32_t n_vis;               // visible splats (project)
    uint32_t k_chunk[2];          // (tile, splat) entries per chunk (binning scan)
    uint32_t not_done;            // tiles still accepting splats after chunk 0
    uint32_t err;
    uint32_t wide_n[2];           // wide splats per chunk (binning statistics)
    uint32_t n_chunk[2];          // splats (composite slots) per chunk
    uint32_t key_min_inv;         // ~(smallest depth key of a visible splat) (project)
    uint32_t key_max;             // largest depth key of a visible splat (project)
    uint32_t sat_key;             // depth key of the farthest splat a tile saturated at (the frame's end, k_chunk1)
    uint32_t unit_n[kUnitShards]; // chunk-0 work units per shard (k_cull; see ProjParams::units)
    uint32_t c1_parts;            // chunk 1: items listed in ProjParams::plist: 64-slot blocks (partitions without block bounds)
    uint32_t c0_parts;            // chunk 0: projection partitions listed in ProjParams::plist0 (k_part_list)
    uint32_t seed_T;              // a seeded frame's chunk threshold (k_seed_pick; ProjParams::thresh_dev)
    uint32_t frame_T;             // the frame's chunk threshold, whichever its source (k_part_list)
    uint32_t sat_hist[kSatBuckets];  // tiles saturated by the end of the frame, by saturation depth
                                     // (sat_bucket; summed from the shards at the frame's end)
    uint32_t list_max;            // longest tile list of the frame (either chunk) when > kListMaxMin, else 0
    uint32_t long_n;              // tiles the huge sort shape left to the long-list pass (TileSortParams::long_tiles)
};

// Per-frame counters that many workgroups add to, sharded so that no address takes more than a
// few hundred device-scope atomics (one address serialises them at ~11 ns each): workgroup b adds
// to shard b % kStatShards; the frame's end (k_chunk1) sums the shards into FrameCtl and zeroes them.
// 16 shards: one wave's read of 64 shards was most of the frame's end (11.5 -> 7 us with 16), and
// 16 keeps every address at a few hundred atomics per frame (8160 tiles, <= 2048 workgroups).
#ifndef GS_STAT_SHARDS
#define GS_STAT_SHARDS 16
#endif
constexpr int kStatShards = GS_STAT_SHARDS;
// The wide-splat list (ProjParams::wlist) is sharded by projection partition (shard = partition %
// kWideShards, each shard a region of its partitions' slot count, counter StatShard::wl_n of the
// shard's index): a counter per shard instead of one for the frame (same-address atomics
// serialise; at 4K one counter doubled k_project).
constexpr uint32_t kWideShards = (uint32_t)kStatShards;
__host__ __device__ inline uint32_t wide_shard_cap(uint32_t parts) {
    return (parts + kWideShards - 1) / kWideShards * (uint32_t)kProjTile;
}
struct StatShard {
    unsigned long long k_total;
    uint32_t n_vis, key_min_inv, key_max;
    uint32_t n_chunk[2];
    uint32_t sat_key;             // composite: max saturation key of the shard's tiles
    uint32_t sat_hist[kSatBuckets];  // composite: the shard's tiles by saturation depth
    uint32_t order_n[2];          // shards 0-7: the composite order of XCD band x (k_tile_sort)
    uint32_t wl_n[2];             // wide splats of wide-list shard (= this shard's index) per chunk
                                  // (ProjParams::wlist; zeroed with the shard, not summed)
    uint32_t list_max;            // k_tile_sort: longest list of the shard's tiles (only lists > kListMaxMin)
};
constexpr uint32_t kListMaxMin = 1024;  // shorter lists do not report their length (one atomic per long list)

// Bound of a projection partition (k_part_bounds, at upload): box of its finite positions,
// largest ||R(q) diag(s)||_F^2, count of finite positions.
struct PartBound {
    float lo[3], hi[3], trs;
    uint32_t nfin;
};

// Composite slots.  k_project gives the chunk-0 splats of projection partition `part` (kProjTile
// storage slots) the slots part * kProjTile + q, q < c0[part] (q = the candidate's position in
// the partition's list; an invisible candidate leaves a hole); k_records gives the chunk-1
// splats of that partition part * kProjTile + kProjTile - 1 - q, q < c1[part].  A Gaussian is in
// at most one chunk, so the two never meet.  Per slot: the composite record (3 float4),
// skey = (depth key, reference index) (the per-tile sort key: ties in depth fall back to the
// index, as the reference's stable sort over index-ordered slots), the storage index and the
// packed rect.  Work unit u = part * kProjRounds + round covers slots round * kProjThreads ..
// (+ kProjThreads) of the partition.
__host__ __device__ inline uint32_t proj_parts(uint64_t n) { return (uint32_t)((n + kProjTile - 1) / kProjTile); }
__host__ __device__ inline uint32_t slot_c0(uint32_t part, uint32_t q) { return part * (uint32_t)kProjTile + q; }
__host__ __device__ inline uint32_t slot_c1(uint32_t part, uint32_t q) {
    return part * (uint32_t)kProjTile + (uint32_t)kProjTile - 1u - q;
}
__host__ __device__ inline uint32_t unit_shard_cap(uint32_t parts) {
    return (parts + kUnitShards - 1) / kUnitShards * kProjRounds;
}

// Scene layout in HBM (storage slots in Morton order, orig[] = reference index): a 48-B
// geometry record per Gaussian (3 float4: x, y, z, opacity logit | scale xyz, rot.x | rot.y,
// rot.z, rot.w, 0) gathered by k_project for the chunk-0 candidates, a 16-B cull plane (x, y, z,
// ||R(q) diag(s)||_F^2) streamed by k_cull, and the packed SH coefficients, sh_quads(n_sh) float4
// per Gaussian (coefficient k channel c at 3k + c; 192 B at degree 3), read by k_project for
// the splats it keeps (Morton order makes those reads nearly dense).
// Per-Gaussian records (the debug dump; rec_all): Records::r01 = 3 quads per Gaussian: cx, cy,
// e1x', e1y' | e2x', e2y', log2(op), pixel box x (centre in pixels; quad axes e/|e|^2 *
// sqrt(log2 e); box x0 | x1 << 16, u32 bits) | colour; r2[j] = depth key, tile count, pixel box
// x, pixel box y (u32 bits), written for every visible splat of a frame.
// Composite record, 3 float4 per slot: [0], [1] = the r01 quads, [2] = r, g, b, depth key bits.
__host__ __device__ inline uint32_t sh_quads(int n_sh) { return (uint32_t)(3 * n_sh + 3) / 4; }

struct Records {
    float4* r01;      // debug records, stride quads per Gaussian (null outside the debug dump)
    float4* r2;
    uint32_t stride;  // 3
    uint32_t off;     // 0
};
__host__ __device__ inline float4* rec_r01(const Records& r, uint64_t j) {
    return r.r01 + j * r.stride + r.off;
}

struct ProjParams {
    const float4* geo;        // [n][3] geometry records
    const float4* cull;       // [n] cull planes (x, y, z, ||R(q) diag(s)||_F^2), two-phase frames
    uint32_t n;
    float V[16];              // view, column-major
    float PV[16];             // proj * view (host-computed in the reference's order)
    float scale_mod;
    float P00, P11;
    float focal;              // W * P00 / 2 (src/simple_render.ts:273)
    float w01_spec2;          // lambda_max(W01 W01^T), W01 = rows 0-1 of the view's 3x3 block
                              // (x 1.0001): the conservative cull bound's camera factor
    int W, H;
    int tile_row_begin, tile_row_end, tiles_x;
    Records rec;              // out: r2 of every visible Gaussian (k_records: r01 too)
    FrameCtl* ctl;
    StatShard* stats;         // [kStatShards] (n_vis, k_total, key range, n_chunk)
    uint32_t thresh;          // chunk-0 threshold key: chunk 0 = visible splats with key < thresh
    // composite slots (see slot_c0): records, sort keys, rects, per-partition counts
    float4* crec;
    uint2* skey;
    uint32_t* srect;
    uint32_t* c0;             // [parts] chunk-0 splats per projection partition (k_project)
    uint32_t* c1;             // [parts] chunk-1 splats per projection partition (k_records; zeroed by k_cull)
    uint16_t* cand;           // [parts * kProjTile] chunk-0 candidates: offsets in the partition (k_cull)
    uint32_t* units;          // [kUnitShards][unit_shard_cap] the non-empty chunk-0 work units (k_cull)
    const PartBound* bounds;  // [parts] (k_part_bounds)
    const PartBound* bbounds; // [ceil(n / kCullBlock)] (k_block_bounds), nullable
    const uint32_t* orig;     // [n] reference index of each storage slot (Morton order)
    uint32_t* sidx;           // [slots] storage index of each composite slot
    // [slots] the slots of wide splats (>= wide_tiles box tiles): chunk 0's from the front,
    // chunk 1's from the back, sharded (kWideShards); binning spreads them over all its workgroups
    uint32_t* wlist;
    uint32_t wide_tiles;      // wide_tiles(n_tiles) of the frame (strip)
    // chunk 1: the tiles chunk 0 left unsaturated as bits, umask_w words per strip tile row (bit
    // x & 31 of word x >> 5: tile x), set by the chunk-0 composite and zeroed by k_part_list (see
    // CompositeParams::umask); rec_all: k_records dumps every visible Gaussian's record (debug)
    uint32_t* umask;
    uint32_t umask_w;
    uint32_t* plist;          // [parts] chunk 1: the partitions that may hold chunk-1 splats (k_chunk1)
    uint32_t* plist0;         // [parts] chunk 0: the partitions that may hold candidates (k_part_list)
    int rec_all;
    float cam[3];             // camera position (SH view direction)
    const float4* sh;         // [n][shq] packed SH coefficients
    uint32_t shq;             // sh_quads(n_sh)
    uint32_t key_zero;        // ref_quirks: slot sort key (0, draw rank) -- orig holds the rank
    // A seeded frame (no usable history: a first frame, a camera cut) takes its chunk threshold
    // from the device (thresh_dev = &FrameCtl::seed_T, written by k_seed_pick) instead of thresh.
    const uint32_t* thresh_dev;
    float* seedh;             // [cells][kSeedBuckets] alpha mass by coarse cell and depth bucket
    uint32_t seed_stride;     // one sampled run of kSeedRun Gaussians per seed_stride runs
    uint32_t seed_base;       // depth bucket 0 = keys from (seed_base << kSatShift): the near plane
    int seed_cx, seed_cy;     // coarse cells (kSeedCell px) across the frame / strip
    float seed_tau;           // alpha mass per pixel taken as saturation
    // per-tile chunk-0 cut (k_part_list snapshots it): tile_sat[abs tile] = depth key at which the
    // tile saturated in the last frame that composited it (kSentinel: unknown / not saturated),
    // written by the composites; cut[strip tile] = this frame's bound (tile_cut_bound), nullable
    const uint32_t* tile_sat;
    uint16_t* cut;
    uint32_t* cutb;           // [cut_blocks] min | max << 16 of the block's bounds
    float cut_margin;         // depth factor (>= 1) applied to the saturation key
    uint32_t cull_grid, proj_grid;  // k_cull / k_project grids (0: the defaults)
};
// Per-tile chunk-0 cut (round 6).  A chunked frame's chunk 0 holds every visible splat nearer than
// the global threshold T (the deepest tile's saturation depth), but most tiles saturate well before
// it (bench view: 46 % of the chunk-0 entries are reached, tools/diag/sat_position.py).  With the
// cut, chunk 0 bins entry (tile t, splat) only when the splat's key < cut[t] << 16, cut[t] = the
// tile's saturation key in the last frame scaled by a margin, rounded up to 16 bits (0xFFFF: no
// cut); the entries it leaves out are binned by chunk 1 into the tiles that are still unsaturated
// after chunk 0 (a second walk over chunk 0's units, key >= cut[t], done[t] == 0), behind every
// entry chunk 0 blended there, so each tile still blends its whole list in (key, index) order and
// the image does not depend on the cut.
constexpr int kCutMaxTiles = 16384;  // frames (strips) of at most this many tiles: the band's cut
                                     // bounds fit beside the binning's LDS counters
// keep iff key < c << 16 (a visible splat's key is below 0x80000000, so c = 0xFFFF keeps all)
__host__ __device__ inline bool cut_keep(uint16_t c, uint32_t key) {
    return (key >> 16) < (uint32_t)c;
}
// The bounds' minimum and maximum per block of kCutBlock x kCutBlock tiles (ProjParams::cutb),
// so binning classifies a splat from its rect's few blocks: no entry kept, every entry kept, or
// a test per entry.
constexpr int kCutBlock = 4;
constexpr int kCutMaxBlocks = 2048;  // blocks of a frame with the cut at most (k_chunk1's static LDS)
__host__ __device__ inline uint32_t cut_blocks_x(int tiles_x) { return (uint32_t)(tiles_x + kCutBlock - 1) / kCutBlock; }
__host__ __device__ inline uint32_t cut_blocks(int tiles_x, int rows) {
    return cut_blocks_x(tiles_x) * (uint32_t)((rows + kCutBlock - 1) / kCutBlock);
}

// Coarse depth estimate of a seeded frame: sampled Gaussians' alpha mass op * 2 pi sigma^2 by
// 64x64-pixel cell and quarter-octave depth bucket (sat_bucket's, from the near plane)
constexpr int kSeedCell = 64;
constexpr int kSeedBuckets = 64;
constexpr int kSeedRun = 16;            // a sample = a run of 16 consecutive storage slots (Morton order)
constexpr int kSeedRunsPerCell = 64;    // about this many sampled runs per cell


// Element filter of a radix pass (the first pass of a depth chunk decides chunk membership).
enum RadixFilter {
    kFiltNone = 0,
    kFiltSentinel = 1,  // drop culled Gaussians (key == kSentinel)
    kFiltBelow = 2,     // chunk 0: key < thresh
    kFiltTail = 3       // chunk 1: thresh <= key < kSentinel and the rect touches an unsaturated tile
};

struct SortPass {
    const uint32_t* keys_in;
    const uint32_t* vals_in;  // nullptr: values are the element index (first depth pass)
    const uint32_t* aux_in;   // optional second value array carried with the elements
    uint32_t* keys_out;
    uint32_t* vals_out;
    uint32_t* aux_out;
    uint32_t n;               // element count, or an upper bound when n_dev is set
    const uint32_t* n_dev;    // device-side element count (nullable)
    const uint32_t* gate;     // optional: the pass is empty when *gate == 0
    const uint32_t* part_count;  // optional: partition p holds part_count[p] elements at its front
                                 // (input compacted by k_project; the upsweep is skipped)
    uint32_t parts_max;       // partitions of the upper bound: stride of `offsets`, grid bound
    int ipt;                  // items per thread: partitions of 256 * ipt elements (4, 8 or 16;
                              // 16 when part_count is set, k_project's partitions)
    int merge;                // part_count set: partitions per downsweep workgroup (<= kMaxMerge)
    int shift;
    uint32_t mask;            // digit mask (<= 255)
    int filter;               // RadixFilter
    uint32_t thresh;          // chunk threshold key (kFiltBelow / kFiltTail)
    uint32_t* count_out;      // optional: number of elements kept (written by the downsweep)
    // kFiltTail: the element's tile rect is aux; wide rects from the record; unsaturated-tile SAT
    Records rec;
    const uint32_t* sat;
    int tiles_x, tile_row_begin;
    uint32_t* hist;           // [kHistShards][256] digit histogram of this pass (zeroed; the
                              // upsweep accumulates it, the downsweep scans it into digit bases)
    uint32_t* offsets;        // [parts][256] scratch: partition counts (upsweep)
    uint32_t* gsum;           // [parts / kGroupParts][256] group sums of the counts (zeroed; reset
                              // by the chunk's tile scan)
};

struct BinParams {
    const uint2* skey;            // [slots] (depth key, reference index)
    const uint32_t* sidx;         // [slots] storage index
    const uint32_t* srect;        // [slots] packed tile rectangle
    const uint32_t* cnt;          // [parts] the chunk's splats per projection partition (c0 or c1)
    uint32_t parts;               // projection partitions
    const uint32_t* units;        // chunk 0: the frame's work-unit list (ProjParams::units); chunk 1:
                                  // null (every unit of every partition)
    Records rec;                  // r2 (wide rects)
    const float4* crec;           // composite records, 3 float4 per slot
    const uint8_t* done;          // chunk 1: per-tile "saturated after chunk 0"
    FrameCtl* ctl;
    int chunk;                    // 0 or 1
    int tile_row_begin, tiles_x;
    uint32_t capacity;            // entry capacity of the tile-list arrays
    uint2* ranges;                // [n_tiles] out (k_bin_emit / the tile scan): [begin, end) of each tile's list
    uint32_t n_tiles;
    uint32_t* bmat;               // [kBinParts][n_tiles] entries of binning partition p in tile t,
                                  // then (k_bin_colscan) the entries of the earlier partitions
    uint32_t* tbase;              // [n_tiles] entries per tile, then (chunk 1's tile scan) the tile's begin
    uint32_t* tvals;              // out: composite slots, grouped by tile, unordered in a tile
    int rows;                     // tile rows of the strip
    uint32_t* order;              // chunk 0 (nullable): the composite's tile order, lists longer than
                                  // heavy_len first in each XCD band (k_bin_colscan)
    StatShard* stats;             // order_n counters (shard x = band x)
    uint32_t heavy_len;
    uint32_t band_tiles;          // tiles per binning band (LDS counters / cursors; set by the launcher)
    uint32_t pref_words;          // LDS words of the per-partition unit prefix (set by the launcher)
    uint32_t wide_cap;            // LDS queue of wide splats per workgroup (set by the launcher; 0 with wlist)
    uint32_t wide_tiles;          // splats of >= this many box tiles are wide (ProjParams::wide_tiles)
    const uint32_t* wlist;        // nullable: the chunk's wide splats (ProjParams::wlist), walked
                                  // by the waves of every workgroup in turn instead of the LDS queue
    uint32_t uid_lds;             // 1: the partition's unit entries cached in LDS after the unit
                                  // prefix (set by the launcher when it fits; chunk 0 only)
    // [bin_chk_words(n_tiles)] per binning workgroup (partition, band): checksums of the entries
    // k_bin_count counted per tile (sum of counts, sum of count x bin_hash(tile)); k_bin_emit
    // compares the entries it emitted with them and sets kErrBinning on a difference
    uint2* bchk;
    // per-tile chunk-0 cut (see kCutMaxTiles), nullable: chunk 0 keeps entry (t, g) iff
    // cut_keep(cut[t], key(g)); chunk 1 also walks chunk 0's units (cut_units, counts in the unit
    // entries) and bins the entries chunk 0 left out into the tiles it left unsaturated
    const uint16_t* cut;
    const uint32_t* cutb;         // [cut_blocks(tiles_x, rows)] (ProjParams::cutb)
    const uint32_t* cut_units;
    // binning partitions of this chunk: kBinParts, or kBinPartsSmall for chunk 1 and for chunk 0
    // under a moving camera (render_frame; each holds at most kBinMaxUnits units)
    uint32_t nparts;
};
// Binning workgroups of a chunk at most (the launches' bands of up to kBandTilesMax tiles and
// k_chunk1's of kBandTiles): the size of BinParams::bchk.
__host__ __device__ inline uint32_t bin_chk_words(uint32_t n_tiles) {
    return (uint32_t)kBinParts * ((n_tiles + kBandTiles - 1) / kBandTiles + 1);
}

// Per-tile sort of the tile lists (k_tile_sort): each tile's slots ordered by their sort key,
// key(g) = g (slots are depth ranks) or, with skey, (skey[g].x << 32) | skey[g].y.
struct TileSortParams {
    const uint2* ranges;          // [n_tiles]
    uint32_t* in;                 // unordered lists (k_bin_emit); scratch of ts_long once it has read them
    uint32_t* out;                // the same lists, each in ascending key order
    const uint2* skey;            // nullable
    const uint8_t* done;          // chunk 1: saturated tiles are skipped (nullable)
    uint32_t* scratch;            // [n_tiles][256] long lists' bucket ends (the binning's bmat, dead by then)
    int n_tiles;
    int big;                      // chunk 0 with long lists: 1 = the 256-thread shape (k_tile_sort_big),
                                  // 2 = the huge shape (k_tile_sort_huge: lists of <= 7168 in LDS)
    // chunk 1: the tiles chunk 0 left unsaturated, a compact list (CompositeParams::c1tiles) of
    // *c1_n entries; the launch walks it instead of every tile (nullable)
    const uint32_t* c1tiles;
    const uint32_t* c1_n;
    // the huge shape (big == 2: two 1024-thread workgroups per CU) sorts lists of <= 7168 entries in
    // one LDS round; a longer list's tile, or one with more than kTsHeavy keys in one bucket, is
    // appended here (count FrameCtl::long_n) and sorted afterwards by the 256-thread shape's
    // linear long-list path (launch_tile_sort's second launch; required with big == 2)
    uint32_t* long_tiles;
    uint32_t* long_n;             // &FrameCtl::long_n
    StatShard* stats;             // nullable: list_max
    uint32_t long_grid;           // workgroups of the long-list launch (k_tile_sort_list strides the list)
};

constexpr uint32_t kTsBigMean = 800;  // mean chunk-0 list length from which k_tile_sort_big sorts chunk 0
constexpr uint32_t kTsHugeMean = 3000;  // ... and k_tile_sort_huge

enum CompositeMode { kCompSingle = 0, kCompFirst = 1, kCompSecond = 2 };

struct CompositeParams {
    const uint2* ranges;          // [n_tiles] (begin, end) into tvals
    const uint32_t* tvals;        // composite slots
    const float4* rec;            // composite records (3 float4 per slot)
    const uint32_t* order;        // nullable: tile order (k_tile_sort); identity when null
    int W, H, tiles_x, tile_row_begin, row0;  // row0 = first image row of the output buffer
    int n_tiles;
    float t_min;
    int mode;                     // CompositeMode
    float4* state;                // per pixel (rgb, T or dst.a) of unsaturated tiles, image rows
    uint8_t* done;                // per tile: 1 = saturated after chunk 0
    FrameCtl* ctl;
    StatShard* stats;             // saturation statistics (shard tile % kStatShards)
    uint32_t sat_base;            // sat_bucket's base
    void* out;                    // rows_padded x W pixels
    int out_f16;
    // the tiles chunk 0 leaves unsaturated: appended by the first pass (kCompFirst, position = its
    // FrameCtl::not_done ticket) and walked by chunk 1's per-tile sort and composite (kCompSecond)
    uint32_t* c1tiles;
    int seg;                      // wave pairs per tile (the list split, composite_tile's SEG): 1, 2 or 4
    // row bands per wave (composite_tile's BANDS): 2 (8x8 quarters) or 4 (8x4 bands: a splat
    // costs a step of the bands it reaches only; more list-building per entry).  The image does
    // not depend on it (a pixel sees its list in order; a splat left off its band's list adds
    // exactly zero).  4 for frames whose tiles mostly do not saturate (small faint splats, every
    // entry walked: the sparse scene's composite 482 -> 457 us), 2 otherwise (bench frame +2.5 %)
    int bands;
    uint32_t* tile_sat;           // nullable: [abs tile] the tile's saturation key (kSentinel: none),
                                  // for the next frame's per-tile cut (ProjParams::tile_sat)
    // kCompFirst (nullable): the tiles left unsaturated, one bit each (ProjParams::umask), for
    // chunk 1's rectangle tests
    uint32_t* umask;
    uint32_t umask_w;
};
// Wave pairs per tile for a chunk-0 composite of n_tiles tiles on `cus` CUs (gs_opts.list_split):
// as many as keep every tile resident at once (a SEG-pair workgroup stages SEG x 14.5 KB in LDS:
// 10 / 5 / 2 workgroups per CU for 1 / 2 / 4 pairs), 1 when the frame fills the device anyway.
__host__ __device__ inline int composite_seg(int n_tiles, int cus) {
    if (n_tiles <= 2 * cus) return 4;
    if (n_tiles <= 5 * cus) return 2;
    return 1;
}

struct Chunk1Params {
    ProjParams pp;                // chunk-1 slots (pp.umask = the unsaturated tiles)
    BinParams bp;                 // chunk 1
    TileSortParams tp;
    CompositeParams cp;           // mode kCompSecond
    uint32_t* bar;                // grid-barrier arrival counter, zero at launch (the frame's end zeroes it)
    uint64_t spin_ticks;          // grid-barrier timeout in wall-clock ticks
    int two_chunks;               // chunk 1 may have work (else only the frame's end runs)
    // the frame's end (frame_end_body): statistics shards, pinned-slot copy, sequence number
    StatShard* stats;
    FrameCtl* host_ctl;
    uint32_t* host_seq;
    uint32_t seq;
    int cus;                      // the device's CUs (grids that stride chunk 1's compact tile list)
};
// Words per strip tile row of the unsaturated-tile bits (ProjParams::umask).
__host__ __device__ inline uint32_t umask_words(int tiles_x) { return (uint32_t)(tiles_x + 31) / 32u; }
constexpr uint32_t kUmaskLdsWords = 4096;  // chunk 1's launches test rectangles against an LDS copy up to this size

// launchers (gs_kernels.hip)
void launch_bbox(const uint8_t* aos, uint64_t n, uint32_t rb, uint32_t* bbox, hipStream_t s);
void launch_morton(const uint8_t* aos, uint64_t n, uint32_t rb, const uint32_t* bbox, uint32_t* keys,
                   uint32_t* vals, hipStream_t s);
void launch_transpose(const uint8_t* aos, uint64_t n, int n_sh, const uint32_t* perm, float4* geo, float4* shade,
                      float4* cull, uint32_t* orig, hipStream_t s);
void launch_part_bounds(const float4* cull, uint64_t n, PartBound* out, hipStream_t s);
void launch_block_bounds(const float4* cull, uint64_t n, PartBound* out, hipStream_t s);
// ref_quirks (src/renderer.ts:306): the init-sort pass's (key, value) slots and the draw-ordered
// scene copy (see k_quirk_keys / k_quirk_gather)
void launch_inverse(const uint32_t* orig, uint64_t n, uint32_t* inv, hipStream_t s);
void launch_quirk_keys(const float4* cull, const uint32_t* orig, uint32_t n, uint32_t nk, float4 vrow,
                       const uint32_t* qk, const uint32_t* qv, uint32_t* keys, uint32_t* vals, hipStream_t s);
void launch_quirk_gather(const uint32_t* skeys, const uint32_t* svals, const uint32_t* inv, uint32_t n, uint32_t nk,
                         uint32_t shq, const float4* geo, const float4* shade, const float4* cull, float4* dgeo,
                         float4* dshade, float4* dcull, uint32_t* dorig, uint32_t* qk, uint32_t* qv, hipStream_t s);
void launch_project(const ProjParams& p, hipStream_t s);
// seeded frames, before launch_project: the coarse alpha-mass histogram, then the threshold
void launch_seed(const ProjParams& p, hipStream_t s);
void launch_records(const ProjParams& p, hipStream_t s);  // chunk-1 slots (or, rec_all, every record)
void launch_sort_pass(const SortPass& p, hipStream_t s);
void launch_bin(const BinParams& p, hipStream_t s);    // count, tile scan, emit, wide rows
// stats -> host slot + seq; then FrameCtl zeroed for the next frame
// chunk 1 in one launch (grid: one workgroup per CU; returns at once when chunk 0 saturated every tile)
struct Chunk1Params;
void launch_chunk1(const Chunk1Params& c, int grid, int accum_fp16, hipStream_t s);
// k_chunk1 workgroups (256 threads) resident per CU on this device (0: query failed)
int chunk1_occupancy();
// k_chunk1's grid for `occupancy` workgroups per CU on `cus` CUs: at most 64 and at most what
// fits the device at once (co-residency of the grid barrier); 0 when nothing fits
__host__ __device__ inline int chunk1_grid(int occupancy, int cus) {
    if (occupancy <= 0 || cus <= 0) return 0;
    const long fit = (long)occupancy * cus;  // workgroups the device holds at once
    long g = fit < 64 ? fit : 64;
    if (g > cus) g = cus;  // one per CU at most: it is LDS-heavy and starts beside the next frame's kernels
    return (int)g;
}
// the same as separate launches (for frames expected to leave tiles unsaturated), then the frame's end
void launch_chunk1_split(const Chunk1Params& c, int accum_fp16, hipStream_t s);
void launch_tile_sort(const TileSortParams& p, hipStream_t s);
// ts (nullable): chunk 0's per-tile sort in the composite's launch (composite_sorts)
void launch_composite(const CompositeParams& p, int accum_fp16, hipStream_t s, const TileSortParams* ts = nullptr);
// Does launch_composite sort the tiles itself: one wave pair per tile, frames past the
// quarter-kernel size, chunk-0 lists of the 128-thread sort's shape or of the 256-thread one (the
// composite sorts those with 128 threads too: the sparse scene's lists of ~900 entries, 1036 ->
// 1059-1061 fps), not the huge shape's thousands
int composite_quarter_tiles();
inline bool composite_sorts(const TileSortParams& tp, const CompositeParams& cp) {
    return tp.big <= 1 && cp.seg <= 1 && cp.n_tiles > composite_quarter_tiles() && (cp.bands == 2 || cp.bands == 4);
}
void launch_present(const void* in, int in_f16, int W, int H, int out_kind, void* out, hipStream_t s);

__host__ __device__ inline uint32_t sort_parts(uint64_t n) { return (uint32_t)((n + kSortTile - 1) / kSortTile); }
__host__ __device__ inline uint32_t sort_parts(uint64_t n, int ipt) {
    const uint64_t t = (uint64_t)kSortThreads * (uint64_t)ipt;
    return (uint32_t)((n + t - 1) / t);
}
__host__ __device__ inline uint32_t bin_bands(uint32_t n_tiles, uint32_t band_tiles) {
    return (n_tiles + band_tiles - 1) / band_tiles;
}

}  // namespace gs
