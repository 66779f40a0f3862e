// gs_device.h — shared constants, the device-side frame control block, kernel parameter blocks
// and launchers (host side of gs_kernels.hip).
//
// A frame is a fixed sequence of launches with no host round trip: every count that depends on
// the data (visible splats, entries per chunk, unsaturated tiles) lives in FrameCtl on the device
// and every kernel sizes its work from it (grid-stride loops over a worst-case grid).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gs {

constexpr int kTile = 16;             // 16x16-pixel composite tile
constexpr int kProjThreads = 256;
constexpr int kSortThreads = 256;     // 4 waves
constexpr int kSortIPT = 16;          // items per thread
constexpr int kSortTile = kSortThreads * kSortIPT;  // 4096 elements per radix partition
constexpr int kBinThreads = 256;
constexpr int kBinIPT = 8;
constexpr int kBinTile = kBinThreads * kBinIPT;     // 2048 ranks per binning partition
constexpr int kHistShards = 8;        // global histograms sharded by blockIdx % 8 (XCD group)
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // key of a culled Gaussian (no visible splat has it)
constexpr int kRecFloats = 16;        // 64-B projected record
constexpr int kMaxGrid = 2048;        // persistent grids: 8 workgroups per CU
constexpr uint32_t kMinChunk0 = 65536;  // smallest first chunk (depth ranks)

// Packed tile rectangle carried through the depth sort (32 bits): tx0[0:12) ty0[12:24)
// (w-1)[24:28) (h-1)[28:32).  Rectangles wider or taller than 16 tiles use kRectLarge (the
// binning reads the full rectangle from the record); kRectEmpty = visible but binds no tile.
constexpr uint32_t kRectLarge = 0xFFFFFFFFu;
constexpr uint32_t kRectEmpty = 0xFFFFFFFEu;

// Device-side error bits (FrameCtl::err); a nonzero word fails the frame.
constexpr uint32_t kErrOverflow = 1u;

struct FrameCtl {                 // zeroed at the start of every frame
    unsigned long long k_total;   // sum of tile counts over visible splats (project)
    uint32_t n_vis;               // splats reaching the sort (project)
    uint32_t k_chunk[2];          // (tile, splat) entries per chunk (binning scan)
    uint32_t not_done;            // tiles still accepting splats after chunk 0
    uint32_t err;
    uint32_t pad[9];
};

struct ProjParams {
    const float* planes;      // SoA planes, plane p at planes + p * plane_stride
    uint64_t plane_stride;
    uint32_t n;
    int n_sh;
    float V[16];              // view, column-major
    float PV[16];             // proj * view (host-computed in the reference's order)
    float cam[3];
    float scale_mod;
    float P00, P11;
    int W, H;
    int tile_row_begin, tile_row_end, tiles_x;
    uint32_t* keys_out;       // [n]: depth key or kSentinel
    uint32_t* rect_out;       // [n]: packed tile rectangle
    float4* rec;              // [n][4]: projected records
    FrameCtl* ctl;
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
    uint32_t parts_max;       // sort_parts(upper bound): stride of `offsets`, grid bound
    int shift;
    uint32_t mask;            // digit mask (<= 255)
    int filter_sentinel;      // 1: drop keys == kSentinel (they carry no digit)
    uint32_t* hist;           // [kHistShards][256] digit histogram of this pass (zeroed; the
                              // upsweep accumulates it, the scan turns it into digit bases)
    uint32_t* offsets;        // [256][parts_max] scratch: partition counts, then offsets
};

struct BinParams {
    const uint32_t* sorted_vals;  // [n_vis] Gaussian index in depth order
    const uint32_t* sorted_rect;  // [n_vis] packed tile rectangle in depth order
    const float4* rec;            // records (full rectangle of kRectLarge splats)
    const uint8_t* done;          // chunk 1: per-tile "saturated after chunk 0"
    FrameCtl* ctl;
    int chunk;                    // 0 or 1
    float chunk_f;                // chunk 0 = ceil(chunk_f * n_vis) depth ranks (>= kMinChunk0);
                                  // >= 1: chunk 0 takes every rank
    int tile_row_begin, tiles_x;
    uint32_t n_max;               // upper bound of n_vis (grid / scratch sizing)
    uint32_t capacity;            // entry capacity of out arrays
    uint32_t* part_tot;           // [bin_parts(n_max) + 1] scratch
    uint32_t* tkeys;              // out: strip-relative tile id
    uint32_t* tvals;              // out: Gaussian index
};

enum CompositeMode { kCompSingle = 0, kCompFirst = 1, kCompSecond = 2 };

struct CompositeParams {
    const uint2* ranges;          // [n_tiles] (begin, end) into tvals
    const uint32_t* tvals;
    const float4* rec;
    int W, H, tiles_x, tile_row_begin, row0;  // row0 = first image row of the output buffer
    int n_tiles;
    float t_min;
    int mode;                     // CompositeMode
    float4* state;                // per pixel (rgb, T or dst.a) of unsaturated tiles, image rows
    uint8_t* done;                // per tile: 1 = saturated after chunk 0
    FrameCtl* ctl;
    void* out;                    // rows_padded x W pixels
    int out_f16;
};

// launchers (gs_kernels.hip)
void launch_transpose(const uint8_t* aos, uint64_t n, int n_sh, float* planes, uint64_t stride,
                      hipStream_t s);
void launch_project(const ProjParams& p, hipStream_t s);
void launch_sort_pass(const SortPass& p, hipStream_t s);
void launch_bin(const BinParams& p, hipStream_t s);
void launch_ranges(const uint32_t* tkeys, const uint32_t* k_dev, uint32_t k_max, uint2* ranges,
                   hipStream_t s);
void launch_composite(const CompositeParams& p, int accum_fp16, hipStream_t s);

__host__ __device__ inline uint32_t sort_parts(uint64_t n) { return (uint32_t)((n + kSortTile - 1) / kSortTile); }
__host__ __device__ inline uint32_t bin_parts(uint64_t n) { return (uint32_t)((n + kBinTile - 1) / kBinTile); }

}  // namespace gs
