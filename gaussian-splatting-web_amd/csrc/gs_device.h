// gs_device.h — shared constants and kernel-launch entry points (host side of gs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gs {

constexpr int kTile = 16;             // 16x16-pixel composite tile
constexpr int kProjThreads = 256;
constexpr int kSortThreads = 256;     // 4 waves
constexpr int kSortIPT = 16;          // items per thread
constexpr int kSortTile = kSortThreads * kSortIPT;  // 4096 elements per Onesweep partition
constexpr int kBinThreads = 256;
constexpr int kBinIPT = 8;
constexpr int kBinTile = kBinThreads * kBinIPT;     // 2048 ranks per binning partition
constexpr int kHistShards = 8;        // global histograms sharded by blockIdx % 8 (XCD group)
constexpr int kRadixBins = 256;
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // key of a culled Gaussian (no visible splat has it)
constexpr int kRecFloats = 16;        // 64-B projected record

// Device-side error word bits (ctx->d_err); a nonzero word fails the frame.
constexpr uint32_t kErrSpinSort = 1u, kErrSpinBin = 2u, kErrOverflow = 4u;

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
    float4* rec;              // [n][4]: projected records
    uint32_t* hist;           // [kHistShards][4][256] depth-key digit histograms (zeroed)
    unsigned long long* counters;  // [0] = n_vis, [1] = K (sum of tile counts)
};

struct SortPass {
    const uint32_t* keys_in;
    const uint32_t* vals_in;  // nullptr: values are the element index (first depth pass)
    uint32_t* keys_out;
    uint32_t* vals_out;       // may be nullptr? no: always written
    uint32_t n;               // elements read
    int shift;
    uint32_t mask;            // digit mask (<= 255)
    int filter_sentinel;      // 1: drop keys == kSentinel (they carry no digit)
    const uint32_t* hist;     // [kHistShards][npass][256] slice base for this pass, stride hist_stride
    int hist_stride;          // elements between shards
    uint32_t* status;         // [parts][256] look-back words (zeroed)
    uint32_t* ticket;         // partition ticket counter (zeroed)
    uint32_t* err;
};

struct BinParams {
    const uint32_t* sorted_vals;  // [n_vis] Gaussian index in depth order
    const float4* rec;
    uint32_t n_vis;
    int tile_row_begin, tiles_x;
    uint64_t capacity;            // entry capacity of out arrays
    uint32_t* tkeys;              // out: strip-relative tile id
    uint32_t* tvals;              // out: Gaussian index
    uint32_t* hist;               // [kHistShards][2][256] tile-id digit histograms (zeroed)
    unsigned long long* status;   // [parts] look-back words (zeroed)
    uint32_t* ticket;
    uint32_t* err;
};

struct CompositeParams {
    const uint2* ranges;          // [n_tiles] (begin, end) into tvals
    const uint32_t* tvals;
    const float4* rec;
    int W, H, tiles_x, tile_row_begin, row0;  // row0 = first image row of the output buffer
    int n_tiles;
    float t_min;
    void* out;                    // rows_padded x W pixels
    int out_f16;
};

// launchers (gs_kernels.hip)
void launch_transpose(const uint8_t* aos, uint64_t n, int n_sh, float* planes, uint64_t stride,
                      hipStream_t s);
void launch_project(const ProjParams& p, int grid, hipStream_t s);
void launch_hist_keys(const uint32_t* keys, uint32_t n, int begin_bit, int end_bit, int npass,
                      uint32_t* hist, hipStream_t s);
void launch_sort_pass(const SortPass& p, hipStream_t s);
void launch_bin(const BinParams& p, hipStream_t s);
void launch_ranges(const uint32_t* tkeys, uint64_t k, uint2* ranges, hipStream_t s);
void launch_composite(const CompositeParams& p, int accum_fp16, hipStream_t s);

inline uint32_t sort_parts(uint64_t n) { return (uint32_t)((n + kSortTile - 1) / kSortTile); }
inline uint32_t bin_parts(uint64_t n) { return (uint32_t)((n + kBinTile - 1) / kBinTile); }

}  // namespace gs
