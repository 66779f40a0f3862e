// gs_kernels.hip — CDNA4 (gfx950) kernels of the splat forward path.
//
// Upload (once per scene): k_bbox, k_morton, a device radix sort (k_radix_*), k_transpose (the
// reference AoS record, src/ply.ts:249-257 -> geometry records, packed SH, cull planes, Morton
// storage order), k_part_bounds.
// Per frame (9 launches, no host round trip):
//   k_part_list   per 1024-Gaussian partition (one lane each): bound test -> list of partitions
//   k_cull        per listed partition: per Gaussian the depth key (src/shaders.ts:36-68) and a
//                 conservative cull; chunk-0 candidates + work units
//   k_project     per candidate: vs_points (src/simple_render.ts:217-332) and the SH colour
//                 (:26-66), the composite slot record, sort key and packed tile rectangle
//                 (geometry and SH staged through LDS in coalesced 1-KiB pieces)
//   k_bin_count / k_bin_colscan / k_bin_emit   two-level counting sort of (tile, slot) entries
//   k_tile_sort   per tile: its slots by (depth key, reference index) = the reference's stable
//                 depth sort (src/renderer.ts:175-183) restricted to the tile
//   k_composite   16x16 tile: front-to-back "under" blending of fs_main's alpha
//                 (src/simple_render.ts:169-200, blend state :455-471), batches staged in LDS
//                 (k_composite_ts: a still camera's frames sort each tile in the composite's launch)
//   k_chunk1      chunk 1 (tiles chunk 0 left unsaturated) as one launch of 64 co-resident
//                 workgroups with grid barriers (a plain launch: one 256-thread workgroup per CU
//                 at most, so the grid always fits beside the other kernels), then the frame's
//                 end (statistics shards -> FrameCtl -> pinned host slot); or, after frames that
//                 left tiles unsaturated and under a moving camera, as separate launches
//                 (k_c1_parts, k_c1_records, binning, k_c1_tiles, k_frame_end)
//
// Inter-workgroup hand-offs (the grid barrier) follow cdna_hip_programming.md Guideline 16:
// agent-scope release / acquire, bounded spins, counters zeroed by the frame's end.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <type_traits>
#include <vector>

#include "gs_device.h"

namespace gs {
namespace {

constexpr float kSqrtLog2e = 1.2011224087864498f;  // sqrt(log2(e))

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint64_t lanemask_lt() {
    return (1ull << lane_id()) - 1ull;
}

// float_to_sortable_uint, src/shaders.ts:36-40 (negative f -> bits ^ 0x80000001).
__device__ __forceinline__ uint32_t sortable_key(float f) {
    const uint32_t fu = __float_as_uint(f);
    const uint32_t mask = (uint32_t)(-((int32_t)fu >> 31)) | 0x80000000u;
    return fu ^ mask;
}

// Inclusive wave scan (64 lanes).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, 64);
        if ((int)lane_id() >= d) v += t;
    }
    return v;
}

// Exclusive scan over an NT-thread block; returns exclusive prefix, *total = block sum.
// `tmp` = NT / 64 words of LDS.  Contains __syncthreads() (wave barriers at NT = 64).
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* tmp, uint32_t* total) {
    const uint32_t incl = wave_incl_scan(v);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 63) tmp[w] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) base += tmp[i];
        tot += tmp[i];
    }
    *total = tot;
    __syncthreads();
    return base + incl - v;
}
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* tmp, uint32_t* total) {
    return block_excl_scan<256>(v, tmp, total);
}

// ============================================================================ scene upload
// The scene is stored in spatial (Morton) order: k_bbox + k_morton give every record a 30-bit
// Morton code of its position in the scene's box (non-finite positions last), a stable radix
// sort orders them, k_transpose writes storage slot s from record perm[s] and keeps orig[s] =
// perm[s] (the reference's index: ties in depth are broken by it).  k_part_bounds then bounds
// each projection partition (kProjTile consecutive slots) for the per-partition cull.

// ordered-uint encoding of a float (monotone), for min / max with integer atomics
#ifdef GS_KTIME
// diagnostics builds only: per-workgroup wall-clock stamps of the projection kernels
// (kernel k: 0 k_cull, 1 k_project; stamp 0 entry, 1 after the first dependent loads, 2 exit | items << 40)
__device__ unsigned long long g_kt[2][8192][6];
#define KT_MARK(kk_, ii_, xx_) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_kt[kk_][blockIdx.x][ii_] = (wall_clock64() & 0xffffffffffull) | ((unsigned long long)(xx_) << 40); } while (0)
__device__ unsigned long long g_fe[8];  // the frame's end: wall clock at its steps (lane 0 of block 0)
#define FE_MARK(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_fe[k] = wall_clock64(); } while (0)
#else
#define FE_MARK(k) do { } while (0)
#define KT_MARK(kk_, ii_, xx_) do { } while (0)
#endif
__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// bbox[0..2] = min, bbox[3..5] = max of the finite positions (ordered uints; bbox[0..2] start at
// ~0, bbox[3..5] at 0)
__global__ __launch_bounds__(256) void k_bbox(const uint8_t* __restrict__ aos, uint64_t n, uint32_t rb,
                                              uint32_t* __restrict__ bbox) {
    __shared__ uint32_t s[6];
    if (threadIdx.x < 6) s[threadIdx.x] = threadIdx.x < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    uint32_t lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, hi[3] = {0u, 0u, 0u};
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const float* r = (const float*)(aos + i * rb);
        const float x = r[0], y = r[1], z = r[2];
        if (!(isfinite(x) && isfinite(y) && isfinite(z))) continue;
        const float v[3] = {x, y, z};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = min(lo[k], f2ord(v[k]));
            hi[k] = max(hi[k], f2ord(v[k]));
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        atomicMin(&s[k], lo[k]);
        atomicMax(&s[3 + k], hi[k]);
    }
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&bbox[threadIdx.x], s[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&bbox[threadIdx.x], s[threadIdx.x]);
}

__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(256) void k_morton(const uint8_t* __restrict__ aos, uint64_t n, uint32_t rb,
                                                const uint32_t* __restrict__ bbox, uint32_t* __restrict__ keys,
                                                uint32_t* __restrict__ vals) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* r = (const float*)(aos + i * rb);
    uint32_t code = 0xFFFFFFFFu;  // non-finite positions last (never visible)
    if (isfinite(r[0]) && isfinite(r[1]) && isfinite(r[2])) {
        code = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float lo = ord2f(bbox[k]), hi = ord2f(bbox[3 + k]);
            const float ext = hi - lo;
            float t = ext > 0.0f ? (r[k] - lo) / ext : 0.0f;
            t = fminf(fmaxf(t, 0.0f), 1.0f);
            code |= spread3(min((uint32_t)(t * 1024.0f), 1023u)) << (2 - k);
        }
    }
    keys[i] = code;
    vals[i] = (uint32_t)i;
}

// Storage slot i from reference record perm[i] (or i): geometry record, cull plane, shading block.
// sigmoid (src/simple_render.ts:118-125), as the projection evaluates it
__device__ __forceinline__ float sigmoid_ref(float logit) {
    if (logit >= 0.0f) return 1.0f / (1.0f + expf(-logit));
    const float e = expf(logit);
    return e / (1.0f + e);
}

__global__ __launch_bounds__(256) void k_transpose(const uint8_t* __restrict__ aos, uint64_t n,
                                                   int n_sh, const uint32_t* __restrict__ perm,
                                                   float4* __restrict__ geo, float4* __restrict__ shade,
                                                   float4* __restrict__ cull, uint32_t* __restrict__ orig) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t src = perm ? perm[i] : i;
    orig[i] = (uint32_t)src;
    const float* r = (const float*)(aos + src * (uint64_t)(64 + 16 * n_sh));
    // src/ply.ts:249-257 record: pos[0:3] | scale[4:7] | rot[8:12] | opacity[12] | sh[k] at 16+4k
    geo[3 * i + 0] = make_float4(r[0], r[1], r[2], r[12]);  // position, opacity logit
    geo[3 * i + 1] = make_float4(r[4], r[5], r[6], r[8]);   // scale, rot.x
    geo[3 * i + 2] = make_float4(r[9], r[10], r[11], 0.0f); // rot.y, rot.z, rot.w
    {  // cull plane: position and ||R(q) diag(s)||_F^2 (k_project's conservative bound)
        const float qx = r[8], qy = r[9], qz = r[10], qw = r[11];
        const float r00 = 1.0f - 2.0f * (qy * qy + qz * qz), r01 = 2.0f * (qx * qy - qw * qz),
                    r02 = 2.0f * (qx * qz + qw * qy), r10 = 2.0f * (qx * qy + qw * qz),
                    r11 = 1.0f - 2.0f * (qx * qx + qz * qz), r12 = 2.0f * (qy * qz - qw * qx),
                    r20 = 2.0f * (qx * qz - qw * qy), r21 = 2.0f * (qy * qz + qw * qx),
                    r22 = 1.0f - 2.0f * (qx * qx + qy * qy);
        const float t = (r00 * r00 + r10 * r10 + r20 * r20) * r[4] * r[4] +
                        (r01 * r01 + r11 * r11 + r21 * r21) * r[5] * r[5] +
                        (r02 * r02 + r12 * r12 + r22 * r22) * r[6] * r[6];
        // a Gaussian whose opacity is below 1/255 (or NaN) is never visible (every fragment's
        // alpha <= op is discarded, src/simple_render.ts:169-200; project_core's op test): its
        // cull plane is marked (w = -1) and every cull rejects it before loading more (a faint
        // scene: logit ~ N(-4, 2) has 22 % of them)
        const bool faint = !(sigmoid_ref(r[12]) >= 1.0f / 255.0f);
        cull[i] = make_float4(r[0], r[1], r[2], faint ? kCullFaint : t * 1.0001f);
    }
    const uint32_t q = sh_quads(n_sh);  // SH coefficients sh[k][c] at 3k + c, packed
    float v[4 * 12];
#pragma unroll
    for (int t = 0; t < 4 * 12; ++t) v[t] = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < n_sh)
#pragma unroll
            for (int c = 0; c < 3; ++c) v[3 * k + c] = r[16 + 4 * k + c];
    float4* o = shade + i * q;
#pragma unroll
    for (uint32_t t = 0; t < 12; ++t)
        if (t < q) o[t] = make_float4(v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]);
}

// Per block of kCullBlock (64) consecutive storage slots, one wave each: the same bound as
// k_part_bounds' (box of the finite positions, largest ||R(q) diag(s)||_F^2, finite count).  The
// partition bound decides whether a partition is visited at all; inside a visited partition a
// wave tests its block's bound before loading its 64 cull planes (a strip's partitions straddle
// its edges, chunk 1's partitions reach an unsaturated tile with a few of their blocks).
__global__ __launch_bounds__(256) void k_block_bounds(const float4* __restrict__ cull, uint64_t n,
                                                      PartBound* __restrict__ out) {
    const uint64_t blk = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t i = blk * kCullBlock + (threadIdx.x & 63);
    if (blk * kCullBlock >= n) return;
    uint32_t lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, hi[3] = {0u, 0u, 0u}, trs = 0u, fin = 0u;
    if (i < n) {
        const float4 c = cull[i];
        if (isfinite(c.x) && isfinite(c.y) && isfinite(c.z) && !(c.w < 0.0f)) {  // (kCullFaint)
            const float v[3] = {c.x, c.y, c.z};
#pragma unroll
            for (int d = 0; d < 3; ++d) lo[d] = hi[d] = f2ord(v[d]);
            trs = f2ord(c.w != c.w ? INFINITY : c.w);
            fin = 1;
        }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = min(lo[d], (uint32_t)__shfl_xor((int)lo[d], s, 64));
            hi[d] = max(hi[d], (uint32_t)__shfl_xor((int)hi[d], s, 64));
        }
        trs = max(trs, (uint32_t)__shfl_xor((int)trs, s, 64));
        fin += (uint32_t)__shfl_xor((int)fin, s, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        PartBound b;
        for (int d = 0; d < 3; ++d) {
            b.lo[d] = ord2f(lo[d]);
            b.hi[d] = ord2f(hi[d]);
        }
        b.trs = fin ? ord2f(trs) : 0.0f;
        b.nfin = fin;
        out[blk] = b;
    }
}

// Per projection partition (kProjTile consecutive storage slots): the box of its finite
// positions, the largest ||R(q) diag(s)||_F^2 (NaN counts as infinite) and its count of finite
// positions (zero: nothing in it can be visible).
__global__ __launch_bounds__(256) void k_part_bounds(const float4* __restrict__ cull, uint64_t n,
                                                     PartBound* __restrict__ out) {
    __shared__ uint32_t s[8];
    if (threadIdx.x < 8) s[threadIdx.x] = threadIdx.x < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    const uint64_t p0 = (uint64_t)blockIdx.x * kProjTile;
    uint32_t lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, hi[3] = {0u, 0u, 0u}, trs = 0u, fin = 0u;
    for (uint32_t k = threadIdx.x; k < (uint32_t)kProjTile; k += 256) {
        const uint64_t i = p0 + k;
        if (i >= n) break;
        const float4 c = cull[i];
        if (!(isfinite(c.x) && isfinite(c.y) && isfinite(c.z)) || c.w < 0.0f) continue;  // (kCullFaint)
        const float v[3] = {c.x, c.y, c.z};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = min(lo[d], f2ord(v[d]));
            hi[d] = max(hi[d], f2ord(v[d]));
        }
        trs = max(trs, f2ord(c.w != c.w ? INFINITY : c.w));
        ++fin;
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        atomicMin(&s[d], lo[d]);
        atomicMax(&s[3 + d], hi[d]);
    }
    atomicMax(&s[6], trs);
    atomicAdd(&s[7], fin);
    __syncthreads();
    if (threadIdx.x == 0) {
        PartBound b;
        for (int d = 0; d < 3; ++d) {
            b.lo[d] = ord2f(s[d]);
            b.hi[d] = ord2f(s[3 + d]);
        }
        b.trs = s[7] ? ord2f(s[6]) : 0.0f;
        b.nfin = s[7];
        out[blockIdx.x] = b;
    }
}

// ============================================================================ k_project
// ---- WGSL-order projection.  Everything that decides visibility, the depth key or the
// splat footprint is evaluated in the reference's order with contraction off, so it is
// bit-identical to the oracle restatement (oracle/gs_oracle.cpp project_one).
struct m3 { float c[3][3]; };  // column-major, c[col][row]

__device__ __forceinline__ m3 m3_from9(float a0, float a1, float a2, float a3, float a4, float a5,
                                       float a6, float a7, float a8) {
    m3 m;
    m.c[0][0] = a0; m.c[0][1] = a1; m.c[0][2] = a2;
    m.c[1][0] = a3; m.c[1][1] = a4; m.c[1][2] = a5;
    m.c[2][0] = a6; m.c[2][1] = a7; m.c[2][2] = a8;
    return m;
}
__device__ __forceinline__ m3 m3_mul(const m3& A, const m3& B) {
#pragma clang fp contract(off)
    m3 R;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i)
            R.c[j][i] = (A.c[0][i] * B.c[j][0] + A.c[1][i] * B.c[j][1]) + A.c[2][i] * B.c[j][2];
    return R;
}
__device__ __forceinline__ m3 m3_t(const m3& A) {
    m3 R;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) R.c[j][i] = A.c[i][j];
    return R;
}

struct Footprint {
    float cx, cy, e1x, e1y, e2x, e2y;
};

// vs_points (src/simple_render.ts:228-320) up to the quad axes in framebuffer pixels.
__device__ __forceinline__ void project_footprint(const ProjParams& p, float x, float y, float z,
                                                  float sx, float sy, float sz, float qx, float qy,
                                                  float qz, float qw, float& vz, float4& clip,
                                                  Footprint& f) {
#pragma clang fp contract(off)
    // (V*[p,1]).z  (src/shaders.ts:67) and (P*V)*[p,1] (:228), v.w = 1
    vz = ((p.V[2] * x + p.V[6] * y) + p.V[10] * z) + p.V[14] * 1.0f;
    clip.x = ((p.PV[0] * x + p.PV[4] * y) + p.PV[8] * z) + p.PV[12] * 1.0f;
    clip.y = ((p.PV[1] * x + p.PV[5] * y) + p.PV[9] * z) + p.PV[13] * 1.0f;
    clip.z = ((p.PV[2] * x + p.PV[6] * y) + p.PV[10] * z) + p.PV[14] * 1.0f;
    clip.w = ((p.PV[3] * x + p.PV[7] * y) + p.PV[11] * z) + p.PV[15] * 1.0f;
    // CalcMatrixFromRotationScale (:97-117)
    const float mod = p.scale_mod;
    const m3 ms = m3_from9(sx * mod, 0.0f, 0.0f, 0.0f, sy * mod, 0.0f, 0.0f, 0.0f, sz * mod);
    const m3 mr = m3_from9(1.0f - 2.0f * (qy * qy + qz * qz), 2.0f * (qx * qy - qw * qz),
                           2.0f * (qx * qz + qw * qy), 2.0f * (qx * qy + qw * qz),
                           1.0f - 2.0f * (qx * qx + qz * qz), 2.0f * (qy * qz - qw * qx),
                           2.0f * (qx * qz - qw * qy), 2.0f * (qy * qz + qw * qx),
                           1.0f - 2.0f * (qx * qx + qy * qy));
    const m3 M = m3_mul(mr, ms);
    const m3 sig = m3_mul(M, m3_t(M));
    // cov3d * splatScale2 (= 1)
    const float c00 = sig.c[0][0] * 1.0f, c01 = sig.c[0][1] * 1.0f, c02 = sig.c[0][2] * 1.0f;
    const float c11 = sig.c[1][1] * 1.0f, c12 = sig.c[1][2] * 1.0f, c22 = sig.c[2][2] * 1.0f;
    // J's third row (with the limx/limy clamp) never reaches cov[0][0], cov[0][1], cov[1][1].
    const float focal = (float)p.W * p.P00 / 2.0f;
    const m3 J = m3_from9(focal / vz, 0.0f, 0.0f, 0.0f, focal / vz, 0.0f, 0.0f, 0.0f, 0.0f);
    const m3 W3 = m3_from9(p.V[0], p.V[1], p.V[2], p.V[4], p.V[5], p.V[6], p.V[8], p.V[9], p.V[10]);
    const m3 T = m3_mul(J, W3);
    const m3 Vrk = m3_from9(c00, c01, c02, c01, c11, c12, c02, c12, c22);
    const m3 cov = m3_mul(T, m3_mul(Vrk, m3_t(T)));
    const float d1 = cov.c[0][0] + 0.3f, d2 = cov.c[1][1] + 0.3f, off = -cov.c[0][1];
    // eigen basis (:305-314), safe_normalize_v2 (:205-216)
    const float mid = 0.5f * (d1 + d2);
    const float ra = (d1 - d2) / 2.0f;
    const float radius = sqrtf(ra * ra + off * off);
    const float l1 = mid + radius;
    const float l2m = mid - radius;
    const float l2 = l2m < 0.1f ? 0.1f : l2m;
    float nx = off, ny = l1 - d1;
    if (nx != 0.0f) nx = nx + 1e-10f;
    if (ny != 0.0f) ny = ny + 1e-10f;
    const float nl = sqrtf(nx * nx + ny * ny);
    const float dvx = nx / nl, dvy = -(ny / nl);
    const float r1 = sqrtf(2.0f * l1), r2 = sqrtf(2.0f * l2);
    // std::min / WGSL min order: NaN stays NaN (and the splat is dropped)
    const float s1 = 4096.0f < r1 ? 4096.0f : r1, s2 = 4096.0f < r2 ? 4096.0f : r2;
    // framebuffer pixels (row 0 = top): corner = c + q.x e1 + q.y e2, e = (v.x, -v.y)
    f.e1x = s1 * dvx;
    f.e1y = -(s1 * dvy);
    f.e2x = s2 * dvy;
    f.e2y = -(s2 * -dvx);
    f.cx = (clip.x / clip.w + 1.0f) * (float)p.W / 2.0f;
    f.cy = (1.0f - clip.y / clip.w) * (float)p.H / 2.0f;
}

// Pixel centres inside [c-h, c+h], clipped to columns [0, W-1] and rows [y_lo, y_hi].
__device__ __forceinline__ bool pixel_rect(float cx, float cy, float hx, float hy, int W, int y_lo,
                                           int y_hi, float& xl, float& xh, float& yl, float& yh) {
#pragma clang fp contract(off)
    xl = fmaxf(ceilf(cx - hx - 0.5f), 0.0f);
    xh = fminf(floorf(cx + hx - 0.5f), (float)(W - 1));
    yl = fmaxf(ceilf(cy - hy - 0.5f), (float)y_lo);
    yh = fminf(floorf(cy + hy - 0.5f), (float)y_hi);
    return (xl <= xh) && (yl <= yh);
}

// The same conservative cull from the Gaussian's cull plane (x, y, z, ||R(q) diag(s)||_F^2),
// written at upload: false = provably invisible in this strip.  (cx0, cy0) +- hb bounds the pixel
// centres its quad can cover.
__device__ __forceinline__ bool cull_keep_box(const ProjParams& p, float4 c, int row_lo, int row_hi, float& vz0,
                                              float& cx0, float& cy0, float& hb) {
#pragma clang fp contract(off)
    const float x = c.x, y = c.y, z = c.z;
    vz0 = ((p.V[2] * x + p.V[6] * y) + p.V[10] * z) + p.V[14] * 1.0f;  // = project_footprint's vz
    if (c.w < 0.0f) return false;  // kCullFaint: opacity below 1/255 (a NaN bound stays conservative)
    const float cw = ((p.PV[3] * x + p.PV[7] * y) + p.PV[11] * z) + p.PV[15] * 1.0f;
    const float cz = ((p.PV[2] * x + p.PV[6] * y) + p.PV[10] * z) + p.PV[14] * 1.0f;
    if (!((cw > 0.0f) && (cz >= 0.0f) && (cz <= cw))) return false;  // :230 + near/far (exact)
    const float cxc = ((p.PV[0] * x + p.PV[4] * y) + p.PV[8] * z) + p.PV[12];
    const float cyc = ((p.PV[1] * x + p.PV[5] * y) + p.PV[9] * z) + p.PV[13];
    const float a = p.focal / vz0;
    const float trs = c.w * p.scale_mod * p.scale_mod;
    hb = 4.0f * fmaxf(sqrtf(2.0f * (a * a * p.w01_spec2 * trs + 0.6f)), 0.45f) * 1.02f + 2.0f;
    cx0 = (cxc / cw + 1.0f) * (float)p.W * 0.5f;
    cy0 = (1.0f - cyc / cw) * (float)p.H * 0.5f;
    return !(cy0 + hb < (float)row_lo - 1.0f || cy0 - hb > (float)row_hi + 1.0f || cx0 + hb < -1.0f ||
             cx0 - hb > (float)p.W);
}
__device__ __forceinline__ bool cull_keep(const ProjParams& p, float4 c, int row_lo, int row_hi, float& vz0) {
    float cx0, cy0, hb;
    return cull_keep_box(p, c, row_lo, row_hi, vz0, cx0, cy0, hb);
}

// One Gaussian's projection: depth key, packed tile rect, tile count and projected record.
struct Proj {
    uint32_t key, prect, ntiles, bbx, bby;
    float4 r0, r1;
};

// Cull, footprint, depth key, tile rect and projected record of Gaussian i; false (key =
// kSentinel) when invisible.  Deterministic: records_body recomputes the same record bit for bit.
__device__ __forceinline__ bool project_core_g(const ProjParams& p, uint32_t i, const float4 g0, const float4 g1,
                                               const float4 g2, int row_lo, int row_hi, bool cull, Proj& o) {
    // no contraction anywhere in it: k_project (chunk 0), c1_records_body (chunk 1) and the debug
    // dump inline their own copies, and a splat's record and tile rect must not depend on which
    // copy projected it (the image is invariant under the chunk split; see the binning's ellipse)
#ifndef GS_PROJ_CONTRACT_FAST  // (diagnostics builds only: A/B of the contraction's cost)
#pragma clang fp contract(off)
#endif
    o.key = kSentinel;
    o.prect = kRectEmpty;
        const float x = g0.x, y = g0.y, z = g0.z;
        const float sx = g1.x, sy = g1.y, sz = g1.z;
        const float qx = g1.w, qy = g2.x, qz = g2.y, qw = g2.z;

        // Cheap conservative cull (a row strip, or off screen): bound the quad's half extent by
        //   2 (s1 + s2) <= 4 max(sqrt(2 (d1 + d2)), 0.45),  d1 + d2 = C00 + C11 + 0.6,
        //   C00 + C11 = a^2 tr(W01 Sigma W01^T) <= a^2 lambda_max(W01 W01^T) tr(Sigma),
        //   tr(Sigma) = ||R(q) diag(s mod)||_F^2,  a = focal/vz
        // (lambda1 <= trace of the PSD 2-D covariance; tr(A S) <= lambda_max(A) tr(S) for PSD
        // A, S; W01 = the rows of W3 that reach C[0:2,0:2]) and skip
        // the full projection when that box misses the strip; only provably invisible Gaussians
        // are skipped, so the visible set is unchanged (a NaN bound never culls).
        bool pre = true;
        if (cull) {
#pragma clang fp contract(off)
            // clip z, w exactly as project_footprint rounds them: the near/far test is the real one
            const float vz0 = ((p.V[2] * x + p.V[6] * y) + p.V[10] * z) + p.V[14] * 1.0f;
            const float cw = ((p.PV[3] * x + p.PV[7] * y) + p.PV[11] * z) + p.PV[15] * 1.0f;
            const float cz = ((p.PV[2] * x + p.PV[6] * y) + p.PV[10] * z) + p.PV[14] * 1.0f;
            const float cxc = ((p.PV[0] * x + p.PV[4] * y) + p.PV[8] * z) + p.PV[12];
            const float cyc = ((p.PV[1] * x + p.PV[5] * y) + p.PV[9] * z) + p.PV[13];
            const float r00 = 1.0f - 2.0f * (qy * qy + qz * qz), r01 = 2.0f * (qx * qy - qw * qz),
                        r02 = 2.0f * (qx * qz + qw * qy), r10 = 2.0f * (qx * qy + qw * qz),
                        r11 = 1.0f - 2.0f * (qx * qx + qz * qz), r12 = 2.0f * (qy * qz - qw * qx),
                        r20 = 2.0f * (qx * qz - qw * qy), r21 = 2.0f * (qy * qz + qw * qx),
                        r22 = 1.0f - 2.0f * (qx * qx + qy * qy);
            const float msx = sx * p.scale_mod, msy = sy * p.scale_mod, msz = sz * p.scale_mod;
            const float trs = (r00 * r00 + r10 * r10 + r20 * r20) * msx * msx +
                              (r01 * r01 + r11 * r11 + r21 * r21) * msy * msy +
                              (r02 * r02 + r12 * r12 + r22 * r22) * msz * msz;
            const float a = p.focal / vz0;
            const float hb = 4.0f * fmaxf(sqrtf(2.0f * (a * a * p.w01_spec2 * trs + 0.6f)), 0.45f) * 1.02f + 2.0f;
            const float cx0 = (cxc / cw + 1.0f) * (float)p.W * 0.5f;
            const float cy0 = (1.0f - cyc / cw) * (float)p.H * 0.5f;
            if (!((cw > 0.0f) && (cz >= 0.0f) && (cz <= cw)))  // :230 + near/far: dropped anyway
                pre = false;
            else if (cy0 + hb < (float)row_lo - 1.0f || cy0 - hb > (float)row_hi + 1.0f ||
                     cx0 + hb < -1.0f || cx0 - hb > (float)p.W)
                pre = false;
        }
        if (!pre) return false;
        const float logit = g0.w;

        float vz;
        float4 clip;
        Footprint f;
        project_footprint(p, x, y, z, sx, sy, sz, qx, qy, qz, qw, vz, clip, f);
        bool vis = (clip.w > 0.0f) && (clip.z >= 0.0f) && (clip.z <= clip.w);  // :230, near/far clip
        const float op = sigmoid_ref(logit);
        vis = vis && (op >= 1.0f / 255.0f);  // alpha <= op: below 1/255 every fragment is discarded
        vis = vis && isfinite(f.cx) && isfinite(f.cy) && isfinite(f.e1x) && isfinite(f.e1y) &&
              isfinite(f.e2x) && isfinite(f.e2y);
        // visible = the quad's bounding box holds a pixel centre of this strip
        float qxl, qxh, qyl, qyh;
        float qhx, qhy;
        {
#pragma clang fp contract(off)
            qhx = 2.0f * (fabsf(f.e1x) + fabsf(f.e2x));
            qhy = 2.0f * (fabsf(f.e1y) + fabsf(f.e2y));
        }
        vis = vis && pixel_rect(f.cx, f.cy, qhx, qhy, p.W, row_lo, row_hi, qxl, qxh, qyl, qyh);

        if (!vis) return false;
        {
            const uint32_t key = sortable_key(vz);
            // binning rectangle: quad box intersected with the alpha >= 1/255 disc box, widened by
            // a small margin so that float rounding can never drop a covered pixel
            const float R = sqrtf(fmaxf(logf(255.0f * op), 0.0f));
            float hx = fminf(qhx, R * sqrtf(f.e1x * f.e1x + f.e2x * f.e2x));
            float hy = fminf(qhy, R * sqrtf(f.e1y * f.e1y + f.e2y * f.e2y));
            hx = hx * 1.0001f + 0.02f;
            hy = hy * 1.0001f + 0.02f;
            float xl, xh, yl, yh;
            uint32_t ntiles = 0, bbx = 0xFFFFu, bby = 0xFFFFu;  // empty box
            if (pixel_rect(f.cx, f.cy, hx, hy, p.W, row_lo, row_hi, xl, xh, yl, yh)) {
                bbx = (uint32_t)xl | ((uint32_t)xh << 16);
                bby = (uint32_t)yl | ((uint32_t)yh << 16);
                const uint32_t tx0 = (uint32_t)xl >> 4, tx1 = (uint32_t)xh >> 4,
                               ty0 = (uint32_t)yl >> 4, ty1 = (uint32_t)yh >> 4;
                ntiles = (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
                o.prect = (tx1 - tx0 < 16 && ty1 - ty0 < 16)
                            ? (tx0 | (ty0 << 12) | ((tx1 - tx0) << 24) | ((ty1 - ty0) << 28))
                            : kRectLarge;
            }
            // projected record (colour: store_colour, for the splats whose records are stored):
            // u' = d.(e1/|e1|^2)*sqrt(log2 e), so u'^2+v'^2 = (u^2+v^2) log2 e and
            // alpha = op * exp(-(u^2+v^2)) = exp2(log2(op) - (u'^2+v'^2))
            const float k1 = kSqrtLog2e / (f.e1x * f.e1x + f.e1y * f.e1y);
            const float k2 = kSqrtLog2e / (f.e2x * f.e2x + f.e2y * f.e2y);
            o.r0 = make_float4(f.cx, f.cy, f.e1x * k1, f.e1y * k1);
            o.r1 = make_float4(f.e2x * k2, f.e2y * k2, log2f(op), __uint_as_float(bbx));
            o.key = key;
            o.ntiles = ntiles;
            o.bbx = bbx;
            o.bby = bby;
        }
        return true;
}

// project_core_g with Gaussian i's geometry record loaded here.
__device__ __forceinline__ bool project_core(const ProjParams& p, uint32_t i, int row_lo, int row_hi,
                                             bool cull, Proj& o) {
    const float4 g0 = p.geo[3 * (uint64_t)i], g1 = p.geo[3 * (uint64_t)i + 1], g2 = p.geo[3 * (uint64_t)i + 2];
    return project_core_g(p, i, g0, g1, g2, row_lo, row_hi, cull, o);
}

// SH colour of a Gaussian at (px, py, pz) from its packed coefficients sh (nq quads,
// coefficient k channel c at 3k + c), src/simple_render.ts:5-67, :321: one thread, the
// reference's expression order with contraction off (bit-identical to the oracle).
// shq[STRIDE t] = quad t of the packed coefficients (STRIDE 64: a wave's LDS staging, k_project)
template <int STRIDE = 1>
__device__ __forceinline__ float4 sh_colour(const float4* __restrict__ shq, uint32_t nq, float px, float py, float pz,
                                            const float* cam) {
#pragma clang fp contract(off)
    float f[48];
#pragma unroll
    for (uint32_t t = 0; t < 12; ++t) {
        const float4 q = t < nq ? shq[STRIDE * t] : make_float4(0.f, 0.f, 0.f, 0.f);
        f[4 * t] = q.x;
        f[4 * t + 1] = q.y;
        f[4 * t + 2] = q.z;
        f[4 * t + 3] = q.w;
    }
    const float dx = px - cam[0], dy = py - cam[1], dz = pz - cam[2];
    const float l = sqrtf(dx * dx + dy * dy + dz * dz);
    const float X = dx / l, Y = dy / l, Z = dz / l;
    const float xx = X * X, yy = Y * Y, zz = Z * Z, xy = X * Y, xz = X * Z, yz = Y * Z;
    const float C0 = 0.28209479177387814f, C1 = 0.4886025119029199f;
    const float C20 = 1.0925484305920792f, C21 = -1.0925484305920792f, C22 = 0.31539156525252005f,
                C23 = -1.0925484305920792f, C24 = 0.5462742152960396f;
    const float C30 = -0.5900435899266435f, C31 = 2.890611442640554f, C32 = -0.4570457994644658f,
                C33 = 0.3731763325901154f, C34 = -0.4570457994644658f, C35 = 1.445305721320277f,
                C36 = -0.5900435899266435f;
    float col[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* sh = f + c;  // sh[3 k] = coefficient k, channel c
        float r = C0 * sh[0];
        r = r + C1 * (-Y * sh[3] + Z * sh[6] - X * sh[9]);
        r = r + C20 * xy * sh[12] + C21 * yz * sh[15] + C22 * (2.0f * zz - xx - yy) * sh[18] +
            C23 * xz * sh[21] + C24 * (xx - yy) * sh[24];
        r = r + C30 * Y * (3.0f * xx - yy) * sh[27] + C31 * xy * Z * sh[30] +
            C32 * Y * (4.0f * zz - xx - yy) * sh[33] + C33 * Z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[36] +
            C34 * X * (4.0f * zz - xx - yy) * sh[39] + C35 * Z * (xx - yy) * sh[42] +
            C36 * X * (xx - 3.0f * yy) * sh[45];
        r = r + 0.5f;
        col[c] = fmaxf(r, 0.0f);
    }
    return make_float4(col[0], col[1], col[2], 0.0f);
}

// SH colour of storage slot j (its position from the geometry record).
__device__ __forceinline__ float4 colour_of(const ProjParams& p, uint32_t j) {
    const float4 g0 = p.geo[3 * (uint64_t)j];
    return sh_colour(p.sh + (uint64_t)j * p.shq, p.shq, g0.x, g0.y, g0.z, p.cam);
}

// Gaussian j's colour after its per-Gaussian record quads (debug dump, rec_all).
__device__ __forceinline__ void store_colour(const ProjParams& p, uint32_t j) {
    rec_r01(p.rec, j)[2] = colour_of(p, j);
}

// A visible splat's composite slot: records r0, r1 (the colour quad follows: k_colour or
// k_records), its sort key (depth key, index) and packed rect; and its per-Gaussian r2.
__device__ __forceinline__ void store_slot(const ProjParams& p, uint32_t slot, uint32_t i, uint32_t oi, const Proj& o) {
    float4* r = p.crec + 3 * (uint64_t)slot;
    r[0] = o.r0;
    r[1] = o.r1;
    p.skey[slot] = make_uint2(p.key_zero ? 0u : o.key, oi);
    p.sidx[slot] = i;
    p.srect[slot] = o.prect;
    if (o.prect == kRectLarge)  // binning reads the pixel box of a rect wider or taller than 16 tiles
        p.rec.r2[i] = make_float4(__uint_as_float(o.key), __uint_as_float(o.ntiles), __uint_as_float(o.bbx),
                                  __uint_as_float(o.bby));
}

// Every visible Gaussian's per-Gaussian record (rec_all: the debug dump gs_debug_last_records):
// the projection of k_project from the cull plane and geometry record, with its colour.
__device__ __forceinline__ void records_body(const ProjParams& p, uint32_t blk, uint32_t nblk) {
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;
    for (uint32_t i = blk * blockDim.x + threadIdx.x; i < p.n; i += nblk * blockDim.x) {
        float vz;
        Proj o;
        if (!cull_keep(p, p.cull[i], row_lo, row_hi, vz) || !project_core(p, i, row_lo, row_hi, false, o)) continue;
        float4* r = rec_r01(p.rec, i);
        r[0] = o.r0;
        r[1] = o.r1;
        p.rec.r2[i] = make_float4(__uint_as_float(o.key), __uint_as_float(o.ntiles), __uint_as_float(o.bbx),
                                  __uint_as_float(o.bby));
        store_colour(p, i);
    }
}

__global__ __launch_bounds__(256) void k_records(ProjParams p) {
    records_body(p, blockIdx.x, gridDim.x);
}

// The interval form of cull_keep over a partition's box, in float with slack far above the
// roundings of both this bound and the per-Gaussian test (1e-4 of each term's magnitude, 4 px on
// the quad bound): clip coordinates are affine (extremes at the 8 corners), the ratios x/w, y/w
// take their extremes at the corners when every corner has w > 0, the quad bound grows with
// focal / |vz| and ||R diag(s)||_F^2.  vis = false: no Gaussian of the box passes near/far;
// [kmin, kmax] bounds the depth keys in the box; `bounded`: the pixel box [xl, xh] x [yl, yh]
// (quad bound included) holds every pixel centre any quad of the box covers.
struct PartTest {
    bool vis, bounded;
    uint32_t kmin, kmax;
    float xl, xh, yl, yh;
};
__device__ PartTest part_test(const ProjParams& p, const PartBound& b) {
    PartTest t;
    t.vis = false;
    t.bounded = false;
    t.kmin = 0;
    t.kmax = kSentinel;
    t.xl = t.xh = t.yl = t.yh = 0.0f;
    if (!b.nfin) return t;
    // coefficient rows: vz (V row 2), clip x, y, z, w (PV rows 0-3), column-major matrices
    const float C[5][4] = {{p.V[2], p.V[6], p.V[10], p.V[14]},
                           {p.PV[0], p.PV[4], p.PV[8], p.PV[12]},
                           {p.PV[1], p.PV[5], p.PV[9], p.PV[13]},
                           {p.PV[2], p.PV[6], p.PV[10], p.PV[14]},
                           {p.PV[3], p.PV[7], p.PV[11], p.PV[15]}};
    float mn[5], mx[5], sl[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {  // the affine form's range over the box (per-axis extremes)
        float lo = C[k][3], hi = C[k][3], mag = fabsf(C[k][3]);
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float a0 = C[k][d] * b.lo[d], a1 = C[k][d] * b.hi[d];
            lo += fminf(a0, a1);
            hi += fmaxf(a0, a1);
            mag += fmaxf(fabsf(a0), fabsf(a1));
        }
        sl[k] = 1e-4f * mag + 1e-30f;
        mn[k] = lo - sl[k];
        mx[k] = hi + sl[k];
    }
    if (!(mx[4] > 0.0f)) return t;        // every clip w <= 0
    if (!(mx[3] >= 0.0f)) return t;       // every clip z < 0 (near)
    if (!(mn[3] <= mx[4])) return t;      // every clip z > w (far)
    t.vis = true;
    // depth keys: negative vz keys grow with |vz|, non-negative ones with vz (sortable_key); 64
    // keys of slack for the low-bit flip and rounding
    if (mx[0] < 0.0f) {
        t.kmin = sortable_key(mx[0]);
        t.kmax = sortable_key(mn[0]);
    } else {
        t.kmin = mn[0] > 0.0f ? sortable_key(mn[0]) : 0u;
        t.kmax = sortable_key(mx[0]);
    }
    t.kmin = t.kmin > 64u ? t.kmin - 64u : 0u;
    t.kmax = t.kmax < kSentinel - 64u ? t.kmax + 64u : kSentinel;
    if (!(mn[4] > 0.0f)) return t;         // a corner with w <= 0: no ratio bound
    if (!(mn[0] > 0.0f || mx[0] < 0.0f)) return t;  // vz crosses 0
    float pxl = INFINITY, pxh = -INFINITY, pyl = INFINITY, pyh = -INFINITY;
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // pixel centre of each corner
        const float x = (c & 1) ? b.hi[0] : b.lo[0], y = (c & 2) ? b.hi[1] : b.lo[1], z = (c & 4) ? b.hi[2] : b.lo[2];
        const float cx = C[1][0] * x + C[1][1] * y + C[1][2] * z + C[1][3];
        const float cy = C[2][0] * x + C[2][1] * y + C[2][2] * z + C[2][3];
        const float cw = C[4][0] * x + C[4][1] * y + C[4][2] * z + C[4][3];
        const float px = (cx / cw + 1.0f) * (float)p.W * 0.5f, py = (1.0f - cy / cw) * (float)p.H * 0.5f;
        pxl = fminf(pxl, px); pxh = fmaxf(pxh, px);
        pyl = fminf(pyl, py); pyh = fmaxf(pyh, py);
    }
    const float az = fminf(fabsf(mn[0]), fabsf(mx[0]));
    const float a = p.focal / az;
    const float trs = b.trs * p.scale_mod * p.scale_mod;
    // the corner ratios' own error: relative slack on the pixel extent plus 4 px
    const float hb = 4.0f * fmaxf(sqrtf(2.0f * (a * a * p.w01_spec2 * trs + 0.6f)), 0.45f) * 1.03f + 4.0f +
                     1e-3f * (float)max(p.W, p.H);
    if (!(hb < 1e30f)) return t;
    t.bounded = true;
    t.xl = pxl - hb;
    t.xh = pxh + hb;
    t.yl = pyl - hb;
    t.yh = pyh + hb;
    return t;
}

// The frame's chunk threshold: the host's (from earlier frames) or, in a seeded frame, the one
// k_seed_pick left in FrameCtl.
__device__ __forceinline__ uint32_t frame_thresh(const ProjParams& p) {
    return p.thresh_dev ? *p.thresh_dev : p.thresh;
}

// Can a Gaussian of partition b be a chunk-0 candidate of this frame (pass cull_keep with key <
// T)?
__device__ bool part_maybe(const ProjParams& p, const PartBound& b, int row_lo, int row_hi, uint32_t T) {
    const PartTest t = part_test(p, b);
    if (!t.vis) return false;
    if (T != kSentinel && t.kmin >= T) return false;
    if (!t.bounded) return true;
    return !(t.yh < (float)row_lo - 1.0f || t.yl > (float)row_hi + 1.0f || t.xh < -1.0f || t.xl > (float)p.W);
}

// Tiles of the strip that a pixel-centre box [xl, xh] x [yl, yh] (widened by 1 px) may touch;
// false when it misses the strip.  NaN or infinite bounds widen to the strip's edges.
__device__ __forceinline__ bool box_tiles(const ProjParams& p, float xl, float xh, float yl, float yh,
                                          uint32_t& tx0, uint32_t& ty0, uint32_t& tx1, uint32_t& ty1) {
    const float row_lo = (float)(p.tile_row_begin * kTile);
    const float row_hi = (float)(min(p.tile_row_end * kTile, p.H) - 1);
    if (yh < row_lo - 1.0f || yl > row_hi + 1.0f || xh < -1.0f || xl > (float)p.W) return false;
    const float x0 = fminf(fmaxf(xl - 1.0f, 0.0f), (float)(p.W - 1));
    const float x1 = fmaxf(fminf(xh + 1.0f, (float)(p.W - 1)), 0.0f);
    const float y0 = fminf(fmaxf(yl - 1.0f, row_lo), row_hi);
    const float y1 = fmaxf(fminf(yh + 1.0f, row_hi), row_lo);
    tx0 = (uint32_t)x0 >> 4;
    tx1 = (uint32_t)x1 >> 4;
    ty0 = (uint32_t)y0 >> 4;
    ty1 = (uint32_t)y1 >> 4;
    return tx0 <= tx1 && ty0 <= ty1;
}

// The per-tile cut at projection: a chunk-0 candidate whose key is at or past every cut bound of
// the blocks its conservative box reaches has no chunk-0 entry (binning's splat_mode would drop
// it), so it is not projected in chunk 0; chunk 1 projects it (c1_records_body) if one of those
// tiles is still unsaturated after chunk 0.  k_cull and chunk 1 evaluate this on the same inputs
// (the cull plane, the frame's block map snapshot), so a Gaussian lands in exactly one chunk.
// cutb: the block map (k_cull: its LDS copy).  Boxes of more than 16 blocks are never skipped.
__device__ __forceinline__ bool cut_skip(const ProjParams& p, const uint32_t* cutb, uint32_t key, float cx0, float cy0,
                                         float hb) {
    uint32_t tx0, ty0, tx1, ty1;
    if (!box_tiles(p, cx0 - hb, cx0 + hb, cy0 - hb, cy0 + hb, tx0, ty0, tx1, ty1)) return false;
    const uint32_t rb = (uint32_t)p.tile_row_begin, bxn = cut_blocks_x(p.tiles_x);
    const uint32_t bx0 = tx0 / kCutBlock, bx1 = tx1 / kCutBlock, by0 = (ty0 - rb) / kCutBlock, by1 = (ty1 - rb) / kCutBlock;
    if ((bx1 - bx0 + 1) * (by1 - by0 + 1) > 16) return false;
    uint32_t mx = 0;
    for (uint32_t by = by0; by <= by1; ++by)
        for (uint32_t bx = bx0; bx <= bx1; ++bx) mx = max(mx, cutb[by * bxn + bx] >> 16);
    return (key >> 16) >= mx;
}

// A wide splat's slot into the chunk's list (ProjParams::wlist): the shard of its partition,
// chunk 0 from the shard region's front, chunk 1 from its back (a partition's slots of both
// chunks fit its block, so a shard's two lists fit its region); one counter add per wave.  Every
// lane of the wave calls it, and the wave's slots lie in one partition.
__device__ __forceinline__ void wide_append(const ProjParams& p, int chunk, bool wide, uint32_t slot) {
    const uint64_t b = __ballot(wide);
    if (!b) return;
    const uint32_t lane = lane_id();
    const uint32_t sh = (uint32_t)__builtin_amdgcn_readfirstlane((int)((slot / (uint32_t)kProjTile) % kWideShards));
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&p.stats[sh].wl_n[chunk], (uint32_t)__popcll(b));
    base = __shfl(base, 0, 64);
    const uint32_t j = base + (uint32_t)__popcll(b & lanemask_lt()), cap = wide_shard_cap(proj_parts(p.n));
    if (wide) {
        if (j < cap) p.wlist[(uint64_t)sh * cap + (chunk ? cap - 1u - j : j)] = slot;
        else atomicOr(&p.ctl->err, kErrState);  // (never: a shard's partitions hold at most cap slots)
    }
}

// Does the tile rectangle [tx0, tx1] x [ty0, ty1] (strip tile rows, absolute) hold a tile chunk 0
// left unsaturated?  m: the unsaturated-tile bits (ProjParams::umask, or chunk 1's LDS copy of
// them), a word or two per row of the rectangle.
__device__ __forceinline__ bool unsat_any(const ProjParams& p, const uint32_t* m, uint32_t tx0, uint32_t ty0,
                                          uint32_t tx1, uint32_t ty1) {
    const uint32_t mw = p.umask_w, rb = (uint32_t)p.tile_row_begin, w0 = tx0 >> 5, w1 = tx1 >> 5;
    const uint32_t lo = ~0u << (tx0 & 31u), hi = ~0u >> (31u - (tx1 & 31u));
    for (uint32_t ty = ty0; ty <= ty1; ++ty) {
        const uint32_t* row = m + (ty - rb) * mw;
        if (w0 == w1) {
            if (row[w0] & lo & hi) return true;
            continue;
        }
        if ((row[w0] & lo) | (row[w1] & hi)) return true;
        for (uint32_t w = w0 + 1; w < w1; ++w)
            if (row[w]) return true;
    }
    return false;
}

// The unsaturated-tile bits into LDS (`words` of room) when they fit, else the global array;
// contains a barrier (every thread of the workgroup calls it).
__device__ __forceinline__ const uint32_t* umask_lds(const ProjParams& p, uint32_t* lds, uint32_t words) {
    const uint32_t n = (uint32_t)(p.tile_row_end - p.tile_row_begin) * p.umask_w;
    if (n > words) return p.umask;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) lds[i] = p.umask[i];
    __syncthreads();
    return lds;
}

// Can partition b hold a chunk-1 splat: a Gaussian at or past thresh whose quad may touch a tile
// chunk 0 left unsaturated?
__device__ bool part_maybe_c1(const ProjParams& p, const PartBound& b, uint32_t T, const uint32_t* um) {
    const PartTest t = part_test(p, b);
    if (!t.vis || (t.kmax < T && !p.cut)) return false;  // (with the cut, nearer splats may be chunk 1's too)
    uint32_t tx0, ty0, tx1, ty1;
    if (!t.bounded) {
        tx0 = 0;
        tx1 = (uint32_t)p.tiles_x - 1;
        ty0 = (uint32_t)p.tile_row_begin;
        ty1 = (uint32_t)p.tile_row_end - 1;
    } else if (!box_tiles(p, t.xl, t.xh, t.yl, t.yh, tx0, ty0, tx1, ty1)) {
        return false;
    }
    return unsat_any(p, um, tx0, ty0, tx1, ty1);
}

// Chunk 1, step 1: every thread of the grid tests partitions (part_maybe_c1 against the
// unsaturated-tile bits um); the ones that may hold a chunk-1 splat are appended to plist (one
// counter add per wave; list order does not matter: a partition's chunk-1 slots are its own).
// With block bounds (p.bbounds) the list holds 64-slot blocks instead of partitions: a partition
// that reaches an unsaturated tile mostly does so with a few of its 16 blocks (orbit frames list
// ~1000-2000 partitions at the scene's edge, next to ~2300 empty off-scene tiles).
__device__ __forceinline__ uint32_t c1_items(const ProjParams& p) {
    return p.bbounds ? (uint32_t)((p.n + kCullBlock - 1) / kCullBlock) : proj_parts(p.n);
}
__device__ __forceinline__ void c1_parts_body(const ProjParams& p, uint32_t blk, uint32_t nblk, const uint32_t* um) {
    const uint32_t parts = c1_items(p), lane = lane_id(), T = frame_thresh(p);
    const PartBound* bnd = p.bbounds ? p.bbounds : p.bounds;
    for (uint32_t q0 = blk * blockDim.x + (threadIdx.x & ~63u); q0 < parts; q0 += nblk * blockDim.x) {
        const uint32_t q = q0 + lane;
        const bool want = q < parts && part_maybe_c1(p, bnd[q], T, um);
        const uint64_t b = __ballot(want);
        if (!b) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&p.ctl->c1_parts, (uint32_t)__popcll(b));
        base = __shfl(base, 0, 64);
        if (want) p.plist[base + (uint32_t)__popcll(b & lanemask_lt())] = q;
    }
}

// Chunk 1, step 2: the listed partitions' Gaussians, 64 consecutive ones per wave iteration, the
// grid's waves striding over (listed partition, 64-Gaussian block) pairs (a workgroup per
// partition walked its 16 blocks four at a time: a chain of dependent loads per block, 65 us for
// ~1000 listed partitions under a moving camera).  From the cull plane, a Gaussian at or past
// thresh whose conservative box touches an unsaturated tile is projected; the visible ones whose
// rect touches one get a chunk-1 slot (slot_c1) with their record and colour.  The filter before
// project_core only skips Gaussians the exact rect test after it would reject.
__device__ __forceinline__ void c1_records_body(const ProjParams& p, uint32_t blk, uint32_t nblk, const uint32_t* um) {
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;
    const uint32_t lane = lane_id(), nl = p.ctl->c1_parts, T = frame_thresh(p);
    const uint32_t kBlocks = p.bbounds ? 1u : (uint32_t)kProjTile / 64u;  // waves per listed item
    const uint32_t wpb = blockDim.x >> 6;
    for (uint32_t v = blk * wpb + (threadIdx.x >> 6); v < nl * kBlocks; v += nblk * wpb) {
        const uint32_t i0 = p.bbounds ? p.plist[v] * (uint32_t)kCullBlock
                                      : p.plist[v / kBlocks] * (uint32_t)kProjTile + (v % kBlocks) * 64u;
        const uint32_t part = i0 / (uint32_t)kProjTile;
        {
            const uint32_t i = i0 + lane;
            bool want = false;
            float vz, cx0, cy0, hb;
            if (i < p.n && cull_keep_box(p, p.cull[i], row_lo, row_hi, vz, cx0, cy0, hb) &&
                (sortable_key(vz) >= T || (p.cut && cut_skip(p, p.cutb, sortable_key(vz), cx0, cy0, hb)))) {
                uint32_t tx0, ty0, tx1, ty1;
                want = box_tiles(p, cx0 - hb, cx0 + hb, cy0 - hb, cy0 + hb, tx0, ty0, tx1, ty1) &&
                       unsat_any(p, um, tx0, ty0, tx1, ty1);
            }
            Proj o;
            want = want && project_core(p, i, row_lo, row_hi, false, o);
            if (want) {
                const uint32_t pr = o.prect;
                want = pr != kRectEmpty;
                if (want && pr != kRectLarge) {
                    const uint32_t x0 = pr & 0xfffu, y0 = (pr >> 12) & 0xfffu;
                    want = unsat_any(p, um, x0, y0, x0 + ((pr >> 24) & 15u), y0 + (pr >> 28));
                }
            }
            const uint64_t b = __ballot(want);
            if (!b) continue;
            uint32_t base = 0;
            const uint32_t ntiles = want ? o.ntiles : 0u;
            unsigned long long kt = ntiles;
            for (int d = 32; d >= 1; d >>= 1) kt += __shfl_xor(kt, d, 64);
            if (lane == 0) {
                const uint32_t c = (uint32_t)__popcll(b);
                base = atomicAdd(&p.c1[part], c);
                StatShard* st = p.stats + (i0 >> 6) % kStatShards;
                atomicAdd(&st->n_chunk[1], c);
                atomicAdd(&st->k_total, kt);
            }
            base = __shfl(base, 0, 64);
            const uint32_t slot = slot_c1(part, base + (uint32_t)__popcll(b & lanemask_lt()));
            if (want) {
                store_slot(p, slot, i, p.orig[i], o);
                float4 c = colour_of(p, i);
                c.w = __uint_as_float(o.key);
                p.crec[3 * (uint64_t)slot + 2] = c;
            }
            if (p.wlist) wide_append(p, 1, want && o.ntiles >= p.wide_tiles, slot);
        }
    }
}

// The frame's list of non-empty chunk-0 work units (k_cull appends them, kUnitShards shards).
struct UnitList {
    const uint32_t* units;  // null: unit j is j
    uint32_t cap;
    uint32_t pre[kUnitShards + 1];
    uint32_t total;
};
// A shard count past the shard's capacity (state the frame did not write) is an error, not a
// read past the list: the frame's units are dropped and kErrState fails the frame.
__device__ __forceinline__ UnitList load_units(const uint32_t* units, FrameCtl* ctl, uint32_t parts) {
    UnitList L;
    L.units = units;
    L.cap = unit_shard_cap(parts);
    L.pre[0] = 0;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < kUnitShards; ++k) {
        const uint32_t c = ctl->unit_n[k];
        bad = bad || c > L.cap;
        L.pre[k + 1] = L.pre[k] + c;
    }
    L.total = L.pre[kUnitShards];
    if (bad) {
        if (threadIdx.x == 0) atomicOr(&ctl->err, kErrState);
        L.total = 0;
    }
    return L;
}
// A listed unit: bits [0, 20) = partition * kProjRounds + round, bits [20, 28) = its candidate
// count - 1 (so k_project and binning need no count load).  Unlisted units (chunk 1: every unit
// j of every partition) are the bare number j.
__device__ __forceinline__ uint32_t unit_id(uint32_t u) { return u & 0xFFFFFu; }
__device__ __forceinline__ uint32_t unit_count(uint32_t u) { return ((u >> 20) & 0xFFu) + 1u; }

__device__ __forceinline__ uint32_t unit_at(const UnitList& L, uint32_t j) {
    if (!L.units) return j;
    uint32_t k = 0, base = 0;  // selects, not an indexed array: no scratch round trip
#pragma unroll
    for (int t = 1; t < kUnitShards; ++t)
        if (j >= L.pre[t]) {
            k = (uint32_t)t;
            base = L.pre[t];
        }
    return L.units[(uint64_t)k * L.cap + (j - base)];
}

// Projection, phase A (one workgroup per projection partition of kProjTile storage slots; the
// partition's bound is tested first (part_maybe), a ruled-out partition costs one read): every
// Gaussian's 16-B cull plane gives its depth key (vz rounded exactly as project_footprint rounds
// it) and the conservative cull (cull_keep: exact near/far, a provable bound on the quad box
// against this frame's rows).  Survivors nearer than thresh are the partition's chunk-0
// candidates (cand: their offsets in index order; c0 = their count, the partition's chunk-0
// slots; its non-empty work units are appended to the frame's list); survivors at or past thresh
// are only counted (n_vis is exact when the frame has one chunk and no partition was ruled out
// by the threshold) and enter the depth range.
// Projection, phase 0: the partition test (part_maybe on each partition's bound), one lane per
// partition; the partitions that may hold a chunk-0 candidate are appended to plist0 (one counter
// add per wave; list order does not matter: a partition's slots and units are its own).  Every
// partition's chunk counts are zeroed here (k_cull sets c0 of the listed ones, chunk 1 adds to c1).
// A ruled-out partition costs one 32-B read and one lane, and k_cull's workgroups visit only the
// listed ones (a strip lists about an eighth of them).
// Per-tile cut bound (see kCutMaxTiles) from a tile's last saturation key: its depth scaled by
// the margin, just past it (exclusive), rounded up to the 16-bit bound cut_keep compares with.
__device__ __forceinline__ uint16_t tile_cut_bound(uint32_t sat, float margin) {
    if (sat == kSentinel) return 0xFFFFu;
    const float v = __uint_as_float((sat & 0x80000000u) ? (sat ^ 0x80000000u) : (sat ^ 0x80000001u)) * margin;
    if (!isfinite(v)) return 0xFFFFu;
    const uint32_t k = sortable_key(v);
    if (k >= 0xFFFF0000u) return 0xFFFFu;
    return (uint16_t)(((k + 1u) + 0xFFFFu) >> 16);
}

__global__ __launch_bounds__(256) void k_part_list(ProjParams p) {
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;
    const uint32_t parts = proj_parts(p.n), lane = lane_id();
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (p.cut) {  // this frame's per-tile cut bounds, a snapshot (the composites keep updating
                  // tile_sat), and their minimum and maximum per block: a thread per block
        const uint32_t tx = (uint32_t)p.tiles_x, rows = (uint32_t)(p.tile_row_end - p.tile_row_begin);
        const uint32_t base = (uint32_t)p.tile_row_begin * tx, bxn = cut_blocks_x(p.tiles_x);
        const uint32_t nb = cut_blocks(p.tiles_x, (int)rows);
        for (uint32_t b = q; b < nb; b += gridDim.x * blockDim.x) {
            const uint32_t x0 = (b % bxn) * kCutBlock, y0 = (b / bxn) * kCutBlock;
            uint32_t sat[kCutBlock][kCutBlock];  // (the block's 16 loads in flight together)
#pragma unroll
            for (int y = 0; y < kCutBlock; ++y)
#pragma unroll
                for (int x = 0; x < kCutBlock; ++x)
                    sat[y][x] = y0 + y < rows && x0 + x < tx ? p.tile_sat[base + (y0 + y) * tx + x0 + x] : 0u;
            uint32_t mn = 0xFFFFu, mx = 0u;
#pragma unroll
            for (int y = 0; y < kCutBlock; ++y)
#pragma unroll
                for (int x = 0; x < kCutBlock; ++x)
                    if (y0 + y < rows && x0 + x < tx) {
                        const uint32_t c = tile_cut_bound(sat[y][x], p.cut_margin);
                        p.cut[(y0 + y) * tx + x0 + x] = (uint16_t)c;
                        mn = min(mn, c);
                        mx = max(mx, c);
                    }
            p.cutb[b] = mn | (mx << 16);
        }
    }
    if (p.umask) {  // the unsaturated-tile bits this frame's chunk-0 composite sets
        const uint32_t nw = (uint32_t)(p.tile_row_end - p.tile_row_begin) * p.umask_w;
        for (uint32_t i = q; i < nw; i += gridDim.x * blockDim.x) p.umask[i] = 0u;
    }
    const uint32_t T = frame_thresh(p);
    if (q == 0) p.ctl->frame_T = T;
    const bool want = q < parts && part_maybe(p, p.bounds[q], row_lo, row_hi, T);
    if (q < parts) {
        p.c1[q] = 0;
        if (!want) p.c0[q] = 0;
    }
    const uint64_t b = __ballot(want);
    if (!b) return;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&p.ctl->c0_parts, (uint32_t)__popcll(b));
    base = __shfl(base, 0, 64);
    if (want) p.plist0[base + (uint32_t)__popcll(b & lanemask_lt())] = q;
}

// ---- seeded frames: a frame with no usable history (the first frame of a scene, a camera cut)
// takes its chunk threshold from a coarse estimate of where its tiles saturate, instead of running
// every visible splat as one chunk.  k_seed_hist: a sample of the scene (every seed_stride-th
// run of kSeedRun storage slots; about kSeedRunsPerCell runs per cell, as each run of Morton-ordered
// Gaussians is one small clump of the scene) through the
// exact near/far test and the conservative screen box; each kept Gaussian adds its alpha mass,
// op * 2 pi sigma^2 (sigma^2 ~ a^2 ||R diag(s)||_F^2 / 3 + 0.3, the per-axis variance of its 2-D
// footprint; the integral of op exp(-d^T C^-1 d / 2)), weighted by the stride, to the 64x64-px
// cells of its 2-sigma box at its quarter-octave depth bucket.  k_seed_pick: per cell the first
// depth bucket at which the mass per pixel reaches seed_tau (sum alpha >= -ln t_min: saturated),
// then the chunk controller's rule on those depths (the 95 % quantile of the saturating cells'
// buckets, its upper edge, depth x 1.10; one chunk when under 20 % of the cells saturate).  The
// threshold only moves work between the chunks: the image does not depend on it.
__device__ __forceinline__ float key_depth(uint32_t k) {  // the float a depth key encodes
    return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : (k ^ 0x80000001u));
}

constexpr int kSeedMaxCells = 4096;  // cell atomics per sampled Gaussian at most

__global__ __launch_bounds__(256) void k_seed_hist(ProjParams p) {
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;
    const uint32_t nrun = (p.n + kSeedRun - 1) / kSeedRun;
    const uint32_t nsr = (nrun + p.seed_stride - 1) / p.seed_stride;
    const float wgt = (float)p.seed_stride * 6.28318531f;
    constexpr uint32_t kRunsPerBlock = 256 / kSeedRun;
    const uint32_t lane = lane_id(), lead = lane & ~(uint32_t)(kSeedRun - 1);
    // (the loop runs whole waves: a sampled run is 16 lanes of one wave, reduced with shuffles)
    for (uint32_t sr0 = blockIdx.x * kRunsPerBlock; sr0 < nsr; sr0 += gridDim.x * kRunsPerBlock) {
        const uint32_t sr = sr0 + threadIdx.x / kSeedRun;
        const uint32_t i = sr * p.seed_stride * kSeedRun + threadIdx.x % kSeedRun;
        bool ok = sr < nsr && i < p.n;
        float share = 0.0f;
        int x0 = 0, x1 = -1, y0 = 0, y1 = -1, b = 0;
        if (ok) {
            const float4 c = p.cull[i];
            float vz, cx0, cy0, hb;
            ok = cull_keep_box(p, c, row_lo, row_hi, vz, cx0, cy0, hb);
            if (ok) {
                const float op = 1.0f / (1.0f + __expf(-p.geo[3 * (uint64_t)i].w));
                const float a = p.focal / vz;
                const float var = a * a * c.w * p.scale_mod * p.scale_mod * (1.0f / 3.0f) + 0.3f;
                ok = op >= 1.0f / 255.0f && var < 1e12f;
                if (ok) {
                    const float r = 2.0f * sqrtf(var);
                    const float fx0 = floorf((cx0 - r) * (1.0f / kSeedCell)), fx1 = floorf((cx0 + r) * (1.0f / kSeedCell));
                    const float fy0 = floorf((cy0 - r - (float)row_lo) * (1.0f / kSeedCell));
                    const float fy1 = floorf((cy0 + r - (float)row_lo) * (1.0f / kSeedCell));
                    share = op * var * wgt / ((fx1 - fx0 + 1.0f) * (fy1 - fy0 + 1.0f));
                    x0 = (int)fmaxf(fx0, 0.0f);
                    x1 = (int)fminf(fx1, (float)(p.seed_cx - 1));
                    y0 = (int)fmaxf(fy0, 0.0f);
                    y1 = (int)fminf(fy1, (float)(p.seed_cy - 1));
                    b = min(max((int)(sortable_key(vz) >> kSatShift) - (int)p.seed_base, 0), kSeedBuckets - 1);
                }
            }
        }
        // the run's Gaussians are neighbours (Morton order): the lanes whose cell box and depth
        // bucket equal the run leader's add their shares once, through the leader (one set of
        // atomics per run instead of one per Gaussian); the others add their own
        const uint32_t kx = ok ? ((uint32_t)x0 | ((uint32_t)x1 << 16)) : 0xFFFFFFFFu;
        const uint32_t ky = ok ? ((uint32_t)y0 | ((uint32_t)y1 << 16)) : 0xFFFFFFFFu;
        const int lx = __shfl((int)kx, (int)lead, 64), ly = __shfl((int)ky, (int)lead, 64), lb = __shfl(b, (int)lead, 64);
        const bool same = ok && (int)kx == lx && (int)ky == ly && b == lb;
        float sum = same ? share : 0.0f;
#pragma unroll
        for (int d = kSeedRun / 2; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
        const bool mine = ok && (!same || lane == lead);
        const float add = same ? sum : share;
        if (mine) {
            // every cell of the box (a 4K frame has 2040); a box of more than kSeedMaxCells cells
            // (larger frames) visits every sy-th row, each visited row taking the mass of the rows
            // it stands for, so the mass the splat adds is its whole share either way
            const int nx = x1 - x0 + 1, ny = y1 - y0 + 1;
            const int sy = max(1, (nx * ny + kSeedMaxCells - 1) / kSeedMaxCells);
            const float addr = add * (float)ny / (float)((ny + sy - 1) / sy);
            for (int y = y0; y <= y1; y += sy)
                for (int x = x0; x <= x1; ++x)
                    atomicAdd(&p.seedh[((uint64_t)y * p.seed_cx + x) * kSeedBuckets + b], addr);
        }
    }
}

__global__ __launch_bounds__(1024) void k_seed_pick(ProjParams p) {
    __shared__ uint32_t s_hist[kSeedBuckets];
    const int tid = threadIdx.x;
    if (tid < kSeedBuckets) s_hist[tid] = 0;
    __syncthreads();
    const int rows = min(p.tile_row_end * kTile, p.H) - p.tile_row_begin * kTile;
    const int cells = p.seed_cx * p.seed_cy;
    for (int q = tid; q < cells; q += 1024) {
        const int cx = q % p.seed_cx, cy = q / p.seed_cx;
        const float px = (float)(min(kSeedCell, p.W - cx * kSeedCell) * min(kSeedCell, rows - cy * kSeedCell));
        const float need = p.seed_tau * px;
        float4* h4 = (float4*)(p.seedh + (uint64_t)q * kSeedBuckets);
        float4 hv[kSeedBuckets / 4];
#pragma unroll
        for (int k = 0; k < kSeedBuckets / 4; ++k) hv[k] = h4[k];  // every load in flight at once
#pragma unroll
        for (int k = 0; k < kSeedBuckets / 4; ++k) h4[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // zero for the next seeded frame
        float cum = 0.0f;
        int sb = -1;
#pragma unroll
        for (int k = 0; k < kSeedBuckets / 4; ++k) {
            const float v[4] = {hv[k].x, hv[k].y, hv[k].z, hv[k].w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                cum += v[t];
                if (sb < 0 && cum >= need) sb = 4 * k + t;
            }
        }
        if (sb >= 0) atomicAdd(&s_hist[sb], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t sat = 0;
        for (int b = 0; b < kSeedBuckets; ++b) sat += s_hist[b];
        uint32_t T = kSentinel;
        if (cells > 0 && (float)sat >= 0.2f * (float)cells) {
            const float want = 0.95f * (float)sat;
            uint32_t cum = 0;
            int b = 0;
            for (; b < kSeedBuckets - 1; ++b) {
                cum += s_hist[b];
                if ((float)cum >= want) break;
            }
            const uint64_t e = ((uint64_t)p.seed_base + (uint64_t)b + 1) << kSatShift;
            const float v = key_depth((uint32_t)min<uint64_t>(e, 0xFFFFFFFEull)) * 1.10f;
            if (isfinite(v)) {
                const uint32_t k = sortable_key(v);
                T = k >= kSentinel - 1u ? kSentinel : k + 1u;
            }
        }
        p.ctl->seed_T = T;
    }
}

template <bool CUT>  // CUT: the frame has the per-tile cut (cut_skip; else none of its code or LDS)
__global__ __launch_bounds__(kProjThreads) void k_cull(ProjParams p) {
    __shared__ uint32_t s_vis, s_kmin_inv, s_kmax;
    __shared__ unsigned long long s_mask[kProjRounds][kProjThreads / 64];
    __shared__ uint32_t s_base[kProjRounds][kProjThreads / 64];
    __shared__ uint32_t s_total;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (tid == 0) { s_vis = 0; s_kmin_inv = 0; s_kmax = 0; }
    uint32_t my_vis = 0, my_kmin_inv = 0, my_kmax = 0;
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;
    const uint32_t parts = proj_parts(p.n), ucap = unit_shard_cap(parts);
    KT_MARK(0, 0, 0);
    uint32_t nl = p.ctl->c0_parts;  // the partitions k_part_list kept
    if (nl > parts) {  // (never: k_part_list lists each partition at most once)
        if (tid == 0) atomicOr(&p.ctl->err, kErrState);
        nl = 0;
    }
    const uint32_t T = frame_thresh(p);
    uint32_t kt_items = 0;
    // Software-pipelined over the workgroup's partitions: the next partition's cull planes are
    // loaded when this one starts (two register sets) and the list entry of the one after it, so
    // the loads are in flight while this partition is tested; the barriers wait for LDS only (a
    // __syncthreads would drain the loads too).  Slots past n read the last plane and list
    // positions past the end the last entry: no branch around a load (its zero fill would wait for it).
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    auto load_planes = [&](uint32_t part, float4 (&c)[kProjRounds]) {
        const uint32_t p0 = part * kProjTile;
#pragma unroll
        for (int it = 0; it < kProjRounds; ++it) c[it] = p.cull[min(p0 + it * kProjThreads + tid, p.n - 1u)];
    };
    // the per-tile cut's block map (cut_skip) into LDS
    __shared__ uint32_t s_cutb[CUT ? kCutMaxBlocks : 1];
    if (CUT) {
        const uint32_t nb = cut_blocks(p.tiles_x, p.tile_row_end - p.tile_row_begin);
        for (uint32_t b = tid; b < nb; b += kProjThreads) s_cutb[b] = p.cutb[b];
    }
    // the workgroup's partitions (list entries blockIdx.x + k gridDim.x) into LDS at once
    __shared__ uint32_t s_part[128];
    const uint32_t nmine = nl > blockIdx.x ? (nl - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
    for (uint32_t k = tid; k < min(nmine, 128u); k += kProjThreads) s_part[k] = p.plist0[blockIdx.x + k * gridDim.x];
    lds_barrier();
    auto part_at = [&](uint32_t k) { return k < 128u ? s_part[k] : p.plist0[blockIdx.x + k * gridDim.x]; };
    // the workgroup's work units: all in shard blockIdx.x % kUnitShards (the grid is a multiple of
    // kUnitShards or one partition per workgroup, so a shard holds the units of the list positions
    // j == shard (mod kUnitShards): at most unit_shard_cap of them, as sharding by partition did)
    constexpr uint32_t kCullUnitsLds = 512;
    __shared__ uint32_t s_units[kCullUnitsLds];
    __shared__ uint32_t s_nu, s_pos;
    if (tid == 0) s_nu = 0;
    lds_barrier();
    const uint32_t ush = blockIdx.x % kUnitShards;
    auto flush_units = [&] {  // (after a barrier: every thread reads s_nu)
        const uint32_t nu = s_nu;
        if (!nu) return;
        if (tid == 0) s_pos = atomicAdd(&p.ctl->unit_n[ush], nu);
        lds_barrier();
        for (uint32_t r = tid; r < nu; r += kProjThreads) p.units[(uint64_t)ush * ucap + s_pos + r] = s_units[r];
        lds_barrier();
        if (tid == 0) s_nu = 0;
        lds_barrier();
    };
    float4 ca[kProjRounds], cb[kProjRounds];  // ping-pong: no register moves between partitions
    uint32_t k = 0;
    uint32_t part = 0;
    if (nmine) {
        part = part_at(0);
        load_planes(part, ca);
    }
    // one partition: its planes in c, the next one's loaded into cn
    auto step = [&](float4 (&c)[kProjRounds], float4 (&cn)[kProjRounds]) {
        const uint32_t part_next = k + 1 < nmine ? part_at(k + 1) : part;
        load_planes(part_next, cn);  // (past the last: this partition again, unused)
        if (kt_items++ == 0) KT_MARK(0, 1, part);
        const uint32_t p0 = part * kProjTile;
        uint32_t cand = 0;  // bit it: slot p0 + it * kProjThreads + tid is a candidate
#pragma unroll
        for (int it = 0; it < kProjRounds; ++it) {
            const uint32_t i = p0 + it * kProjThreads + tid;
            bool cd = false;
            float vz, cx0, cy0, hb;
            if (i < p.n && cull_keep_box(p, c[it], row_lo, row_hi, vz, cx0, cy0, hb)) {
                const uint32_t key = sortable_key(vz);
                cd = key < T && !(CUT && cut_skip(p, s_cutb, key, cx0, cy0, hb));
                if (!cd) {  // past the threshold: counted, not projected
                    ++my_vis;
                    my_kmin_inv = max(my_kmin_inv, ~key);
                    my_kmax = max(my_kmax, key);
                }
            }
            cand |= (cd ? 1u : 0u) << it;
            const uint64_t bb = __ballot(cd);
            if (lane == 0) s_mask[it][w] = bb;
        }
        lds_barrier();
        if (tid < 64) {  // exclusive prefix of the (round, wave) ballots: index order
            constexpr int nb = kProjRounds * (kProjThreads / 64);
            const uint32_t cnt = tid < nb ? __popcll(s_mask[tid / (kProjThreads / 64)][tid % (kProjThreads / 64)]) : 0u;
            const uint32_t incl = wave_incl_scan(cnt);
            if (tid < nb) s_base[tid / (kProjThreads / 64)][tid % (kProjThreads / 64)] = incl - cnt;
            if (tid == 63) s_total = incl;
        }
        lds_barrier();
#pragma unroll
        for (int it = 0; it < kProjRounds; ++it) {
            const uint64_t bb = s_mask[it][w];
            if ((cand >> it) & 1u) p.cand[p0 + s_base[it][w] + __popcll(bb & lanemask_lt())] = (uint16_t)(it * kProjThreads + tid);
        }
        if (tid == 0) {
            const uint32_t tot = s_total;
            p.c0[part] = tot;
            // the partition's work units, gathered in LDS and appended to the frame's list once per
            // workgroup below (a returning atomic per partition on eight shared counters serialised
            // the one-chunk 50 M frame's cull: 49 K of them)
            const uint32_t nu = (tot + kProjThreads - 1) / kProjThreads;
            for (uint32_t r = 0; r < nu; ++r)
                s_units[s_nu + r] = (part * kProjRounds + r) | ((min(tot - r * kProjThreads, (uint32_t)kProjThreads) - 1u) << 20);
            s_nu += nu;
        }
        lds_barrier();  // (s_mask, s_base and s_total are rewritten by the next partition)
        if (s_nu > kCullUnitsLds - kProjRounds) flush_units();  // (room for one more partition's units)
        part = part_next;
        ++k;
    };
    while (k < nmine) {
        step(ca, cb);
        if (k >= nmine) break;
        step(cb, ca);
    }
    flush_units();
    if (my_vis) {
        atomicAdd(&s_vis, my_vis);
        atomicMax(&s_kmin_inv, my_kmin_inv);
        atomicMax(&s_kmax, my_kmax);
    }
    __syncthreads();
    if (tid == 0 && s_vis) {
        StatShard* st = p.stats + blockIdx.x % kStatShards;
        atomicAdd(&st->n_vis, s_vis);
        atomicMax(&st->key_min_inv, s_kmin_inv);
        atomicMax(&st->key_max, s_kmax);
    }
    KT_MARK(0, 2, kt_items);
}

// Projection, phase B: candidate q of a partition (slot slot_c0(part, q)) projected from its
// 48-B geometry record, one work unit (kProjThreads candidates) per workgroup iteration over the
// frame's unit list; a visible one gets its records and (from its shading block, one thread per
// splat in the reference's expression order: sh_colour) its colour in its slot, an invisible one
// leaves the slot a hole (rect kRectHole).  Publishes the visible count, their tile total, the depth range.
#ifdef GS_PROJ_NT  // (A/B builds: the model read with the streaming policy)
#define GS_PROJ_LOAD_POLICY " nt"
#else
#define GS_PROJ_LOAD_POLICY ""
#endif
template <bool SH12>  // SH12: degree-3 scenes (12 coefficient quads), staged through LDS
__global__ __launch_bounds__(kProjThreads, 3) void k_project(ProjParams p) {
    __shared__ unsigned long long s_k;
    __shared__ uint32_t s_vis, s_kmin_inv, s_kmax;
    // per wave: the SH quads of its 64 candidates, [candidate][quad] (viewed flat), loaded
    // straight into LDS (global_load_lds: no registers held, in flight while the footprint is
    // computed)
    // ([candidate][13 quads]: 12 coefficient quads and one of padding, so the 16 lanes of each
    // ds_read_b128 group land on 16 distinct 16-B slots of the bank row; a 12-quad stride put
    // them on 4, a 4-way conflict on every coefficient read)
    __shared__ float4 s_sh[SH12 ? kProjThreads / 64 : 1][SH12 ? 13 : 1][64];
    const int tid = threadIdx.x;
    const int wv = tid >> 6, lane = tid & 63;
    if (tid == 0) { s_k = 0; s_vis = 0; s_kmin_inv = 0; s_kmax = 0; }
    __syncthreads();
    uint32_t my_vis = 0, my_kmin_inv = 0, my_kmax = 0;
    unsigned long long my_k = 0;
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;
    KT_MARK(1, 0, 0);
    const UnitList L = load_units(p.units, p.ctl, proj_parts(p.n));
    uint32_t kt_items = 0;
    // The workgroup's units are software-pipelined: the next unit's list entry is loaded when this
    // unit starts and its candidate offset once this unit's footprint is computed, so a unit
    // starts with its geometry loads instead of two dependent round trips (list -> candidate).
    auto cand_of = [&](uint32_t uu) -> uint32_t {
        const uint32_t id = unit_id(uu);
        return (uint32_t)tid < unit_count(uu)
                   ? (uint32_t)p.cand[(id / kProjRounds) * kProjTile + (id % kProjRounds) * kProjThreads + tid]
                   : 0u;
    };
    uint32_t j = blockIdx.x;
    uint32_t u = j < L.total ? unit_at(L, j) : 0u;
    uint32_t cq = j < L.total ? cand_of(u) : 0u;
    for (; j < L.total; j += gridDim.x) {
        const uint32_t id = unit_id(u), jn = j + gridDim.x;
        const uint32_t un = jn < L.total ? unit_at(L, jn) : 0u;
        if (kt_items++ == 0) KT_MARK(1, 1, id);
        const uint32_t part = id / kProjRounds, q = (id % kProjRounds) * kProjThreads + tid;
        const uint32_t p0 = part * kProjTile;
        const bool act = (uint32_t)tid < unit_count(u);
        const uint32_t slot = slot_c0(part, q);
        const uint32_t i = p0 + cq;
        uint32_t oi = 0;
        float4 g0, g1, g2;
        Proj o;
        bool vis = false;
        if (SH12) {
            // Coalesced staging through this wave's 13 KiB of LDS.  Every piece is 1 KiB in which
            // consecutive lanes take consecutive 16-B chunks of one candidate's record (lane l of
            // piece k: chunk (64 k + l) % m of candidate (64 k + l) / m, m = 3 geometry / 13 SH
            // chunks, SH chunk 12 = padding, loaded as a repeat of chunk 11), so a piece touches
            // about 9 cache lines instead of up to 64.  The SH layout is [candidate][13 quads]: its
            // pieces 0-9 land at once, the geometry's 3 pieces in the last 3 KiB; once the
            // geometry is read out, SH pieces 10-12 land there.  Every lane takes part (an
            // inactive candidate reads its partition's first record).
            const uint32_t ia = act ? i : p0;
            const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)&s_sh[wv][0][0]);
            // an opaque copy of the lane id: the pieces' source lanes are recomputed per unit
            // instead of being hoisted into 15 loop-invariant registers (k_project sits at the
            // 168-VGPR limit of 3 waves per SIMD)
            uint32_t ln;
            asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"((uint32_t)lane));
            auto piece = [&](const float4* src, uint32_t dst) {
                uint32_t m0save;
                asm volatile(
                    "s_mov_b32 %[msave], m0\n"
                    "s_mov_b32 m0, %[lds]\n s_nop 0\n"
                    "global_load_lds_dwordx4 %[sp], off" GS_PROJ_LOAD_POLICY "\n"
                    "s_mov_b32 m0, %[msave]\n"
                    : [msave] "=&s"(m0save)
                    : [sp] "v"(src), [lds] "s"(dst)
                    : "memory");
            };
            asm volatile("global_load_dword %[oi], %[op], off" : [oi] "=&v"(oi) : [op] "v"(p.orig + ia) : "memory");
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t idx = 64u * k + ln, sc = idx / 3u, ch = idx % 3u;
                const uint32_t isrc = (uint32_t)__shfl((int)ia, (int)sc, 64);
                piece(p.geo + 3 * (uint64_t)isrc + ch, lds + 10240u + 1024u * k);
            }
            auto sh_piece = [&](int k) {
                const uint32_t idx = 64u * k + ln, sc = idx / 13u, ch = min(idx % 13u, 11u);
                const uint32_t isrc = (uint32_t)__shfl((int)ia, (int)sc, 64);
                piece(p.sh + 12 * (uint64_t)isrc + ch, lds + 1024u * k);
            };
#pragma unroll
            for (int k = 0; k < 10; ++k) sh_piece(k);
            // the geometry (issued before the 10 SH pieces) is in LDS once at most 10 are outstanding
            asm volatile("s_waitcnt vmcnt(10)" : "+v"(oi) :: "memory");
            const float4* sg = (const float4*)&s_sh[wv][0][0] + 640 + 3 * lane;
            g0 = sg[0];
            g1 = sg[1];
            g2 = sg[2];
            // the reads are done before SH pieces 10-12 overwrite the geometry's staging
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 10; k < 13; ++k) sh_piece(k);
        }
        if (act) {
            if (!SH12) {
                oi = p.orig[i];
                const float4* gi = p.geo + 3 * (uint64_t)i;
                g0 = gi[0];
                g1 = gi[1];
                g2 = gi[2];
            }
            vis = project_core_g(p, i, g0, g1, g2, row_lo, row_hi, false, o);
        }
        // the next unit's candidate: its load overlaps this unit's colour and stores (waiting for
        // the unit entry also drains this unit's SH loads, which are due by now)
        const uint32_t cqn = jn < L.total ? cand_of(un) : 0u;
        if (p.wlist) wide_append(p, 0, act && vis && o.prect != kRectEmpty && o.ntiles >= p.wide_tiles, slot);
        if (act) {
            if (vis) {
                store_slot(p, slot, i, oi, o);
                if (o.prect != kRectEmpty) {  // the SH colour of a splat that binds a tile
                    float4 col;
                    if (SH12) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        col = sh_colour<1>(&s_sh[wv][0][0] + 13 * lane, 12, g0.x, g0.y, g0.z, p.cam);
                    } else {
                        col = sh_colour(p.sh + (uint64_t)i * p.shq, p.shq, g0.x, g0.y, g0.z, p.cam);
                    }
                    col.w = __uint_as_float(o.key);
                    p.crec[3 * (uint64_t)slot + 2] = col;
                }
                ++my_vis;
                my_k += o.ntiles;
                my_kmin_inv = max(my_kmin_inv, ~o.key);
                my_kmax = max(my_kmax, o.key);
            } else {
                p.srect[slot] = kRectHole;
            }
        }
        u = un;
        cq = cqn;
    }
    if (my_vis) {
        atomicAdd(&s_vis, my_vis);
        atomicAdd(&s_k, my_k);
        atomicMax(&s_kmin_inv, my_kmin_inv);
        atomicMax(&s_kmax, my_kmax);
    }
    __syncthreads();
    if (tid == 0 && s_vis) {
        StatShard* st = p.stats + blockIdx.x % kStatShards;
        atomicAdd(&st->n_vis, s_vis);
        atomicAdd(&st->n_chunk[0], s_vis);
        atomicAdd(&st->k_total, s_k);
        atomicMax(&st->key_min_inv, s_kmin_inv);
        atomicMax(&st->key_max, s_kmax);
    }
    KT_MARK(1, 2, kt_items);
}

// ============================================================================ radix pass
// One stable LSD pass = two launches, no inter-workgroup waiting:
//   k_radix_upsweep    per partition (256 x IPT elements): digit histogram -> counts[part][digit],
//                      the pass's global histogram and group sums gsum[part / 32][digit] (atomics)
//   k_radix_downsweep  per partition: its offsets (digit base from the global histogram + earlier
//                      groups' sums + earlier partitions of its group), stable local ranks (wave
//                      ballots, element order inside the partition = (wave, item, lane)), LDS
//                      staging, contiguous writes per digit run
// This replaces webgpu-radix-sort's 16 x 2-bit passes (RS:621-654) with 8-bit digits.

// Sum of column entries a[0], a[256], ..., a[256 (m - 1)]: 8 independent loads in flight.
__device__ __forceinline__ uint32_t sum_column(const uint32_t* __restrict__ a, uint32_t m) {
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t k = 0;
    for (; k + 8 <= m; k += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += a[(uint64_t)(k + u) * 256];
    }
    for (; k < m; ++k) acc[0] += a[(uint64_t)k * 256];
    return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

__device__ __forceinline__ uint32_t radix_n(const SortPass& p) {
    if (p.gate && *p.gate == 0) return 0;
    return p.n_dev ? *p.n_dev : p.n;
}
// kFiltTail: does the element's tile rect (aux; wide rects from the record of Gaussian j) touch
// a tile chunk 0 left unsaturated?  Summed-area table lookups (L2-resident).
__device__ __forceinline__ bool tail_overlaps(const SortPass& p, uint32_t pr, uint32_t j) {
    if (pr == kRectEmpty) return false;
    uint32_t x0, y0, x1, y1;
    if (pr == kRectLarge) {
        const float4 m = p.rec.r2[j];
        const uint32_t bx = __float_as_uint(m.z), by = __float_as_uint(m.w);
        x0 = (bx & 0xffffu) >> 4; y0 = (by & 0xffffu) >> 4; x1 = bx >> 20; y1 = by >> 20;
    } else {
        x0 = pr & 0xfffu; y0 = (pr >> 12) & 0xfffu;
        x1 = x0 + ((pr >> 24) & 15u); y1 = y0 + (pr >> 28);
    }
    const uint32_t sw = (uint32_t)p.tiles_x + 1, rb = (uint32_t)p.tile_row_begin;
    const uint32_t* a = p.sat + (uint64_t)(y0 - rb) * sw;
    const uint32_t* b = p.sat + (uint64_t)(y1 + 1 - rb) * sw;
    return (b[x1 + 1] - b[x0]) - (a[x1 + 1] - a[x0]) != 0u;
}

__device__ __forceinline__ bool radix_valid(const SortPass& p, uint32_t n, uint64_t idx, uint32_t key, uint32_t aux) {
    if (idx >= n) return false;
    switch (p.filter) {
        case kFiltNone: return true;
        case kFiltSentinel: return key != kSentinel;
        case kFiltBelow: return key < p.thresh;
        default: return key >= p.thresh && key != kSentinel && tail_overlaps(p, aux, (uint32_t)idx);
    }
}

template <int IPT>
__global__ __launch_bounds__(kSortThreads) void k_radix_upsweep(SortPass p) {
    constexpr int kTileN = kSortThreads * IPT;
    __shared__ uint32_t s_hist[4][256];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t n = radix_n(p), parts = (n + kTileN - 1) / kTileN;
    uint32_t total = 0;  // this workgroup's count of digit `tid` over all its partitions
    for (uint32_t part = blockIdx.x; part < parts; part += gridDim.x) {
        for (int t = tid; t < 1024; t += kSortThreads) (&s_hist[0][0])[t] = 0;
        __syncthreads();
        const uint64_t wbase = (uint64_t)part * kTileN + (uint64_t)w * (IPT * 64);
#pragma unroll 4
        for (int it = 0; it < IPT; ++it) {
            const uint64_t idx = wbase + it * 64 + lane;
            const uint32_t key = idx < n ? p.keys_in[idx] : kSentinel;
            const uint32_t aux = (p.filter == kFiltTail && idx < n) ? p.aux_in[idx] : 0u;
            if (radix_valid(p, n, idx, key, aux)) atomicAdd(&s_hist[w][(key >> p.shift) & p.mask], 1u);
        }
        __syncthreads();
        const uint32_t c = s_hist[0][tid] + s_hist[1][tid] + s_hist[2][tid] + s_hist[3][tid];
        p.offsets[(uint64_t)part * 256 + tid] = c;  // partition-major
        if (c) atomicAdd(&p.gsum[(part / kGroupParts) * 256 + tid], c);
        total += c;
        __syncthreads();
    }
    // global digit histogram of this pass (kHistShards shards, zeroed with the frame)
    if (total) atomicAdd(&p.hist[(blockIdx.x % kHistShards) * 256 + tid], total);
}

template <int IPT>
__global__ __launch_bounds__(kSortThreads) void k_radix_downsweep(SortPass p) {
    constexpr int kTileN = kSortThreads * IPT;
    __shared__ uint32_t s_wave_hist[4][256];
    __shared__ uint32_t s_digit_start[256];
    __shared__ uint32_t s_global[256];
    __shared__ uint32_t s_keys[kTileN];
    __shared__ uint32_t s_vals[kTileN];
    __shared__ uint32_t s_aux[kTileN];
    __shared__ uint32_t s_tmp[8];

    __shared__ uint32_t s_sub[kMaxMerge + 1];  // element prefix of the round's partitions
    __shared__ uint32_t s_nsub;

    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t n = radix_n(p), parts = (n + kTileN - 1) / kTileN;
    const bool has_aux = p.aux_in != nullptr;
    // A workgroup takes `merge` consecutive partitions and ranks them in rounds of whole
    // partitions whose elements fit the tile: the scan's offsets of a round's first partition
    // place the round's digit-d elements contiguously, since the partitions follow each other.
    // (merge > 1 only for the compacted input of k_project, whose partitions are mostly empty.)
    const uint32_t M = p.part_count ? max(1u, min((uint32_t)p.merge, (uint32_t)kMaxMerge)) : 1u;
    const uint32_t units = (parts + M - 1) / M;
    // digit d's base: exclusive scan of the pass's global histogram (every workgroup computes it;
    // workgroup 0 also reports the elements this pass keeps)
    uint32_t dbase;
    {
        uint32_t tot = 0;
        for (int sh = 0; sh < kHistShards; ++sh) tot += p.hist[sh * 256 + tid];
        uint32_t gtotal;
        dbase = block_excl_scan256(tot, s_tmp, &gtotal);
        if (blockIdx.x == 0 && tid == 0 && p.count_out) *p.count_out = gtotal;
    }
    for (uint32_t unit = blockIdx.x; unit < units; unit += gridDim.x) {
      const uint32_t se = min((unit + 1) * M, parts);
      for (uint32_t sp = unit * M; sp < se;) {  // workgroup-uniform
        // element counts of partitions sp .. se-1 (compacted input: only partition q's first
        // part_count[q] elements exist), loaded in parallel, then cut into the round
        if (tid < (int)(se - sp))
            s_sub[tid + 1] = p.part_count ? p.part_count[sp + tid] : min((uint32_t)kTileN, n - (sp + tid) * kTileN);
        __syncthreads();
        if (tid == 0) {
            uint32_t tot = 0, k = 0;
            s_sub[0] = 0;
            for (uint32_t q = sp; q < se; ++q) {
                const uint32_t c = s_sub[k + 1];
                if (k > 0 && tot + c > (uint32_t)kTileN) break;
                tot += c;
                s_sub[++k] = tot;
            }
            s_nsub = k;
        }
        for (int t = tid; t < 1024; t += kSortThreads) (&s_wave_hist[0][0])[t] = 0;
        {   // digit tid's first output position for partition sp: its base, the group sums of the
            // earlier groups and the counts of the earlier partitions of sp's group (no scan launch)
            const uint32_t g = sp / kGroupParts;
            s_global[tid] = dbase + sum_column(p.gsum + tid, g) +
                            sum_column(p.offsets + (uint64_t)g * kGroupParts * 256 + tid, sp - g * kGroupParts);
        }
        __syncthreads();
        const uint32_t nsub = s_nsub, total = s_sub[nsub];

        uint32_t keys[IPT], vals[IPT], aux[IPT], rank[IPT];
#pragma unroll
        for (int it = 0; it < IPT; ++it) {
            const uint32_t slot = (uint32_t)w * (IPT * 64) + it * 64 + lane;
            const bool in = slot < total;
            uint64_t idx = 0;
            if (in) {
                uint32_t k = 0;
                while (k + 1 < nsub && slot >= s_sub[k + 1]) ++k;
                idx = (uint64_t)(sp + k) * kTileN + (slot - s_sub[k]);
            }
            keys[it] = in ? p.keys_in[idx] : kSentinel;
            vals[it] = in ? (p.vals_in ? p.vals_in[idx] : (uint32_t)idx) : 0u;
            aux[it] = (in && has_aux) ? p.aux_in[idx] : 0u;
            rank[it] = (in && radix_valid(p, n, idx, keys[it], aux[it])) ? 0u : 0x80000000u;  // top bit: unsorted
        }
        __syncthreads();
        if (p.filter != kFiltNone) {
            // filtered pass: compact each wave's kept elements, in order, into the front rows of its
            // slice of the stage (order within the partition is unchanged), so ranking only visits
            // rows that hold kept elements
            uint32_t* wk = s_keys + w * (IPT * 64);
            uint32_t* wv = s_vals + w * (IPT * 64);
            uint32_t* wa = s_aux + w * (IPT * 64);
            uint32_t m = 0;
#pragma unroll
            for (int it = 0; it < IPT; ++it) {
                const bool valid = (rank[it] & 0x80000000u) == 0u;
                const uint64_t b = __ballot(valid);
                if (valid) {
                    const uint32_t q = m + __popcll(b & lanemask_lt());
                    wk[q] = keys[it];
                    wv[q] = vals[it];
                    if (has_aux) wa[q] = aux[it];
                }
                m += __popcll(b);
            }
            __syncthreads();
#pragma unroll
            for (int it = 0; it < IPT; ++it) {
                const uint32_t q = it * 64 + lane;
                const bool valid = q < m;
                keys[it] = valid ? wk[q] : kSentinel;
                vals[it] = valid ? wv[q] : 0u;
                aux[it] = (valid && has_aux) ? wa[q] : 0u;
                rank[it] = valid ? 0u : 0x80000000u;
            }
            __syncthreads();
        }
#pragma unroll
        for (int it = 0; it < IPT; ++it) {
            const bool valid = (rank[it] & 0x80000000u) == 0u;
            const uint32_t digit = (keys[it] >> p.shift) & p.mask;
            uint64_t peers = __ballot(valid);
            if (peers == 0) continue;  // wave-uniform: no kept element in this row
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const bool bit = (digit >> b) & 1u;
                const uint64_t bb = __ballot(bit);
                peers &= bit ? bb : ~bb;
            }
            if (valid) {
                const uint32_t lower = __popcll(peers & lanemask_lt());
                const uint32_t prev = s_wave_hist[w][digit];
                rank[it] = prev + lower;
                if (lower + 1 == (uint32_t)__popcll(peers)) s_wave_hist[w][digit] = prev + lower + 1;
            }
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();

        const int d = tid;
        const uint32_t c0 = s_wave_hist[0][d], c1 = s_wave_hist[1][d], c2 = s_wave_hist[2][d],
                       c3 = s_wave_hist[3][d];
        uint32_t tile_total;
        const uint32_t dstart = block_excl_scan256(c0 + c1 + c2 + c3, s_tmp, &tile_total);
        s_digit_start[d] = dstart;
        s_wave_hist[0][d] = 0;
        s_wave_hist[1][d] = c0;
        s_wave_hist[2][d] = c0 + c1;
        s_wave_hist[3][d] = c0 + c1 + c2;
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IPT; ++it) {
            if ((rank[it] & 0x80000000u) == 0u) {
                const uint32_t digit = (keys[it] >> p.shift) & p.mask;
                const uint32_t pos = s_digit_start[digit] + s_wave_hist[w][digit] + rank[it];
                s_keys[pos] = keys[it];
                s_vals[pos] = vals[it];
                if (has_aux) s_aux[pos] = aux[it];
            }
        }
        __syncthreads();
        for (uint32_t q = tid; q < tile_total; q += kSortThreads) {
            const uint32_t k = s_keys[q];
            const uint32_t digit = (k >> p.shift) & p.mask;
            const uint32_t dest = s_global[digit] + (q - s_digit_start[digit]);
            p.keys_out[dest] = k;
            p.vals_out[dest] = s_vals[q];
            if (has_aux) p.aux_out[dest] = s_aux[q];
        }
        __syncthreads();
        sp += nsub;
      }
    }
}

// ============================================================================ binning
// Chunk c is the depth-sorted array of its splats: chunk 0 = visible splats with key < T, chunk 1
// = those with key >= T whose rect touches a tile chunk 0 left unsaturated (binned into those
// tiles only).  Concatenated, the two stable sorts are the full stable order.
// Launches per chunk, no inter-workgroup waiting: per-partition entry counts, one scan, the
// emission in depth order, then the row-wise emission of wide splats.  Entry positions come from
// the scan alone, so whichever kernel writes an entry, every tile's list stays in depth order.
struct TileRect {
    uint32_t x0, y0, x1, y1;  // inclusive, absolute tile coordinates
};

__device__ __forceinline__ bool rect_unpack(const BinParams& p, uint32_t pr, uint32_t j, TileRect& r) {
    if (pr == kRectEmpty || pr == kRectHole) return false;
    if (pr == kRectLarge) {  // tile box from the pixel box in the record
        const float4 m = p.rec.r2[j];
        const uint32_t bx = __float_as_uint(m.z), by = __float_as_uint(m.w);
        r = {(bx & 0xffffu) >> 4, (by & 0xffffu) >> 4, bx >> 20, by >> 20};
    } else {
        r.x0 = pr & 0xfffu;
        r.y0 = (pr >> 12) & 0xfffu;
        r.x1 = r.x0 + ((pr >> 24) & 15u);
        r.y1 = r.y0 + (pr >> 28);
    }
    return true;
}

__device__ __forceinline__ uint32_t tile_id(const BinParams& p, uint32_t tx, uint32_t ty) {
    return (ty - (uint32_t)p.tile_row_begin) * (uint32_t)p.tiles_x + tx;
}

__device__ __forceinline__ bool rect_wide(const BinParams& p, const TileRect& r) {
    return (r.x1 - r.x0 + 1) * (r.y1 - r.y0 + 1) >= p.wide_tiles;
}

// ---- exact-ish binning: the alpha >= 1/255 region of a splat is the ellipse
//   u'^2 + v'^2 <= log2(op) + log2(255),  u' = d.e1', v' = d.e2'  (d = pixel - centre, record axes)
// (the quad's |u|,|v| <= 2 only removes pixels from it).  It is convex, so in every tile row the
// tiles holding one of its pixel centres form one contiguous column range, computed in closed
// form below and widened (log2 margin, 0.02 px + relative) so that no pixel the composite would
// blend is ever dropped.  Count, emission and the wide path call the same functions, and those
// functions are compiled without floating-point contraction: with hipcc's default (fusion left to
// the backend) each inlined copy could fuse a different mul + add into an FMA, so the count
// (inside bin_walk), the emission loop and wide_entries rounded one column bound differently and
// a splat's entry could be counted in a tile it was not emitted into -- one list position left
// stale (a duplicate of an older frame's entry) and the splat missing.
// With every operation rounded on its own, every copy computes the same bits, so a tile's count
// and its entries agree exactly; k_bin_emit checks that (bin_chk, kErrBinning).
#ifndef GS_BIN_CONTRACT_FAST  // (diagnostics builds only: the round-5 code generation, for the A/B)
#define GS_BIN_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define GS_BIN_NO_CONTRACT
#endif
struct Ellipse {
    float cx, cy, m00, m01, det, l, hy, dys, xm, rm00, ml;  // xm: x margin; rm00 = 1 / m00; ml = m00 l
    uint32_t px0, px1;                             // pixel box columns
    bool ok;                                       // false: use the whole box row (degenerate)
};

// Hardware sqrt / reciprocal (about 1 ulp): the ranges only need to be conservative, and the
// margins above are orders of magnitude wider than their error.
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ Ellipse ellipse_of(const float4 q0, const float4 q1) {
    GS_BIN_NO_CONTRACT
    Ellipse e;
    const float ax = q0.z, ay = q0.w, bx = q1.x, by = q1.y;
    const uint32_t bbx = __float_as_uint(q1.w);
    e.cx = q0.x;
    e.cy = q0.y;
    e.px0 = bbx & 0xffffu;
    e.px1 = bbx >> 16;
    // (explicit FMAs: the speed of contraction, the same bits in every inlined copy)
    e.m00 = __builtin_fmaf(ax, ax, bx * bx);
    e.m01 = __builtin_fmaf(ax, ay, bx * by);
    const float m11 = __builtin_fmaf(ay, ay, by * by);
    const float da = __builtin_fmaf(ax, by, -(ay * bx));
    e.det = da * da;
    e.l = q1.z + 7.99435343f + 2e-3f;  // log2(op) + log2(255) + margin
    e.ml = e.m00 * e.l;
    const float rdet = frcp(e.det);
    const float hx = fsqrt(e.l * m11 * rdet);
    e.hy = fsqrt(e.l * e.m00 * rdet) * 1.0001f + 0.02f;
    e.dys = -e.m01 * fsqrt(e.l * rdet * frcp(m11));  // y offset of the rightmost point
    e.xm = 0.02f + 1e-4f * hx;
    e.rm00 = frcp(e.m00);
    e.ok = e.l > 0.0f && e.det > 0.0f && isfinite(hx) && isfinite(e.hy) && isfinite(e.dys) &&
           isfinite(e.rm00) && isfinite(e.cx) && isfinite(e.cy);
    return e;
}

// Pixel columns [pl, ph] of a band of pixel rows (a tile row: 16 ty .. 16 ty + 15) holding a
// pixel centre of the ellipse, inside the box; false when there is none.
// dy0 / dy1: the band's first and last pixel-row centres minus the ellipse centre's y.
__device__ __forceinline__ bool ellipse_cols_dy(const Ellipse& e, float dy0, float dy1, uint32_t& pl_,
                                                uint32_t& ph_) {
    GS_BIN_NO_CONTRACT
    if (!e.ok) {
        pl_ = e.px0;
        ph_ = e.px1;
        return true;
    }
    const float lo = fmaxf(dy0, -e.hy);
    const float hi = fminf(dy1, e.hy);
    if (!(lo <= hi)) return false;
    const float d1 = fminf(fmaxf(e.dys, lo), hi), d0 = fminf(fmaxf(-e.dys, lo), hi);
    const float g1 = fsqrt(fmaxf(__builtin_fmaf(-(e.det * d1), d1, e.ml), 0.0f));
    const float g0 = fsqrt(fmaxf(__builtin_fmaf(-(e.det * d0), d0, e.ml), 0.0f));
    const float xmax = __builtin_fmaf(__builtin_fmaf(-e.m01, d1, g1), e.rm00, e.cx) + e.xm;
    const float xmin = __builtin_fmaf(-__builtin_fmaf(e.m01, d0, g0), e.rm00, e.cx) - e.xm;
    // pixel columns px with px + 0.5 in [xmin, xmax], inside the box
    const float pl = fmaxf(ceilf(xmin - 0.5f), (float)e.px0), ph = fminf(floorf(xmax - 0.5f), (float)e.px1);
    if (!(pl <= ph)) {
        if (isfinite(xmin) && isfinite(xmax)) return false;
        pl_ = e.px0;  // NaN/inf: the whole box row (conservative)
        ph_ = e.px1;
        return true;
    }
    pl_ = (uint32_t)pl;
    ph_ = (uint32_t)ph;
    return true;
}

__device__ __forceinline__ bool ellipse_cols_band(const Ellipse& e, uint32_t y0, uint32_t y1, uint32_t& pl_,
                                                  uint32_t& ph_) {  // pixel rows y0 .. y1
    GS_BIN_NO_CONTRACT
    return ellipse_cols_dy(e, (float)y0 + 0.5f - e.cy, (float)y1 + 0.5f - e.cy, pl_, ph_);
}

__device__ __forceinline__ bool ellipse_cols(const Ellipse& e, uint32_t ty, uint32_t& pl_, uint32_t& ph_) {
    return ellipse_cols_band(e, ty * kTile, ty * kTile + kTile - 1, pl_, ph_);
}

// Tile columns [xa, xb] of tile row ty holding a pixel centre of the ellipse (inside the box).
__device__ __forceinline__ bool ellipse_row(const Ellipse& e, uint32_t ty, uint32_t& xa, uint32_t& xb) {
    uint32_t pl, ph;
    if (!ellipse_cols(e, ty, pl, ph)) return false;
    xa = pl >> 4;
    xb = ph >> 4;
    return true;
}

// ---- binning into per-tile lists, a two-level counting sort without global atomics.  The
// chunk's slots come in units of (projection partition, round of kProjThreads slots); binning
// partition b (of BinParams::nparts) takes units b, b + nparts, ... (interleaved: balanced whatever
// the scene order, also when a few partitions hold all the splats); the tiles are cut into bands
// of <= kBandTiles.
//   k_bin_count    workgroup (partition b, band): LDS counters of its splats' entries per tile
//                  (ellipse rows; chunk 1: unsaturated tiles only) -> bmat[b][t]
//   k_bin_colscan  per tile: exclusive prefix of bmat[.][t] over the partitions, tile totals
//   (tile scan)    exclusive scan of the totals in tile order -> ranges (k_bin_emit does it per
//                  workgroup; k_chunk1 runs tile_scan_body once)
//   k_bin_emit     workgroup (b, band): LDS cursors tbase[t] + bmat[b][t]; each entry takes a
//                  position with an LDS atomic (lists are unordered inside a tile: k_tile_sort)
// Count and emission walk the same ellipse rows, so a tile's count and its entries agree.
constexpr uint32_t kWideQueue = 512;     // wide splats queued per binning workgroup (k_chunk1)
constexpr uint32_t kWideQueueMax = 8192; // ... and at most, in the binning launches
constexpr size_t kBinLdsMaxWords = 40448; // 158 KiB: the binning launches' dynamic LDS bound

// The chunk's work units: chunk 0 the frame's list (k_cull), chunk 1 every unit of every partition.
__device__ __forceinline__ UnitList bin_unit_list(const BinParams& p) {
    if (p.units) return load_units(p.units, p.ctl, p.parts);
    UnitList L;
    L.units = nullptr;
    L.total = p.parts * (uint32_t)kProjRounds;
    return L;
}

__device__ __forceinline__ uint32_t bin_units(const UnitList& L, uint32_t b, uint32_t np) {
    return L.total > b ? (L.total - b + np - 1) / np : 0u;
}

// The slots of binning partition b (units b, b + nparts, ... of the chunk's list):
// s_pref[k] = slots of its first k units; returns the total.  Contains barriers.
// LISTED: the chunk's units come from k_cull's list, counts packed in the entries (chunk 0);
// otherwise every unit of every partition, counts from p.cnt (chunk 1)
template <int NT, bool LISTED>
__device__ uint32_t bin_slots(const BinParams& p, const UnitList& L, uint32_t b, uint32_t* s_pref, uint32_t* s_tmp) {
    const uint32_t m = min(bin_units(L, b, p.nparts), kBinMaxUnits);
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    constexpr int per = kBinMaxUnits / NT;
    uint32_t* s_uid = LISTED && p.uid_lds ? s_pref + p.pref_words : nullptr;  // (bin_slot reads them)
    uint32_t c[per], sum = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const uint32_t j = (uint32_t)tid * per + k;
        c[k] = 0;
        if (j < m) {
            const uint32_t u = unit_at(L, b + j * p.nparts);
            if (LISTED) {
                c[k] = unit_count(u);
                if (s_uid) s_uid[j] = u;
            } else {
                const uint32_t part = u / kProjRounds, r0 = (u % kProjRounds) * kProjThreads;
                const uint32_t cn = p.cnt[part];
                c[k] = cn > r0 ? min(cn - r0, (uint32_t)kProjThreads) : 0u;
            }
        }
        sum += c[k];
    }
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) s_tmp[w] = incl;
    __syncthreads();
    uint32_t base = incl - sum, total = 0;
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) base += s_tmp[i];
        total += s_tmp[i];
    }
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const uint32_t j = (uint32_t)tid * per + k;
        if (j <= m) s_pref[j] = base;
        base += c[k];
    }
    __syncthreads();
    return total;
}

// The r-th slot of binning partition b (r < total of bin_slots).
__device__ __forceinline__ uint32_t bin_slot(const BinParams& p, const UnitList& L, uint32_t b,
                                             const uint32_t* s_pref, uint32_t r) {
    const uint32_t m = min(bin_units(L, b, p.nparts), kBinMaxUnits);
    uint32_t lo = 0, hi = m;  // largest k < m with s_pref[k] <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_pref[mid] <= r) lo = mid; else hi = mid;
    }
    // (the unit entry from LDS when bin_slots cached it: no global round trip per slot)
    const uint32_t u = unit_id(p.uid_lds && L.units ? s_pref[p.pref_words + lo] : unit_at(L, b + lo * p.nparts)),
                   part = u / kProjRounds;
    const uint32_t q = (u % kProjRounds) * kProjThreads + (r - s_pref[lo]);
    return p.chunk ? slot_c1(part, q) : slot_c0(part, q);
}

// The per-tile cut filter of a binning walk (see kCutMaxTiles): s = the band's cut bounds in LDS
// (entry t - t_lo), mode 0 = every entry (chunk 1: of the unsaturated tiles), 1 = chunk 0 with the
// cut (cut_keep), 2 = chunk 1's walk over chunk 0's splats (the entries the cut left out, in the
// tiles chunk 0 left unsaturated).  Count and emission filter identically.
struct CutWalk {
    const uint16_t* s;
    const uint32_t* sb;  // the frame's block minima / maxima in LDS (cut_blocks)
    uint32_t t_lo, bxn, rb;
    int mode;
    // per entry, with a splat's class m (splat_mode): 0 keep, 1 cut_keep, 2 cut out and the tile
    // unsaturated, 3 the tile unsaturated
    __device__ __forceinline__ bool keep(const BinParams& p, uint32_t t, uint32_t key, int m) const {
        if (m == 0) return true;
        if (m == 3) return !p.done[t];
        const bool k = cut_keep(s[t - t_lo], key);
        return m == 1 ? k : (!k && !p.done[t]);
    }
    // A splat's class from the blocks of its tile rect: -1 none of its entries passes the walk's
    // filter, 0 (mode 1) all do, 3 (mode 2) all are cut out (then the done test only), else `mode`
    // (a test per entry); rects of more than 16 blocks are tested per entry.
    __device__ __forceinline__ int splat_mode(const TileRect& tr, uint32_t key) const {
        if (mode == 0) return 0;
        const uint32_t bx0 = tr.x0 / kCutBlock, bx1 = tr.x1 / kCutBlock;
        const uint32_t by0 = (tr.y0 - rb) / kCutBlock, by1 = (tr.y1 - rb) / kCutBlock;
        if ((bx1 - bx0 + 1) * (by1 - by0 + 1) > 16) return mode;
        uint32_t mn = 0xFFFFu, mx = 0u;
        for (uint32_t by = by0; by <= by1; ++by)
            for (uint32_t bx = bx0; bx <= bx1; ++bx) {
                const uint32_t v = sb[by * bxn + bx];
                mn = min(mn, v & 0xFFFFu);
                mx = max(mx, v >> 16);
            }
        const uint32_t k16 = key >> 16;
        if (mode == 1) return k16 >= mx ? -1 : (k16 < mn ? 0 : 1);
        return k16 < mn ? -1 : (k16 >= mx ? 3 : 2);
    }
};

// Entries of one splat (composite slot g, depth key `key`) in tiles [t_lo, t_hi): f(tile) per
// entry.  (Starting each lane's walk at a lane-dependent row and column, so that neighbouring
// splats' LDS counter atomics stop colliding, measured binning 72 -> 78 us: the collisions are
// cheaper than the walk.)
template <class F>
__device__ __forceinline__ void splat_entries(const BinParams& p, const TileRect& tr, const Ellipse& e,
                                              uint32_t t_lo, uint32_t t_hi, uint32_t key, const CutWalk& cw, int m, F&& f) {
    const uint32_t tx = (uint32_t)p.tiles_x, rb = (uint32_t)p.tile_row_begin;
    const uint32_t ya = max(tr.y0, rb + t_lo / tx), yb = min(tr.y1, rb + (t_hi - 1) / tx);
    for (uint32_t ty = ya; ty <= yb; ++ty) {
        uint32_t xa, xb;
        if (!ellipse_row(e, ty, xa, xb)) continue;
        xa = max(xa, tr.x0);
        xb = min(xb, tr.x1);
        const uint32_t t0 = (ty - rb) * tx;
        if (p.chunk == 0) {  // the row's run clipped to the band, then four entries at a time (their
                             // counter atomics independent, in flight together: one-chunk 50 M / 4K
                             // count 0.87 -> 0.77 ms)
            xa = max(xa, t_lo > t0 ? t_lo - t0 : 0u);
            if (t_hi <= t0) continue;
            xb = min(xb, t_hi - 1u - t0);
            uint32_t x = xa;
            if (m) {  // (four bound reads in flight together, then the kept entries)
                for (; x + 3u <= xb; x += 4u) {
                    const bool k0 = cw.keep(p, t0 + x, key, m), k1 = cw.keep(p, t0 + x + 1u, key, m);
                    const bool k2 = cw.keep(p, t0 + x + 2u, key, m), k3 = cw.keep(p, t0 + x + 3u, key, m);
                    if (k0) f(t0 + x);
                    if (k1) f(t0 + x + 1u);
                    if (k2) f(t0 + x + 2u);
                    if (k3) f(t0 + x + 3u);
                }
                for (; x <= xb; ++x)
                    if (cw.keep(p, t0 + x, key, m)) f(t0 + x);
                continue;
            }
            for (; x + 3u <= xb; x += 4u) {
                f(t0 + x);
                f(t0 + x + 1u);
                f(t0 + x + 2u);
                f(t0 + x + 3u);
            }
            for (; x <= xb; ++x) f(t0 + x);
            continue;
        }
        for (uint32_t x = xa; x <= xb; ++x) {
            const uint32_t t = t0 + x;
            if (t < t_lo || t >= t_hi) continue;
            if (p.chunk == 1 && p.done[t]) continue;
            f(t);
        }
    }
}

// Entries of a wide splat (slot g) in tiles [t_lo, t_hi), walked by a whole wave: lane l takes
// cells l, l + 64, ... of the splat's tile box (in the band), each testing its cell against the
// ellipse's column range in the cell's tile row.  f(tile) per entry.
template <class F>
__device__ __forceinline__ void wide_entries(const BinParams& p, uint32_t g, uint32_t t_lo, uint32_t t_hi,
                                             const CutWalk& cw, F&& f, uint32_t first = lane_id(), uint32_t step = 64u) {
    const uint32_t tx = (uint32_t)p.tiles_x, rb = (uint32_t)p.tile_row_begin;
    TileRect tr;
    rect_unpack(p, p.srect[g], p.sidx[g], tr);
    const uint32_t key = cw.mode ? p.skey[g].x : 0u;
    const float4* q = p.crec + 3 * (uint64_t)g;
    const Ellipse e = ellipse_of(q[0], q[1]);
    const uint32_t ya = max(tr.y0, rb + t_lo / tx), yb = min(tr.y1, rb + (t_hi - 1) / tx);
    if (ya > yb) return;
    const uint32_t w = tr.x1 - tr.x0 + 1, cells = w * (yb - ya + 1);
    for (uint32_t c = first; c < cells; c += step) {
        const uint32_t ty = ya + c / w, x = tr.x0 + c % w;
        uint32_t xa, xb;
        if (!ellipse_row(e, ty, xa, xb) || x < xa || x > xb) continue;
        const uint32_t t = (ty - rb) * tx + x;
        if (t < t_lo || t >= t_hi || (p.chunk == 1 && p.done[t]) || !cw.keep(p, t, key, cw.mode)) continue;
        f(t);
    }
}

constexpr uint32_t kWaveCells = 1024;  // listed wide splats of at most this many box tiles: one wave
// The chunk's listed wide splats (BinParams::wlist) that binning partition `part` walks: list
// entries part, part + nparts, ..., each by the whole workgroup (threads over the splat's tile
// cells), so the wide splats spread over every workgroup (a partition that held many of them
// walked them all itself, one wave per splat: a near view's binning took 300 us).  Count and
// emission walk the same assignment.  f(tile) or f(tile, slot) per entry.
template <int NT, class F>
__device__ __forceinline__ void wide_listed(const BinParams& p, uint32_t part, uint32_t t_lo, uint32_t t_hi,
                                            const CutWalk& cw, F&& f) {
    if (!p.wlist) return;
    uint32_t pre[kWideShards + 1];  // the shards' lists, concatenated
    pre[0] = 0;
    const uint32_t cap = wide_shard_cap(p.parts);
#pragma unroll
    for (uint32_t k = 0; k < kWideShards; ++k) pre[k + 1] = pre[k] + min(p.stats[k].wl_n[p.chunk], cap);
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint32_t wn = pre[kWideShards];
    const uint32_t np = p.nparts;
    const uint32_t share = wn > part ? (wn - part + np - 1) / np : 0u;  // entries part + i nparts
    uint32_t k = 0;  // the workgroup's entries in turn: a splat of at most kWaveCells tile cells goes
                     // to one wave (round-robin), a larger one to every thread of the workgroup
    for (uint32_t i0 = 0; i0 < share; i0 += 64) {
        // 64 entries' slots and tile counts loaded at once (one lane each), then broadcast
        uint32_t g = 0, cells = 0;
        if (i0 + lane < share) {
            const uint32_t j = part + (i0 + lane) * np;
            uint32_t sh = 0, base = 0;  // (selects, not an indexed array: no scratch)
#pragma unroll
            for (uint32_t k = 1; k < kWideShards; ++k)
                if (j >= pre[k]) {
                    sh = k;
                    base = pre[k];
                }
            const uint32_t q = j - base;
            g = p.wlist[(uint64_t)sh * cap + (p.chunk ? cap - 1u - q : q)];
            TileRect tr;
            rect_unpack(p, p.srect[g], p.sidx[g], tr);
            cells = (tr.x1 - tr.x0 + 1) * (tr.y1 - tr.y0 + 1);
        }
        const uint32_t m = min(64u, share - i0);
        for (uint32_t e = 0; e < m; ++e) {
            const uint32_t ge = (uint32_t)__builtin_amdgcn_readlane((int)g, (int)e);
            const bool big = (uint32_t)__builtin_amdgcn_readlane((int)cells, (int)e) > kWaveCells;
            if (!big && (k++ % (NT / 64)) != w) continue;  // (wave-uniform)
            const uint32_t first = big ? threadIdx.x : lane, step = big ? (uint32_t)NT : 64u;
            if constexpr (std::is_invocable_v<F, uint32_t, uint32_t>)
                wide_entries(p, ge, t_lo, t_hi, cw, [&](uint32_t t) { f(t, ge); }, first, step);
            else
                wide_entries(p, ge, t_lo, t_hi, cw, f, first, step);
        }
    }
}

// The slots of binning partition `part` in rank order r = threadIdx.x, + NT, ...: f(g, packed
// rect, storage index, record quads 0 and 1) per slot, each slot's words loaded one slot ahead
// (two register sets, no moves), so a thread's next slot is in flight while it walks the current
// one (the one-chunk 50 M / 4K frame's binning holds ~160 slots per thread at one workgroup per CU).
// Records are loaded for every slot (holes included: valid memory, unused).
template <int NT, class F>
__device__ __forceinline__ void bin_walk(const BinParams& p, const UnitList& L, uint32_t part, const uint32_t* s_pref,
                                         uint32_t total, bool with_key, F&& f) {
    struct In {
        uint32_t g, pr, sj, key;
        float4 q0, q1;
    };
    auto fetch = [&](uint32_t r, In& s) {
        s.g = bin_slot(p, L, part, s_pref, r);
        s.pr = p.srect[s.g];
        s.sj = p.sidx[s.g];
        s.key = with_key ? p.skey[s.g].x : 0u;
        const float4* q = p.crec + 3 * (uint64_t)s.g;
        s.q0 = q[0];
        s.q1 = q[1];
    };
    uint32_t r = threadIdx.x;
    if (r >= total) return;
    In a, b;
    fetch(r, a);
    auto step = [&](In& cur, In& nxt) {
        const uint32_t rn = r + NT;
        fetch(min(rn, total - 1u), nxt);  // (past the end: the last slot again, unused)
        f(cur.g, cur.pr, cur.sj, cur.key, cur.q0, cur.q1);
        r = rn;
    };
    for (;;) {
        step(a, b);
        if (r >= total) break;
        step(b, a);
        if (r >= total) break;
    }
}

// The count/emission invariant (kErrBinning): per binning workgroup, the entries it counted and
// the entries it emitted, both as (sum over its tiles of n_t, sum of n_t * bin_hash(t)) mod 2^32.
// Equal sums mean equal per-tile counts unless two or more tiles differ in a way that cancels in
// both: a net change shows in the first, one entry moved between tiles a and b in the second
// ((a - b) * odd != 0 mod 2^32).  k_bin_count's waves add their sums straight into
// BinParams::bchk[vb] (agent-scope atomics: no barrier at the count's end); k_bin_emit reduces its
// own in LDS (s_chk, zeroed before the walk), compares and zeroes bchk[vb] for the next chunk (the
// host zeroes it with FrameCtl after a frame that did not end).
__device__ __forceinline__ uint32_t bin_hash(uint32_t t) { return t * 0x9E3779B1u + 0x7F4A7C15u; }
__device__ __forceinline__ void bin_chk_add(uint32_t* s_chk, uint32_t a, uint32_t b) {  // whole waves
    a = wave_incl_scan(a);
    b = wave_incl_scan(b);
    if (lane_id() == 63) {
        atomicAdd(&s_chk[0], a);
        atomicAdd(&s_chk[1], b);
    }
}
__device__ __forceinline__ void bin_chk_add_global(uint2* chk, uint32_t a, uint32_t b) {  // whole waves
    a = wave_incl_scan(a);
    b = wave_incl_scan(b);
    if (lane_id() == 63 && (a | b)) {
        atomicAdd(&chk->x, a);
        atomicAdd(&chk->y, b);
    }
}

// Binning partition / band vb: counts of its splats' entries per tile of the band -> bmat row.
// Wide splats (>= wide_tiles box tiles) are queued in LDS (up to wide_cap) and counted by whole
// waves, as k_bin_emit emits them.
// One walk of a unit list (the chunk's, or in chunk 1 also chunk 0's: cw.mode 2): the entries of
// binning partition `part`'s splats in the band added to the LDS counters.  Contains barriers.
template <int NT, bool LISTED>
__device__ __forceinline__ void bin_count_walk(const BinParams& p, uint32_t part, uint32_t t_lo, uint32_t t_hi,
                                               const CutWalk& cw, uint32_t* s_cnt, uint32_t* s_pref, uint32_t* s_tmp,
                                               uint32_t* s_wide, uint32_t& s_nw) {
    const UnitList L = bin_unit_list(p);
    const uint32_t total = bin_slots<NT, LISTED>(p, L, part, s_pref, s_tmp);
    bin_walk<NT>(p, L, part, s_pref, total, cw.mode != 0,
                 [&](uint32_t g, uint32_t pr, uint32_t sj, uint32_t key, float4 q0, float4 q1) {
        TileRect tr;
        if (!rect_unpack(p, pr, sj, tr)) return;
        if (rect_wide(p, tr)) {
            if (p.wlist) return;  // listed: walked below
            const uint32_t qi = atomicAdd(&s_nw, 1u);
            if (qi < p.wide_cap) {
                s_wide[qi] = g;
                return;
            }
        }
        const int m = cw.splat_mode(tr, key);
        if (m < 0) return;
        splat_entries(p, tr, ellipse_of(q0, q1), t_lo, t_hi, key, cw, m, [&](uint32_t t) { atomicAdd(&s_cnt[t - t_lo], 1u); });
    });
    __syncthreads();
    const uint32_t nq = min(s_nw, p.wide_cap);
    for (uint32_t qi = threadIdx.x >> 6; qi < nq; qi += NT / 64)  // wave-uniform
        wide_entries(p, s_wide[qi], t_lo, t_hi, cw, [&](uint32_t t) { atomicAdd(&s_cnt[t - t_lo], 1u); });
    wide_listed<NT>(p, part, t_lo, t_hi, cw, [&](uint32_t t) { atomicAdd(&s_cnt[t - t_lo], 1u); });
}

// Chunk 1's second walk (per-tile cut): chunk 0's units and slots, the entries chunk 0 left out.
__device__ __forceinline__ BinParams cut_pass_params(const BinParams& p) {
    BinParams q = p;
    q.units = p.cut_units;
    q.chunk = 0;
    q.uid_lds = 0;
    return q;
}

// The band's cut bounds into LDS (before the walks' first barrier).
// s_cut: the band's bounds (u16), then the frame's block map (bin_lds_words reserves both).
template <int NT>
__device__ __forceinline__ CutWalk cut_load(const BinParams& p, uint32_t t_lo, uint32_t t_hi, uint16_t* s_cut) {
    uint32_t* s_cutb = (uint32_t*)s_cut + (p.band_tiles + 1) / 2;
    CutWalk cw{s_cut, s_cutb, t_lo, cut_blocks_x(p.tiles_x), (uint32_t)p.tile_row_begin, 0};
    if (!p.cut) return cw;
    for (uint32_t t = t_lo + threadIdx.x; t < t_hi; t += NT) s_cut[t - t_lo] = p.cut[t];
    const uint32_t nb = cut_blocks(p.tiles_x, p.rows);
    for (uint32_t b = threadIdx.x; b < nb; b += NT) s_cutb[b] = p.cutb[b];
    cw.mode = p.chunk == 0 ? 1 : 0;
    return cw;
}

template <int NT, bool LISTED, bool CUT>  // CUT: the frame has the per-tile cut (else none of its code)
__device__ __forceinline__ void bin_count_body(const BinParams& p, uint32_t vb, uint32_t* s_cnt, uint32_t* s_pref, uint32_t* s_tmp,
                                               uint32_t* s_wide, uint32_t* s_nw_p) {
    uint32_t& s_nw = *s_nw_p;
    uint32_t* s_chk = s_nw_p + 1;
    const uint32_t part = vb % p.nparts, band = vb / p.nparts;
    const uint32_t t_lo = band * p.band_tiles, t_hi = min(p.n_tiles, t_lo + p.band_tiles);
    for (uint32_t t = threadIdx.x; t < t_hi - t_lo; t += NT) s_cnt[t] = 0;
    if (threadIdx.x == 0) {
        s_nw = 0;
        s_chk[0] = 0;
        s_chk[1] = 0;
    }
    CutWalk cw = CUT ? cut_load<NT>(p, t_lo, t_hi, (uint16_t*)(s_nw_p + 3)) : CutWalk{nullptr, nullptr, 0u, 0u, 0u, 0};
    bin_count_walk<NT, LISTED>(p, part, t_lo, t_hi, cw, s_cnt, s_pref, s_tmp, s_wide, s_nw);
    if (CUT && p.chunk == 1 && p.cut_units) {
        __syncthreads();  // (every thread has read s_nw and the unit prefix of the first walk)
        if (threadIdx.x == 0) s_nw = 0;
        cw.mode = 2;
        bin_count_walk<NT, true>(cut_pass_params(p), part, t_lo, t_hi, cw, s_cnt, s_pref, s_tmp, s_wide, s_nw);
    }
    __syncthreads();
    uint32_t* row = p.bmat + (uint64_t)part * p.n_tiles;
    uint32_t c1 = 0, c2 = 0;
#pragma unroll 1
    for (uint32_t t = t_lo + threadIdx.x; t < t_hi; t += NT) {
        const uint32_t c = s_cnt[t - t_lo];
        row[t] = c;
        c1 += c;
        c2 += c * bin_hash(t);
    }
#ifndef GS_NO_BIN_CHECK  // (diagnostics builds only: A/B of the invariant's cost)
    bin_chk_add_global(p.bchk + vb, c1, c2);
    (void)s_chk;
#endif
}

// The binning launches size their LDS to the frame: band_tiles counters (one band up to
// kBandTilesMax tiles, so a 4K frame's splats are walked once, not once per 8192-tile band) and
// pref_words of unit prefix (the partition's units at most); a row strip's binning then needs a
// few KB and fits beside the composite of the frame before it.
__device__ __forceinline__ uint32_t* bin_lds() {
    extern __shared__ uint32_t dyn_lds[];
    return dyn_lds;
}
__host__ __device__ inline size_t bin_lds_words(uint32_t band_tiles, uint32_t pref_words, uint32_t wide_cap, uint32_t cut_nb) {
    // (s_nw, s_chk[2], then with the per-tile cut (cut_nb blocks) the band's 16-bit bounds and the block map)
    return (size_t)band_tiles + pref_words + kBinThreads / 64 + wide_cap + 3 + (cut_nb ? (band_tiles + 1) / 2 + cut_nb : 0);
}

template <bool LISTED, bool CUT>  // LISTED: chunk 0 (k_cull's unit list); else chunk 1 (every unit, counts from c1)
__global__ __launch_bounds__(kBinThreads) void k_bin_count(BinParams p) {
    uint32_t* s_cnt = bin_lds();
    uint32_t* s_pref = s_cnt + p.band_tiles;
    uint32_t* s_tmp = s_pref + p.pref_words * (p.uid_lds ? 2u : 1u);  // (then the unit entries)
    uint32_t* s_wide = s_tmp + kBinThreads / 64;
    uint32_t* s_nw = s_wide + p.wide_cap;
    if (p.chunk == 1 && p.ctl->not_done == 0) return;  // chunk 0 saturated every tile
    bin_count_body<kBinThreads, LISTED, CUT>(p, blockIdx.x, s_cnt, s_pref, s_tmp, s_wide, s_nw);
}

// Per tile: exclusive prefix of its column of bmat over the partitions (in place) and the tile's
// total into tbase.  The prefix runs XCD-major: partition p is emitted by workgroup p (and
// p + nparts ...) on XCD p % 8, so ordering the partitions (p % 8, p / 8) gives every XCD one
// contiguous sub-range of each tile's list and its L2 merges the scattered 4-B stores into whole
// lines.  Workgroup = 64 tiles x NW waves; wave w sums ordered partitions [w R, w R + R),
// R = nparts / NW (k_bin_colscan: 8 waves of 32 or 16 rows; k_chunk1's 256-thread phase: 4 of 64 or 32).
constexpr int kColTiles = 64;
static_assert(kBinParts % 64 == 0 && kBinPartsSmall % 64 == 0, "binning partitions split evenly over the 8 XCDs and the column waves");
template <uint32_t NP>
__device__ __forceinline__ uint32_t colscan_part(uint32_t q) {  // q-th of NP partitions in XCD-major order
    return (q % (NP / 8)) * 8 + q / (NP / 8);
}

template <int NW, uint32_t NP>
__device__ __forceinline__ void colscan_rows(const BinParams& p, uint32_t vb, uint32_t (*s_sum)[kColTiles]) {
    constexpr int kColRows = (int)NP / NW;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t = vb * kColTiles + lane;
    const bool ok = t < p.n_tiles;
    uint32_t v[kColRows], sum = 0;
#pragma unroll
    for (int k = 0; k < kColRows; ++k) {
        v[k] = ok ? p.bmat[(uint64_t)colscan_part<NP>(w * kColRows + k) * p.n_tiles + t] : 0u;
        sum += v[k];
    }
    s_sum[w][lane] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int i = 0; i < w; ++i) run += s_sum[i][lane];
    if (ok) {
#pragma unroll
        for (int k = 0; k < kColRows; ++k) {
            p.bmat[(uint64_t)colscan_part<NP>(w * kColRows + k) * p.n_tiles + t] = run;
            run += v[k];
        }
        if (w == NW - 1) p.tbase[t] = run;
    }
    if (w == NW - 1 && p.order) {  // the composite's tile order (chunk 0)
        // XCD band x = tiles [x per, x per + per) is composited by the workgroups on XCD x in order;
        // its tiles with more than heavy_len entries go first (counter order_n[0] of shard x), the
        // rest from the band's end (order_n[1]), so the longest lists do not start in the last,
        // partly filled round of workgroups.  One counter add per (wave, band, class).
        const uint32_t per = (p.n_tiles + 7) >> 3;
        const uint32_t x = ok ? t / per : 8u, band = min(per, p.n_tiles - min(p.n_tiles, x * per));
        const bool heavy = ok && run > p.heavy_len;
        const uint32_t tf = vb * kColTiles, tl = min(tf + kColTiles, p.n_tiles) - 1u;
        for (uint32_t xb = tf / per; xb <= tl / per; ++xb) {  // the bands the wave's tiles fall in
#pragma unroll
            for (int cls = 0; cls < 2; ++cls) {
                const bool mine = ok && x == xb && heavy == (cls == 0);
                const uint64_t bb = __ballot(mine);
                if (!bb) continue;
                uint32_t base = 0;
                if (lane == __builtin_ctzll(bb)) base = atomicAdd(&p.stats[xb].order_n[cls], (uint32_t)__popcll(bb));
                base = __shfl(base, __builtin_ctzll(bb), 64);
                if (mine) {
                    const uint32_t q = base + (uint32_t)__popcll(bb & lanemask_lt());
                    p.order[xb * per + (cls == 0 ? q : band - 1u - q)] = t;
                }
            }
        }
    }
    __syncthreads();
}

template <int NW>
__device__ __forceinline__ void colscan_body(const BinParams& p, uint32_t vb, uint32_t (*s_sum)[kColTiles]) {
    if (p.nparts == kBinPartsSmall) colscan_rows<NW, kBinPartsSmall>(p, vb, s_sum);
    else colscan_rows<NW, kBinParts>(p, vb, s_sum);
}

__global__ __launch_bounds__(512) void k_bin_colscan(BinParams p) {
    __shared__ uint32_t s_sum[8][kColTiles];
    if (p.chunk == 1 && p.ctl->not_done == 0) return;
    colscan_body<8>(p, blockIdx.x, s_sum);
}

// One workgroup: exclusive scan of the tile totals in tile order -> ranges [begin, end) and
// tbase = begin; the chunk's totals (chunk 1, in k_chunk1).

template <int NT>
__device__ __forceinline__ void tile_scan_body(const BinParams& p, uint32_t* s_w) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    constexpr int nw = NT / 64;
    constexpr int ipt = 8;
    const uint32_t cap = p.capacity;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < p.n_tiles; t0 += NT * ipt) {
        uint32_t v[ipt], sum = 0;
#pragma unroll
        for (int k = 0; k < ipt; ++k) {
            const uint32_t t = t0 + (uint32_t)tid * ipt + k;
            v[k] = t < p.n_tiles ? p.tbase[t] : 0u;
            sum += v[k];
        }
        const uint32_t incl = wave_incl_scan(sum);
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint32_t base = carry + incl - sum, total = 0;
        for (int i = 0; i < nw; ++i) {
            if (i < w) base += s_w[i];
            total += s_w[i];
        }
#pragma unroll
        for (int k = 0; k < ipt; ++k) {
            const uint32_t t = t0 + (uint32_t)tid * ipt + k;
            if (t < p.n_tiles) {
                const uint32_t bb = min(base, cap);
                p.ranges[t] = make_uint2(bb, min(base + v[k], cap));
                p.tbase[t] = bb;
            }
            base += v[k];
        }
        carry += total;
        __syncthreads();
    }
    if (tid == 0) {
        p.ctl->k_chunk[p.chunk] = min(carry, cap);
        if (carry > cap) atomicOr(&p.ctl->err, kErrOverflow);
    }
}


// A list entry's store (GS_EMIT_NT: a non-temporal store, A/B builds).
__device__ __forceinline__ void emit_entry(uint32_t* __restrict__ tv, uint32_t pos, uint32_t g) {
#ifdef GS_EMIT_NT
    __builtin_nontemporal_store(g, tv + pos);
#else
    tv[pos] = g;
#endif
}

// The emission's slot loads (GS_EMIT_SLOT_NT: the streaming policy, A/B builds -- the slots are
// read once, the list lines they would evict from L2 are still being filled).
__device__ __forceinline__ uint32_t emit_ld(const uint32_t* a) {
#ifdef GS_EMIT_SLOT_NT
    return __builtin_nontemporal_load(a);
#else
    return *a;
#endif
}
__device__ __forceinline__ float4 emit_ld(const float4* a) {
#ifdef GS_EMIT_SLOT_NT
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(a));
    return make_float4(v[0], v[1], v[2], v[3]);
#else
    return *a;
#endif
}

// One emission walk of a unit list (see bin_count_walk): each entry takes its position from the
// tile's LDS cursor.  stats: the walk adds to the chunk's wide-splat statistics (not chunk 1's
// second walk).
template <int NT, bool LISTED>
__device__ __forceinline__ void bin_emit_walk(const BinParams& p, uint32_t part, uint32_t t_lo, uint32_t t_hi,
                                              const CutWalk& cw, bool stats, uint32_t* s_cur, uint32_t* s_pref,
                                              uint32_t* s_tmp, uint32_t* s_wide, uint32_t& s_nw) {
    const uint32_t cap = p.capacity;
    const UnitList L = bin_unit_list(p);
    const uint32_t total = bin_slots<NT, LISTED>(p, L, part, s_pref, s_tmp);
    // (not bin_walk: with the slot prefetch the emission ran slower, 1.60 -> 1.68 ms at the one-chunk
    // 50 M / 4K frame: its scattered list stores, not its slot loads, bound it)
    for (uint32_t r = threadIdx.x; r < total; r += NT) {
        const uint32_t g = bin_slot(p, L, part, s_pref, r);
        TileRect tr;
        if (!rect_unpack(p, emit_ld(p.srect + g), emit_ld(p.sidx + g), tr)) continue;
        if (rect_wide(p, tr)) {
            if (p.wlist) continue;  // listed: walked below
            const uint32_t qi = atomicAdd(&s_nw, 1u);
            if (qi < p.wide_cap) {
                s_wide[qi] = g;
                continue;
            }
        }
        const uint32_t key = cw.mode ? p.skey[g].x : 0u;
        const int m = cw.splat_mode(tr, key);
        if (m < 0) continue;
        const float4* q = p.crec + 3 * (uint64_t)g;
        splat_entries(p, tr, ellipse_of(emit_ld(q), emit_ld(q + 1)), t_lo, t_hi, key, cw, m, [&](uint32_t t) {
            const uint32_t pos = atomicAdd(&s_cur[t - t_lo], 1u);
            if (pos < cap) emit_entry(p.tvals, pos, g);
        });
    }

    __syncthreads();
    const uint32_t nq = min(s_nw, p.wide_cap);
    if (stats) {  // (the chunk's wide splats: the LDS queues of every workgroup, the listed ones once)
        if (threadIdx.x == 0 && s_nw) atomicAdd(&p.ctl->wide_n[p.chunk], s_nw);
        if (p.wlist && part == 0 && t_lo == 0 && threadIdx.x < kWideShards)
            atomicAdd(&p.ctl->wide_n[p.chunk], p.stats[threadIdx.x].wl_n[p.chunk]);
    }
    for (uint32_t qi = threadIdx.x >> 6; qi < nq; qi += NT / 64) {  // wave-uniform
        const uint32_t g = s_wide[qi];
        wide_entries(p, g, t_lo, t_hi, cw, [&](uint32_t t) {
            const uint32_t pos = atomicAdd(&s_cur[t - t_lo], 1u);
            if (pos < cap) emit_entry(p.tvals, pos, g);
        });
    }
    wide_listed<NT>(p, part, t_lo, t_hi, cw, [&](uint32_t t, uint32_t g) {
        const uint32_t pos = atomicAdd(&s_cur[t - t_lo], 1u);
        if (pos < cap) emit_entry(p.tvals, pos, g);
    });
}

// Wide splats (>= wide_tiles box tiles) are queued in LDS by the thread that meets them and
// emitted row by row by whole waves (lanes over columns); the queue holds kWideQueue splats,
// beyond that the thread emits its splat itself.

// SCAN: tbase holds the tile totals (colscan) and every workgroup scans them itself up to its
// band's end (the tile scan, repeated per workgroup from L2 instead of one more launch on
// the frame's critical path); the workgroups of partition 0 write the band's ranges, the one of
// the last band the chunk's total.  Otherwise tbase holds the list begins (tile_scan_body).
template <int NT, bool SCAN, bool LISTED, bool CUT>
__device__ __forceinline__ void bin_emit_body(const BinParams& p, uint32_t vb, uint32_t* s_cur, uint32_t* s_pref, uint32_t* s_tmp,
                              uint32_t* s_wide, uint32_t* s_nw_p) {
    uint32_t& s_nw = *s_nw_p;
    uint32_t* s_chk = s_nw_p + 1;
    const uint32_t part = vb % p.nparts, band = vb / p.nparts;
    const uint32_t t_lo = band * p.band_tiles, t_hi = min(p.n_tiles, t_lo + p.band_tiles);
    const uint32_t* row = p.bmat + (uint64_t)part * p.n_tiles;
    const uint32_t cap = p.capacity;
    uint32_t d1 = 0, d2 = 0;  // minus the thread's start cursors (the checksum of bin_chk_add)
    if (threadIdx.x == 0) {  // (ordered before bin_chk_add's atomics by the barriers below)
        s_chk[0] = 0;
        s_chk[1] = 0;
    }
    if (SCAN) {
        constexpr int nw = NT / 64, ipt = 8;
        const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
        uint32_t carry = 0;
        for (uint32_t t0 = 0; t0 < t_hi; t0 += NT * ipt) {
            uint32_t v[ipt], sum = 0;
#pragma unroll
            for (int k = 0; k < ipt; ++k) {
                const uint32_t t = t0 + (uint32_t)tid * ipt + k;
                v[k] = t < t_hi ? p.tbase[t] : 0u;
                sum += v[k];
            }
            const uint32_t incl = wave_incl_scan(sum);
            if (lane == 63) s_tmp[w] = incl;
            __syncthreads();
            uint32_t base = carry + incl - sum, tot = 0;
            for (int i = 0; i < nw; ++i) {
                if (i < w) base += s_tmp[i];
                tot += s_tmp[i];
            }
            // A thread's ipt = 8 cursors are contiguous: written as two 16-B words when they lie
            // inside the band and 16-B aligned (lane stride 8 words in single stores is an
            // 8-way LDS bank conflict), one by one at the band's ends.
            const uint32_t tf = t0 + (uint32_t)tid * ipt;
            const bool whole = tf >= t_lo && tf + ipt <= t_hi && ((tf - t_lo) & 3u) == 0;
            uint32_t cur[ipt];
#pragma unroll
            for (int k = 0; k < ipt; ++k) {
                const uint32_t t = tf + k;
                cur[k] = 0;
                if (t >= t_lo && t < t_hi) {
                    const uint32_t bb = min(base, cap);
                    cur[k] = bb + row[t];
                    d1 -= cur[k];
                    d2 -= cur[k] * bin_hash(t);
                    if (!whole) s_cur[t - t_lo] = cur[k];
                    if (part == 0) p.ranges[t] = make_uint2(bb, min(base + v[k], cap));
                }
                base += v[k];
            }
            if (whole) {
                uint4* d = reinterpret_cast<uint4*>(s_cur + (tf - t_lo));
                d[0] = make_uint4(cur[0], cur[1], cur[2], cur[3]);
                d[1] = make_uint4(cur[4], cur[5], cur[6], cur[7]);
            }
            carry += tot;
            __syncthreads();
        }
        if (part == 0 && t_hi == p.n_tiles && threadIdx.x == 0) {
            p.ctl->k_chunk[p.chunk] = min(carry, cap);
            if (carry > cap) atomicOr(&p.ctl->err, kErrOverflow);
        }
    } else {
        for (uint32_t t = t_lo + threadIdx.x; t < t_hi; t += NT) {
            const uint32_t c = p.tbase[t] + row[t];
            s_cur[t - t_lo] = c;
            d1 -= c;
            d2 -= c * bin_hash(t);
        }
        __syncthreads();  // (s_chk zeroed)
    }
#ifndef GS_NO_BIN_CHECK
    bin_chk_add(s_chk, d1, d2);  // the start cursors, now (not held in registers through the walk)
#endif
    if (threadIdx.x == 0) s_nw = 0;
    CutWalk cw = CUT ? cut_load<NT>(p, t_lo, t_hi, (uint16_t*)(s_nw_p + 3)) : CutWalk{nullptr, nullptr, 0u, 0u, 0u, 0};
    bin_emit_walk<NT, LISTED>(p, part, t_lo, t_hi, cw, true, s_cur, s_pref, s_tmp, s_wide, s_nw);
    if (CUT && p.chunk == 1 && p.cut_units) {
        __syncthreads();  // (every thread has read s_nw and the unit prefix of the first walk)
        if (threadIdx.x == 0) s_nw = 0;
        cw.mode = 2;
        bin_emit_walk<NT, true>(cut_pass_params(p), part, t_lo, t_hi, cw, false, s_cur, s_pref, s_tmp, s_wide, s_nw);
    }
    __syncthreads();
#ifndef GS_NO_BIN_CHECK
    // the invariant: every cursor advanced by exactly the tile's count (end - start = n_t)
    uint32_t e1 = 0, e2 = 0;
#pragma unroll 1
    for (uint32_t t = t_lo + threadIdx.x; t < t_hi; t += NT) {
        const uint32_t c = s_cur[t - t_lo];
        e1 += c;
        e2 += c * bin_hash(t);
    }
    bin_chk_add(s_chk, e1, e2);
    const uint2 want = p.bchk[vb];  // (uniform: a scalar load)
    __syncthreads();
    if (threadIdx.x == 0) {
        if (want.x != s_chk[0] || want.y != s_chk[1]) atomicOr(&p.ctl->err, kErrBinning);
        p.bchk[vb] = make_uint2(0u, 0u);  // (zero for the next chunk's count)
    }
#endif
}

template <bool LISTED, bool CUT>
__global__ __launch_bounds__(kBinThreads) void k_bin_emit(BinParams p) {
    uint32_t* s_cur = bin_lds();
    uint32_t* s_pref = s_cur + p.band_tiles;
    uint32_t* s_tmp = s_pref + p.pref_words * (p.uid_lds ? 2u : 1u);  // (then the unit entries)
    uint32_t* s_wide = s_tmp + kBinThreads / 64;
    uint32_t* s_nw = s_wide + p.wide_cap;
    if (p.chunk == 1 && p.ctl->not_done == 0) return;
    bin_emit_body<kBinThreads, true, LISTED, CUT>(p, blockIdx.x, s_cur, s_pref, s_tmp, s_wide, s_nw);
}

// End of a frame: the statistic shards summed into FrameCtl (and zeroed), the saturation
// statistic (depth key of the farthest splat a tile saturated at), then FrameCtl stored into the
// host's pinned slot (mapped, fine-grained) and the sequence number published with a
// system-scope release; the host reads it a frame or two later.  Then FrameCtl is zeroed for the
// next frame.  One wave; lane l sums shard l.
__device__ __forceinline__ void frame_end_body(FrameCtl* ctl, StatShard* stats, FrameCtl* host_ctl, uint32_t* host_seq,
                               uint32_t seq, uint32_t* lds) {
    constexpr uint32_t kWords = sizeof(FrameCtl) / 4;
    constexpr uint32_t kShardWords = sizeof(StatShard) / 4, kStride = kShardWords | 1u;  // odd: no bank conflicts
    static_assert(kWords <= 64 && kStatShards <= 64 && kStatShards >= 8 && kShardWords <= 64, "one wave");
    static_assert(offsetof(StatShard, k_total) == 0 && offsetof(StatShard, n_vis) == 8 &&
                  offsetof(StatShard, key_min_inv) == 12 && offsetof(StatShard, key_max) == 16 &&
                  offsetof(StatShard, n_chunk) == 20 && offsetof(StatShard, sat_key) == 28 &&
                  offsetof(StatShard, sat_hist) == 32, "StatShard word map");
    const uint32_t lane = threadIdx.x;
    FE_MARK(0);
#ifdef GS_KTIME
    {  // diagnostics: latency of one load of FrameCtl, then of one shard word
        const uint32_t a = __hip_atomic_load(&ctl->n_vis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a == 0xdeadbeefu) FE_MARK(7);
        FE_MARK(6);
        const uint32_t b2 = __hip_atomic_load(&stats[lane].n_vis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (b2 == 0xdeadbeefu) FE_MARK(6);
        FE_MARK(7);
    }
#endif
    // the shards into LDS (row = shard) as one flat array of lane-consecutive words, then lane f
    // reduces word f over the shards: a few LDS reads each instead of a shuffle tree per field
    {
        constexpr uint32_t kAll = kStatShards * kShardWords, kPer = (kAll + 63) / 64;
        const uint32_t* sw = (const uint32_t*)stats;
        uint32_t* sz = (uint32_t*)stats;
        uint32_t w[kPer];
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) w[k] = k * 64 + lane < kAll ? sw[k * 64 + lane] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k)
            if (k * 64 + lane < kAll) sz[k * 64 + lane] = 0u;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t i = k * 64 + lane;
            if (i < kAll) lds[(i / kShardWords) * kStride + i % kShardWords] = w[k];
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    FE_MARK(1);
    if (lane == 0) {  // k_total (64-bit)
        unsigned long long kt = 0;
        for (uint32_t j = 0; j < kStatShards; ++j)
            kt += (unsigned long long)lds[j * kStride] | ((unsigned long long)lds[j * kStride + 1] << 32);
        ctl->k_total = kt;
    } else if (lane == offsetof(StatShard, list_max) / 4) {
        uint32_t a = 0;
        for (uint32_t j = 0; j < kStatShards; ++j) a = max(a, lds[j * kStride + lane]);
        ctl->list_max = a;
    } else if (lane >= 2 && lane < 8 + kSatBuckets) {
        const bool is_max = lane == 3 || lane == 4 || lane == 7;  // key_min_inv, key_max, sat_key
        uint32_t a = 0;
        for (uint32_t j = 0; j < kStatShards; ++j) {
            const uint32_t v = lds[j * kStride + lane];
            a = is_max ? max(a, v) : a + v;
        }
        switch (lane) {
            case 2: ctl->n_vis = a; break;
            case 3: ctl->key_min_inv = a; break;
            case 4: ctl->key_max = a; break;
            case 5: ctl->n_chunk[0] = a; break;
            case 6: ctl->n_chunk[1] = a; break;
            case 7: ctl->sat_key = a; break;
            default: ctl->sat_hist[lane - 8] = a; break;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    FE_MARK(2);
    uint32_t* src = (uint32_t*)ctl;
    const uint32_t v = lane < kWords ? src[lane] : 0u;
    if (lane < kWords) ((uint32_t*)host_ctl)[lane] = v;
    // The slot and the sequence word are fine-grained host memory (uncached on the device): the
    // slot's stores complete before the sequence store is issued (vmcnt(0)), and the host reads
    // the slot only after it sees the sequence number.  No system-scope release: that would write
    // the whole L2 back (the frame's dirty lines) for two cache-bypassing stores.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    FE_MARK(3);
    if (lane == 0) __hip_atomic_store(host_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane < kWords) src[lane] = 0u;
    FE_MARK(4);
}

// ============================================================================ k_tile_sort
// One workgroup per tile orders the tile's list by key (the slot itself, or (skey.x, skey.y)),
// ascending; keys are unique.  Lists of up to kTsCap entries are sorted in one round: 1024
// buckets over [kmin, kmax] (a power-of-two width), a counting scatter into LDS, and each
// element's rank = its bucket's start + the smaller keys in its bucket (a bitonic sort in LDS
// when a bucket is heavy).  Longer lists go in rounds of <= kTsCap consecutive keys: a bucket
// histogram of the remaining keys picks the round's upper bound, the round's elements are
// gathered into LDS and sorted the same way.  The output depends only on the keys.
// The shape is a template (TsCfg): chunk 0's lists (a few hundred entries at most tiles) are
// sorted by 128-thread workgroups (TsSmall: 16 KB of LDS and <= 96 VGPRs, five workgroups per
// SIMD pair instead of one 256-thread workgroup per SIMD; 50 -> 40 us at the bench frame);
// chunk 1's lists (thousands of entries in the few tiles that never saturate) by TsBig, as in
// k_chunk1's 256-thread workgroups.
template <int NT_, int IPT_, int BB_, bool VS_ = true>
struct TsCfg {
    static constexpr int NT = NT_;                            // threads
    static constexpr int IPT = IPT_;                          // entries per thread and round
    static constexpr uint32_t Cap = (uint32_t)(NT_ * IPT_);   // entries per round
    static constexpr int BB = BB_;                            // bucket bits
    static constexpr uint32_t Buckets = 1u << BB_;
    static constexpr bool VS = VS_;                           // slots staged in LDS (the bitonic path)
    static_assert(NT_ % 64 == 0 && (1 << BB_) % NT_ == 0, "tile sort shape");
};
using TsBig = TsCfg<256, 8, 10>;
using TsSmall = TsCfg<128, 8, 9>;
// Lists of a few thousand entries (a one-chunk frame at 4K: ~6300 per tile): the whole list's keys
// in LDS, one gather of the keys instead of ts_long's four passes.  Two workgroups per CU, each
// 72 KB of LDS (7168 8-B keys and 4096 bucket counters; no slot staging: the count ranking writes
// the slots from registers, and a list the ranking cannot take -- a bucket of more than kTsHeavy
// keys -- or longer than one round goes to the long-list launch), so one workgroup's phases hide
// the other's latency: with one 128-KB workgroup per CU (1024 threads, 8192 keys and slots) 67 %
// of its wave cycles waited.  One-chunk 50 M / 4K: sort 1.56 -> 1.28 ms at 2 x 512 threads (14
// entries each, 102 VGPRs), frame 7.35 -> 7.11 ms at 2 x 1024 (7 entries each, 56 VGPRs of the 64
// that 8 waves per SIMD allow).
using TsHuge = TsCfg<1024, 7, 12, false>;
constexpr uint32_t kTsHeavy = 64;  // largest bucket ranked by counting

template <class C>
struct TsSharedT {
    unsigned long long k[C::Cap];
    uint32_t v[C::VS ? C::Cap : 1];
    alignas(16) uint32_t cnt[C::Buckets];  // a thread's per = Buckets / NT = 4 (8) counters are one (two) 16-B
                                           // word (ds_read/write_b128, no stride-4 conflicts); after
                                           // the scatter cnt[b] is bucket b's end = bucket b+1's start
    unsigned long long red[2 * (C::NT / 64)];  // block_minmax64's per-wave min | max
    uint32_t tmp[C::NT / 64];              // block_excl_scan's per-wave totals
    uint32_t misc[4];                      // ts_rounds' gather cursor, ts_long's round bounds
    uint32_t any[C::NT / 64];              // block_any's per-wave flags
};

// A workgroup-wide OR with a barrier (as __syncthreads_or, whose library form reads the 3-D
// work-item ids and so kept two more values live through the sort: scratch spills).
template <int NT>
__device__ __forceinline__ bool block_any(bool v, uint32_t* s) {
    const bool w = __any(v);
    if (lane_id() == 0) s[threadIdx.x >> 6] = w ? 1u : 0u;
    __syncthreads();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) r |= s[i];
    return r != 0;  // (no trailing barrier: a caller that writes s again before its next barrier
}                   // alternates between two flag arrays)
using TsShared = TsSharedT<TsBig>;

__device__ __forceinline__ unsigned long long ts_key(const TileSortParams& p, uint32_t g) {
    if (!p.skey) return g;
    const uint2 k = p.skey[g];
    return ((unsigned long long)k.x << 32) | k.y;
}

template <int NT>
__device__ __forceinline__ void block_minmax64(unsigned long long& mn, unsigned long long& mx, unsigned long long* s) {
    for (int d = 32; d >= 1; d >>= 1) {
        mn = min(mn, (unsigned long long)__shfl_xor(mn, d, 64));
        mx = max(mx, (unsigned long long)__shfl_xor(mx, d, 64));
    }
    constexpr int NW = NT / 64;
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) {
        s[w] = mn;
        s[NW + w] = mx;
    }
    __syncthreads();
    mn = s[0];
    mx = s[NW];
#pragma unroll
    for (int i = 1; i < NW; ++i) {
        mn = min(mn, s[i]);
        mx = max(mx, s[NW + i]);
    }
    // no trailing barrier: the per-tile sort writes s again only after several more barriers
}

template <class C>
__device__ __forceinline__ int ts_shift(unsigned long long span) {
    return span == 0 ? 0 : max(0, 64 - (int)__clzll(span) - C::BB);
}

#ifdef GS_TS_TIME  // diagnostics builds only (make diag DIAGFLAGS=-DGS_TS_TIME): the long-list phases
// cycles summed over tiles.  ts_long: minmax, hist, scan, scatter, rounds, heavy; the huge
// shape's one-round lists: load + gather, minmax, count, scan + scatter, rank + write; then tiles, entries
__device__ unsigned long long g_ts_time[8];
#define TS_T(i)                                                                        \
    do {                                                                               \
        if (threadIdx.x == 0) {                                                        \
            const unsigned long long t_ = clock64();                                   \
            atomicAdd(&g_ts_time[(i) - 1], t_ - ts_t0);                                \
            ts_t0 = t_;                                                                \
        }                                                                              \
    } while (0)
#else
#define TS_T(i) \
    do {        \
    } while (0)
#endif

// Sort n <= C::Cap elements held in registers (element j * NT + tid of k/v) with keys in
// [kmin, kmax]; out[rank] = value.  False (nothing written, block-uniform) when a shape without
// slot staging (!C::VS) meets a bucket of more than kTsHeavy keys.
template <class C>
__device__ bool ts_segment(TsSharedT<C>& S, const unsigned long long (&k)[C::IPT], const uint32_t (&v)[C::IPT],
                           uint32_t n, unsigned long long kmin, unsigned long long kmax, uint32_t* __restrict__ out) {
    constexpr int kTsThreads = C::NT, kTsIpt = C::IPT;
    constexpr uint32_t kTsBuckets = C::Buckets;
    const int tid = threadIdx.x;
#ifdef GS_TS_TIME
    constexpr bool kT = C::NT > 256;  // the huge shape's phases
    unsigned long long ts_t0 = clock64();
#endif
    const int s = ts_shift<C>(kmax - kmin);  // S.cnt was zeroed by the caller before block_minmax64's barrier
    uint32_t bk[kTsIpt];
#pragma unroll
    for (int j = 0; j < kTsIpt; ++j) {
        bk[j] = 0;
        if (j * kTsThreads + tid < (int)n) {
            bk[j] = (uint32_t)((k[j] - kmin) >> s);
            atomicAdd(&S.cnt[bk[j]], 1u);
        }
    }
    __syncthreads();
#ifdef GS_TS_TIME
    if (kT) TS_T(3);
#endif
    // a thread's PB consecutive bucket counters as PB / 4 16-B LDS words
    constexpr int PB = (int)(kTsBuckets / kTsThreads), PQ = PB / 4;
    static_assert(PB % 4 == 0, "a thread's bucket counters are whole uint4s");
    uint4 c4[PQ];
    uint32_t sum = 0, big = 0;
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
        c4[q] = reinterpret_cast<const uint4*>(S.cnt)[tid * PQ + q];
        sum += c4[q].x + c4[q].y + c4[q].z + c4[q].w;
        big = max(big, max(max(c4[q].x, c4[q].y), max(c4[q].z, c4[q].w)));
    }
    uint32_t total;
    uint32_t b = block_excl_scan<kTsThreads>(sum, S.tmp, &total);
#pragma unroll
    for (int q = 0; q < PQ; ++q) {  // scatter cursors
        const uint4 st = make_uint4(b, b + c4[q].x, b + c4[q].x + c4[q].y, b + c4[q].x + c4[q].y + c4[q].z);
        reinterpret_cast<uint4*>(S.cnt)[tid * PQ + q] = st;
        b += c4[q].x + c4[q].y + c4[q].z + c4[q].w;
    }
    const bool heavy = block_any<kTsThreads>(big > kTsHeavy, S.any);
    if constexpr (!C::VS)
        if (heavy) return false;
#pragma unroll
    for (int j = 0; j < kTsIpt; ++j) {
        if (j * kTsThreads + tid < (int)n) {
            const uint32_t pos = atomicAdd(&S.cnt[bk[j]], 1u);
            S.k[pos] = k[j];
            if constexpr (C::VS)
                if (heavy) S.v[pos] = v[j];  // the count ranking writes v from registers
        }
    }
    __syncthreads();
#ifdef GS_TS_TIME
    if (kT) TS_T(4);
#endif
    if (!heavy) {
#pragma unroll
        for (int j = 0; j < kTsIpt; ++j) {
            if (j * kTsThreads + tid < (int)n) {
                const uint32_t b0 = bk[j] ? S.cnt[bk[j] - 1] : 0u, b1 = S.cnt[bk[j]];  // bucket bk's [start, end)
                uint32_t r = b0;
                for (uint32_t q = b0; q < b1; ++q) r += S.k[q] < k[j] ? 1u : 0u;
                out[r] = v[j];
            }
        }
    } else if constexpr (C::VS) {  // bitonic sort of the (bucket-ordered) elements, padded to a power of two
        uint32_t P = 1;
        while (P < n) P <<= 1;
        for (uint32_t i = n + tid; i < P; i += kTsThreads) {
            S.k[i] = ~0ull;
            S.v[i] = 0u;
        }
        __syncthreads();
        for (uint32_t size = 2; size <= P; size <<= 1) {
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t i = tid; i < (P >> 1); i += kTsThreads) {
                    const uint32_t lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                    const bool asc = (lo & size) == 0;
                    const unsigned long long a = S.k[lo], bb = S.k[hi];
                    if ((a > bb) == asc) {
                        S.k[lo] = bb;
                        S.k[hi] = a;
                        const uint32_t t = S.v[lo];
                        S.v[lo] = S.v[hi];
                        S.v[hi] = t;
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t i = tid; i < n; i += kTsThreads) out[i] = S.v[i];
    }
    __syncthreads();
#ifdef GS_TS_TIME
    if (kT) TS_T(5);
#endif
    return true;
}

// Sort the n <= C::Cap (key, slot) pairs staged in S.k / S.v (after a barrier) into out[0, n).
template <class C>
__device__ __forceinline__ void ts_lds_round(TsSharedT<C>& S, uint32_t n, uint32_t* __restrict__ out) {
    const int tid = threadIdx.x;
    unsigned long long k[C::IPT];
    uint32_t v[C::IPT];
    unsigned long long mn = ~0ull, mx = 0ull;
#pragma unroll
    for (int j = 0; j < C::IPT; ++j) {
        const uint32_t i = j * C::NT + tid;
        k[j] = 0ull;
        v[j] = 0u;
        if (i < n) {
            k[j] = S.k[i];
            v[j] = S.v[i];
            mn = min(mn, k[j]);
            mx = max(mx, k[j]);
        }
    }
    for (uint32_t b = tid; b < C::Buckets; b += C::NT) S.cnt[b] = 0;  // (ts_segment's counters)
    block_minmax64<C::NT>(mn, mx, S.red);  // (its barrier orders the LDS reads before ts_segment)
    ts_segment<C>(S, k, v, n, mn, mx, out);
}

constexpr int kTsLongU = 4;
// f(i, list[i], key of list[i]) for every i < n, kTsLongU entries per thread in flight.
template <int NT, class F>
__device__ __forceinline__ void ts_long_pass(const TileSortParams& p, const uint32_t* __restrict__ list, uint32_t n, F&& f) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t base = 0; base < n; base += NT * kTsLongU) {
        uint32_t g[kTsLongU];
        unsigned long long key[kTsLongU];
#pragma unroll
        for (int u = 0; u < kTsLongU; ++u) {
            const uint32_t i = base + u * NT + tid;
            g[u] = i < n ? list[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kTsLongU; ++u)
            if (base + u * NT + tid < n) key[u] = ts_key(p, g[u]);
#pragma unroll
        for (int u = 0; u < kTsLongU; ++u) {
            const uint32_t i = base + u * NT + tid;
            if (i < n) f(i, g[u], key[u]);
        }
    }
}

// A list of L > C::Cap entries in rounds of <= C::Cap consecutive keys: per round, a bucket
// histogram of the keys not yet done picks the round's upper bound, the round's elements are
// gathered into LDS and sorted (ts_segment).  Every round re-reads the whole list, so this is
// O(L^2 / Cap): ts_long uses it only for one bucket of more than Cap entries (keys packed in a
// narrow range).  in and out are distinct.
template <class C>
__device__ void ts_rounds(const TileSortParams& p, TsSharedT<C>& S, const uint32_t* __restrict__ in,
                          uint32_t* __restrict__ out, uint32_t L) {
    constexpr int kTsThreads = C::NT;
    constexpr uint32_t kTsCap = C::Cap, kTsBuckets = C::Buckets;
    const int tid = threadIdx.x;
    unsigned long long kmin = ~0ull, kmax = 0ull;
    ts_long_pass<kTsThreads>(p, in, L, [&](uint32_t, uint32_t, unsigned long long key) {
        kmin = min(kmin, key);
        kmax = max(kmax, key);
    });
    block_minmax64<kTsThreads>(kmin, kmax, S.red);
    unsigned long long lo = kmin, hi = 0ull;
    uint32_t done_n = 0;
    constexpr int perb = kTsBuckets / kTsThreads;
    while (done_n < L) {
        const bool bounded = L - done_n > kTsCap;
        if (bounded) {  // hi: the largest bucket boundary with <= kTsCap keys in [lo, hi)
            unsigned long long span = kmax - lo;
            for (;;) {
                const int s = ts_shift<C>(span);
                for (uint32_t b = tid; b < kTsBuckets; b += kTsThreads) S.cnt[b] = 0;
                __syncthreads();
                ts_long_pass<kTsThreads>(p, in, L, [&](uint32_t, uint32_t, unsigned long long key) {
                    if (key >= lo && key - lo <= span) atomicAdd(&S.cnt[(uint32_t)((key - lo) >> s)], 1u);
                });
                __syncthreads();
                static_assert(perb % 4 == 0, "a thread's bucket counters are whole uint4s");
                uint32_t c[perb], sum = 0;
#pragma unroll
                for (int q = 0; q < perb / 4; ++q) {
                    const uint4 c4 = reinterpret_cast<const uint4*>(S.cnt)[tid * (perb / 4) + q];
                    c[4 * q] = c4.x;
                    c[4 * q + 1] = c4.y;
                    c[4 * q + 2] = c4.z;
                    c[4 * q + 3] = c4.w;
                    sum += c4.x + c4.y + c4.z + c4.w;
                }
                uint32_t total;
                uint32_t run = block_excl_scan<kTsThreads>(sum, S.tmp, &total);
                uint32_t fit = 0;
#pragma unroll
                for (int q = 0; q < perb; ++q) {
                    run += c[q];
                    fit += run <= kTsCap ? 1u : 0u;
                }
                uint32_t m;
                block_excl_scan<kTsThreads>(fit, S.tmp, &m);  // buckets whose prefix fits (a prefix of them)
                if (m >= 1) {
                    hi = lo + ((unsigned long long)m << s);
                    break;
                }
                span = (1ull << s) - 1ull;  // the first bucket alone overflows: narrow to it (s > 0)
            }
        }
        if (tid == 0) S.misc[0] = 0;
        __syncthreads();
        ts_long_pass<kTsThreads>(p, in, L, [&](uint32_t, uint32_t g, unsigned long long key) {
            if (key >= lo && (!bounded || key < hi)) {
                const uint32_t pos = atomicAdd(&S.misc[0], 1u);
                S.k[pos] = key;
                S.v[pos] = g;
            }
        });
        __syncthreads();
        const uint32_t nc = S.misc[0];
        ts_lds_round<C>(S, nc, out + done_n);
        done_n += nc;
        lo = hi;
    }
}


// A list of L > C::Cap entries (a long list: a tile of a frame whose tiles do not saturate, or chunk
// 1's), in time linear in L (the rounds of ts_rounds re-read the whole list each, so
// a one-chunk 50 M / 4K frame spent 8.2 ms in this kernel):
//   1. the key range; 2. a histogram of 256 buckets of equal key width over it; 3. their starts;
//   4. a counting scatter of the slots into `out`, grouped by bucket (unordered within one);
//   5. runs of consecutive buckets of <= C::Cap entries in all, each loaded from `out`, sorted in
//      LDS (ts_segment) and written back in place.  A single bucket of more than C::Cap entries
//      is copied to `in` (free once the scatter has read it) and sorted by ts_rounds into `out`.
// Four reads of the list and its keys per entry, one write of the scatter and one of the sort.
constexpr int kTsLongBB = 8;
constexpr uint32_t kTsLongBuckets = 1u << kTsLongBB;
static_assert(kTsLongBuckets <= (uint32_t)kBmatRows, "the long-list scratch is the binning matrix (kBmatRows per tile)");
__device__ __forceinline__ unsigned long long uniform64(unsigned long long x) {
    return ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}


template <class C>
__device__ void ts_long(const TileSortParams& p, TsSharedT<C>& S, uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                        uint32_t L, uint32_t* __restrict__ ends) {  // ends: kTsLongBuckets words of global scratch
    constexpr int NT = C::NT;
    constexpr uint32_t Cap = C::Cap;
    constexpr int PB = (int)kTsLongBuckets / NT;  // buckets per thread (consecutive)
    static_assert(PB >= 1 && kTsLongBuckets % NT == 0 && kTsLongBuckets <= C::Buckets, "long-list buckets");
    const int tid = threadIdx.x;
#ifdef GS_TS_TIME
    unsigned long long ts_t0 = clock64();
    if (tid == 0) {
        atomicAdd(&g_ts_time[6], 1ull);
        atomicAdd(&g_ts_time[7], (unsigned long long)L);
    }
#endif
    unsigned long long kmin = ~0ull, kmax = 0ull;
    // The passes over the list are gathers behind list loads (latency-bound, VERDICT r03 item 5:
    // one entry in flight per thread kept the waves 85 % waiting): kTsLongU entries per thread
    // per step, every list load issued before the first key gather.
    ts_long_pass<NT>(p, in, L, [&](uint32_t, uint32_t, unsigned long long key) {
        kmin = min(kmin, key);
        kmax = max(kmax, key);
    });
    for (uint32_t b = tid; b < kTsLongBuckets; b += NT) S.cnt[b] = 0;
    block_minmax64<NT>(kmin, kmax, S.red);  // (its barrier also orders the zeroed counters)
    kmin = uniform64(kmin);  // (block-uniform values in scalar registers: the rounds below hold
    kmax = uniform64(kmax);  // the full set of a round's keys in vector registers)
    TS_T(1);
    const unsigned long long span = kmax - kmin;
    const int sh = __builtin_amdgcn_readfirstlane(span == 0 ? 0 : max(0, 64 - (int)__clzll(span) - kTsLongBB));
    ts_long_pass<NT>(p, in, L, [&](uint32_t, uint32_t, unsigned long long key) {
        atomicAdd(&S.cnt[(uint32_t)((key - kmin) >> sh)], 1u);
    });
    __syncthreads();
    TS_T(2);
    {
        uint32_t c[PB], sum = 0;
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            c[q] = S.cnt[tid * PB + q];
            sum += c[q];
        }
        uint32_t total;
        uint32_t run = block_excl_scan<NT>(sum, S.tmp, &total);  // (its barriers order the reads above)
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            S.cnt[tid * PB + q] = run;  // scatter cursor = the bucket's start
            run += c[q];
            ends[tid * PB + q] = run;   // (the rounds read them back: registers would spill)
        }
    }
    __syncthreads();
    TS_T(3);
    ts_long_pass<NT>(p, in, L, [&](uint32_t, uint32_t g, unsigned long long key) {
        out[atomicAdd(&S.cnt[(uint32_t)((key - kmin) >> sh)], 1u)] = g;
    });
    __syncthreads();  // (the scatter's stores are visible to the workgroup: one CU, one L1)
    TS_T(4);
    uint32_t pos0 = 0;
    bool heavy = false;
    while (pos0 < L) {
        // m = buckets whose end is <= pos0 + Cap (a prefix: the ends ascend); this round is
        // [pos0, end[m - 1]), or bucket m alone when it holds more than Cap entries
        const uint32_t lim = pos0 + Cap;
        uint32_t end[PB], mine = 0;
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            end[q] = ends[tid * PB + q];
            mine += end[q] <= lim ? 1u : 0u;
        }
        uint32_t m;
        block_excl_scan<NT>(mine, S.tmp, &m);
        m = __builtin_amdgcn_readfirstlane(m);
        // the owner of bucket m - 1 (m >= 1) publishes its end; of bucket m, its end (a heavy bucket)
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            const uint32_t b = (uint32_t)(tid * PB + q);
            if (m >= 1 && b == m - 1) S.misc[1] = end[q];
            if (b == m) S.misc[2] = end[q];
        }
        if (m == 0 && tid == 0) S.misc[1] = 0;
        __syncthreads();
        uint32_t pos1 = __builtin_amdgcn_readfirstlane(S.misc[1]);
        const uint32_t heavy_end = __builtin_amdgcn_readfirstlane(S.misc[2]);
        if (pos1 > pos0) {  // one round: staged in LDS, sorted, written back in place
            const uint32_t n = pos1 - pos0;
            ts_long_pass<NT>(p, out + pos0, n, [&](uint32_t i, uint32_t g, unsigned long long key) {
                S.k[i] = key;
                S.v[i] = g;
            });
            __syncthreads();
            ts_lds_round<C>(S, n, out + pos0);  // (ends with a barrier)
        } else {  // bucket m holds more than Cap entries: left for the pass below
            pos1 = heavy_end;
            heavy = true;
        }
        pos0 = pos1;
    }
    TS_T(5);
    if (!heavy) return;
    // the buckets of more than Cap entries, one at a time: copied to `in`, sorted by ts_rounds
    for (uint32_t b = 0; b < kTsLongBuckets; ++b) {
        const uint32_t e0 = __builtin_amdgcn_readfirstlane(b ? ends[b - 1] : 0u);
        const uint32_t e1 = __builtin_amdgcn_readfirstlane(ends[b]);
        if (e1 - e0 <= Cap) continue;
        for (uint32_t i = e0 + tid; i < e1; i += NT) in[i] = out[i];
        __syncthreads();
        ts_rounds<C>(p, S, in + e0, out + e0, e1 - e0);
        __syncthreads();
    }
    TS_T(6);
}

template <class C>
__device__ __forceinline__ void tile_sort_tile(const TileSortParams& p, const int tile, TsSharedT<C>& S);

// Workgroup item vb -> tile: XCD-banded as k_composite, or the compact list of chunk 1's tiles
// (c1tiles set).
template <class C>
__device__ __forceinline__ void tile_sort_body(const TileSortParams& p, uint32_t vb, TsSharedT<C>& S) {
    int tile;
    if (C::NT == TsBig::NT && p.c1tiles) {  // (chunk 1 runs k_tile_sort_big only)
        if (vb >= *p.c1_n) return;
        tile = __builtin_amdgcn_readfirstlane((int)p.c1tiles[vb]);
    } else {
        const int per = (p.n_tiles + 7) >> 3;
        tile = (int)(vb & 7) * per + (int)(vb >> 3);
        if (tile >= p.n_tiles) return;
        if (p.done && p.done[tile]) return;
    }
    tile_sort_tile<C>(p, tile, S);  // one inlined copy
}

template <class C>
__device__ __forceinline__ void tile_sort_tile(const TileSortParams& p, const int tile, TsSharedT<C>& S) {
    constexpr int kTsThreads = C::NT, kTsIpt = C::IPT;
    constexpr uint32_t kTsCap = C::Cap, kTsBuckets = C::Buckets;
    const uint2 range = p.ranges[tile];
    const uint32_t L = range.y - range.x;
    if (L == 0) return;
    const int tid = threadIdx.x;
    if (L > kListMaxMin && tid == 0 && p.stats) atomicMax(&p.stats[tile % kStatShards].list_max, L);
    if constexpr (!C::VS) {  // (the host always gives this shape a long-list launch)
        if (L > kTsCap) {  // left to the long-list launch (ts_long at 256 threads)
            if (tid == 0) p.long_tiles[atomicAdd(p.long_n, 1u)] = (uint32_t)tile;
            return;
        }
    }
    const uint32_t* __restrict__ in = p.in + range.x;
    uint32_t* __restrict__ out = p.out + range.x;
    unsigned long long k[kTsIpt];
    uint32_t v[kTsIpt];
    if (L == 1) {
        if (tid == 0) out[0] = in[0];
        return;
    }
    if (L <= kTsCap) {
#ifdef GS_TS_TIME
        constexpr bool kT = C::NT > 256;
        unsigned long long ts_t0 = clock64();
        if (kT && tid == 0) {
            atomicAdd(&g_ts_time[6], 1ull);
            atomicAdd(&g_ts_time[7], (unsigned long long)L);
        }
#endif
        unsigned long long mn = ~0ull, mx = 0ull;
#pragma unroll
        for (int j = 0; j < kTsIpt; ++j) {  // every list load in flight before the first key gather
            const uint32_t i = j * kTsThreads + tid;
            v[j] = i < L ? in[i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kTsIpt; ++j) {
            k[j] = 0ull;
            if (j * kTsThreads + tid < L) {
                k[j] = ts_key(p, v[j]);
                mn = min(mn, k[j]);
                mx = max(mx, k[j]);
            }
        }
#ifdef GS_TS_TIME
        if (kT) {
            __syncthreads();  // (diagnostics: every wave's gathers landed)
            TS_T(1);
        }
#endif
        for (uint32_t b = tid; b < kTsBuckets; b += kTsThreads) S.cnt[b] = 0;  // (ts_segment's counters)
        block_minmax64<kTsThreads>(mn, mx, S.red);
#ifdef GS_TS_TIME
        if (kT) TS_T(2);
#endif
        if (!ts_segment<C>(S, k, v, L, mn, mx, out) && tid == 0)  // a heavy bucket: the long-list launch
            p.long_tiles[atomicAdd(p.long_n, 1u)] = (uint32_t)tile;
        return;
    }
    if constexpr (C::VS) ts_long<C>(p, S, p.in + range.x, out, L, p.scratch + (size_t)tile * kTsLongBuckets);
}

__global__ __launch_bounds__(TsSmall::NT, 5) void k_tile_sort(TileSortParams p) {
    __shared__ TsSharedT<TsSmall> S;
    tile_sort_body<TsSmall>(p, blockIdx.x, S);
}
__global__ __launch_bounds__(TsHuge::NT, 2 * TsHuge::NT / 256) void k_tile_sort_huge(TileSortParams p) {
    __shared__ TsSharedT<TsHuge> S;
    tile_sort_body<TsHuge>(p, blockIdx.x, S);
}
__global__ __launch_bounds__(TsBig::NT, 4) void k_tile_sort_big(TileSortParams p) {
    __shared__ TsSharedT<TsBig> S;
    // (chunk 1: workgroup j takes entry j of the compact tile list, the rest return at once; a
    // grid-stride loop over the list would spill: the sort body is at the 128-VGPR bound)
    tile_sort_body<TsBig>(p, blockIdx.x, S);
}
// The same over a compact tile list (chunk 1's unsaturated tiles, the huge shape's long lists)
// with a grid of a few workgroups per CU striding it: one workgroup per possible entry cost a
// full grid of mostly empty workgroups (8160 at 1080p: ~25 us of dispatch for tens of tiles).
__global__ __launch_bounds__(TsBig::NT, 2) void k_tile_sort_list(TileSortParams p) {
    __shared__ TsSharedT<TsBig> S;
    const uint32_t nl = *p.c1_n;
    for (uint32_t j = blockIdx.x; j < nl; j += gridDim.x) {
        tile_sort_tile<TsBig>(p, __builtin_amdgcn_readfirstlane((int)p.c1tiles[j]), S);
        __syncthreads();
    }
}

// ============================================================================ k_composite
// Workgroup = one 16x16 tile, 2 waves; wave h owns the 8-wide column half h, and each lane owns
// two pixels of one column, 8 rows apart (rows r and r + 8), so every per-splat cost (LDS reads,
// x terms, loop control) is shared by two pixels and the y-dependent math runs as packed float2.
// The tile's depth-ordered list is consumed in batches of 128 splats: every thread gathers one
// 48-B composite record into registers (the next batch is issued before the current one is
// blended), parks it in a double-buffered LDS stage and marks which halves its pixel box
// touches; ballots compact the marks into per-half index lists (one 64-entry segment per
// producing wave, so batch order is kept without another barrier).  Each wave walks only its
// half's list and stops once its 128 pixels are saturated.  Per pixel, fs_main's
// alpha = saturate(op * exp(-dot(uv,uv))), discarded below 1/255 and outside |u|,|v| <= 2, is
// blended front to back with the reference's blend state (src/simple_render.ts:169-200, :455-471):
//   FP32        transmittance form: C += col * alpha * T, T *= 1 - alpha; no splat is accepted
//               once T < t_min;
//   FP16_TARGET dst = src * (1 - dst.a) + dst rounded to fp16 after every blend (rgba16float).
// Chunked frames: mode kCompFirst marks saturated tiles done (and writes them out) and parks the
// per-pixel state of the others; kCompSecond resumes those from the state with chunk 1's list.
constexpr int kCompBatch = 128;

// A tile chunk 0 left unsaturated, as its bit for chunk 1's rectangle tests (ProjParams::umask).
__device__ __forceinline__ void umask_set(const CompositeParams& p, int tile) {
    const uint32_t x = (uint32_t)(tile % p.tiles_x), y = (uint32_t)(tile / p.tiles_x);
    atomicOr(&p.umask[y * p.umask_w + (x >> 5)], 1u << (x & 31u));
}

#if defined(GS_COMP_PHASE) && !defined(GS_COMP_TIME)
#define GS_COMP_TIME 1
#endif
#if defined(GS_COMP_STATS) || defined(GS_COMP_TIME)
#define GS_COMP_DIAG 1
#endif
#ifdef GS_COMP_PHASE  // diagnostics: per-wave shader cycles in g_comp_cnt[tile][wave][0..4]:
                      // first batch (load, park, barrier), walks, parks, barriers, gathers
#define CP_T0(v) const unsigned long long v = clock64()
#define CP_ADD(i, v) (dg[i] += clock64() - v)
#else
#define CP_T0(v) do { } while (0)
#define CP_ADD(i, v) do { } while (0)
#endif
#ifdef GS_COMP_DIAG
// diagnostics builds only (make diag): counters of k_composite's per-wave blends (GS_COMP_STATS),
// per-tile wall-clock spans (GS_COMP_TIME or GS_COMP_STATS)
__device__ unsigned long long g_comp_cnt[16384][2][8];  // per tile and wave (plain stores: no atomics)
__device__ unsigned long long g_comp_time[16384][3];  // per tile: start | n << 40, end | blends << 40, hw ids
#endif
// Chunk 0 of frames with at most this many tiles is composited by k_composite_q (4 waves per
// tile).  0: never — with the lockstep quarter lists k_composite is faster for row strips too
// (G = 8 strip 0.087 -> 0.082 ms); k_composite_q stays chunk 1's kernel (a few long lists).
#ifndef GS_QUARTER_TILES
#define GS_QUARTER_TILES 0
#endif
constexpr int kQuarterTiles = GS_QUARTER_TILES;  // at most this many tiles: k_composite_q
typedef float f2 __attribute__((ext_vector_type(2)));
#ifndef GS_COMP_WAVES
#define GS_COMP_WAVES 5
#endif

// Row bands per half-tile wave (lists walked in lockstep, see below): 2 (8x8 quarters, lane
// halves) or 4 (8x4 bands, one per ds_read_b128 lane group).  Four measured slower at the bench
// frame (composite 202 -> 214 us: four band tests per entry in the park step, and the larger list
// area leaves 9 instead of 10 workgroups per CU), so two is the default.
#ifndef GS_COMP_BANDS
#define GS_COMP_BANDS 2
#endif
constexpr int kBands = GS_COMP_BANDS;  // the default (CompositeParams::bands chooses per frame)
static_assert(kBands == 2 || kBands == 4, "row bands per wave");
// Lane l of a wave -> (row band, index in the band).  Two bands: lanes 0-31 and 32-63.  Four: the
// lane groups a ds_read_b128 serves in one LDS cycle each, {0-3,12-15,20-27}, {4-11,16-19,28-31}
// and the same +32 (MI355X_MICROARCH.md, LDS): quads q = (l & 31) >> 2 in {1,2,4,7} form the second
// group (mask 0x96); a quad's index base in its group is 4 (q >> 1).
template <int BANDS>
__device__ __forceinline__ void band_lane(int l, int& band, int& idx) {
    if (BANDS == 2) {
        band = l >> 5;
        idx = l & 31;
    } else {
        const int q = (l & 31) >> 2;
        band = ((0x96 >> q) & 1) + 2 * (l >> 5);
        idx = ((q >> 1) << 2) | (l & 3);
    }
}

// Lanes and lists.  Wave h owns the 8-wide column half h of the tile; its lanes 0-31 hold the
// top 8x8 quarter (rows 0-7) and lanes 32-63 the bottom one, two vertically adjacent pixels per
// lane, blended as a packed float2.  Each quarter has its own list (the splats whose ellipse
// reaches the quarter: its columns within the quarter's 8 rows), and the two lists are walked in
// lockstep: at step k lanes 0-31 blend top[k] and lanes 32-63 bottom[k] (a null record past a
// list's end).  A ds_read_b128 serves lanes {0-31} and {32-63} in separate lane groups, so two
// distinct addresses per wave cost what one broadcast address does: a step costs what a step over
// one half-tile list did, and a splat that reaches only one quarter no longer costs a whole step
// of the wave (max(|top|, |bottom|) steps instead of |top u bottom|).
// List split (SEG > 1, round 5): a workgroup of SEG wave pairs composites one tile; pair s walks
// the s-th of nseg = clamp(n / kSegMin, 1, SEG) equal, contiguous segments of the tile's list
// (a function of the list only: run-to-run deterministic) with its own staging, pair 0 from the
// tile's incoming state and pair s > 0 from (C = 0, T = 1); afterwards pair 0 merges in list
// order, C += T C_s, T *= T_s while T >= t_min.  A pair stops once its own pixels' T < t_min, so
// after the tile's true saturation point a later pair may still add contributions the one-chain
// walk would skip: each is below t_min x colour.  The image therefore meets the fp32 oracle's bar
// (and the WebGPU stand-in's) but is not bit-identical to the one-chain walk (SEG = 1, or any tile
// whose list is shorter than 2 kSegMin, which is).  It divides a tile's serial chain -- what a
// frame with fewer tiles than the chip holds at once (a row strip, chunk 1's unsaturated tiles)
// is bound by -- by nseg.  FP16_TARGET (rgba16float rounding after every blend) has no such
// merge: SEG is 1 there.
constexpr uint32_t kSegMin = 96;  // shortest segment worth a pair of waves

// composite_tile's LDS (the kernel declares it, so a kernel can share it with another phase)
template <int SEG, int BANDS>
struct CompShared {
    // staged record per batch entry: [0] c0u, c0v, a, b  [1] c, d, log2(op), slot (bits)
    // [2] r, g, b, -   with u = a lx + b ly + c0u, v = c lx + d ly + c0v in tile-local pixels;
    // entry kCompBatch of buffer 1 is the null record (log2 op = -inf: alpha 0, nothing blended)
    float4 sR[SEG][2][kCompBatch + 1][3];
    uint16_t sL[SEG][2][2][BANDS][kCompBatch];  // per half, per row band: LDS byte offsets of the
                                                // staged records in sR (segment = producing wave,
                                                // tail: the null record)
    uint32_t sN[SEG][2][2][BANDS][2];           // per half, band, producing wave: list length
    uint32_t s_sat[SEG];                        // depth key of the splat that saturated the pair's last wave
    uint32_t s_any[3][2 * SEG];                 // block_any flags: batches by parity, the tile's end
    uint32_t s_qsat;                            // SEG > 1: the segment in which the merged tile saturated
};

template <bool FP16_TARGET, int SEG, int BANDS>
__device__ __forceinline__ void composite_tile(const CompositeParams& p, const int tile, CompShared<SEG, BANDS>& S) {
    static_assert(SEG == 1 || (!FP16_TARGET && (SEG == 2 || SEG == 4)), "list split: fp32 accumulation, 2 or 4 pairs");
    static_assert(BANDS == 2 || BANDS == 4, "row bands per wave");
    constexpr int kBands = BANDS, kBandRows = 16 / BANDS;
    constexpr int NT = 128 * SEG;
    auto& sR = S.sR;
    auto& sL = S.sL;
    auto& sN = S.sN;
    auto& s_sat = S.s_sat;
    auto& s_any = S.s_any;
    uint32_t& s_qsat = S.s_qsat;
    const int tid = threadIdx.x;
    if (p.mode == kCompSecond && p.done[tile]) return;
#ifdef GS_COMP_DIAG
    const unsigned long long t_begin = wall_clock64();
#endif
    const int sg = SEG > 1 ? __builtin_amdgcn_readfirstlane(tid >> 7) : 0;  // the pair's segment
    const int ptid = SEG > 1 ? (tid & 127) : tid;                            // thread within the pair
    const int h = __builtin_amdgcn_readfirstlane(ptid >> 6), lane = tid & 63;
    int qr, m;  // the lane's row band and its position in the band (band_lane)
    band_lane<BANDS>(lane, qr, m);
    const int tx = tile % p.tiles_x, ty = tile / p.tiles_x + p.tile_row_begin;
    const int tx0 = tx * kTile, ty0 = ty * kTile;
    const int px = tx0 + h * 8 + (m & 7), py = ty0 + qr * kBandRows + 2 * (m >> 3);  // pixels (px, py), (px, py + 1)
    const bool in0 = px < p.W && py < p.H, in1 = px < p.W && py + 1 < p.H;
    const float lx = (float)(px - tx0) + 0.5f;  // tile-local pixel centres
    const f2 ly = {(float)(py - ty0) + 0.5f, (float)(py - ty0) + 1.5f};
    const uint2 range0 = p.ranges[tile];
    // the pair's segment of the list (the whole list when SEG = 1)
    uint32_t nseg = 1;
    uint2 range = range0;
    if (SEG > 1) {
        const uint32_t nall = range0.y - range0.x;
        nseg = min((uint32_t)SEG, max(1u, nall / kSegMin));
        nseg = __builtin_amdgcn_readfirstlane(nseg);
        const uint32_t s = min((uint32_t)sg, nseg);
        range.x = range0.x + (uint32_t)(((uint64_t)nall * s) / nseg);
        range.y = sg < (int)nseg ? range0.x + (uint32_t)(((uint64_t)nall * (s + 1)) / nseg) : range.x;
    }
    const float4* __restrict__ rec = p.rec;
    const uint32_t* __restrict__ tvals = p.tvals;
    const float L = 2.0f * kSqrtLog2e, amin = 1.0f / 255.0f, t_min = p.t_min;
    // sR[sg][1][kCompBatch]
    const uint32_t kNullOff = (uint32_t)((((sg * 2 + 1) * (kCompBatch + 1)) + kCompBatch) * 3 * 16);
    // the lane's pixel coordinates, recomputed where needed after the blend loop from the lane id
    // (mbcnt: not folded into the values computed before the loop, so none of them is held
    // across it — held, they were spilled)
    auto lane_pix = [&](int& x, int& y) {
        const int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        int bb, mm;
        band_lane<BANDS>(l, bb, mm);
        x = tx0 + h * 8 + (mm & 7);
        y = ty0 + bb * kBandRows + 2 * (mm >> 3);
    };
    // parked-state index of the lane's pixels
    auto pix_of = [&](int r) -> uint64_t { return (uint64_t)(py + r) * p.W + px; };
    auto pix_late = [&](int r) -> uint64_t {
        int x, y;
        lane_pix(x, y);
        return (uint64_t)(y + r) * p.W + x;
    };
    f2 cr = {0.0f, 0.0f}, cg = {0.0f, 0.0f}, cb = {0.0f, 0.0f};
    f2 T = {1.0f, 1.0f};   // FP32: transmittance
    f2 ca = {0.0f, 0.0f};  // FP16_TARGET: dst.a
#ifdef GS_COMP_DIAG
    unsigned long long dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    if (p.mode == kCompSecond && sg == 0) {  // (pairs s > 0 start their segment from C = 0, T = 1)
        if (in0) {
            const float4 st = p.state[pix_of(0)];
            cr.x = st.x; cg.x = st.y; cb.x = st.z;
            if (FP16_TARGET) ca.x = st.w; else T.x = st.w;
        }
        if (in1) {
            const float4 st = p.state[pix_of(1)];
            cr.y = st.x; cg.y = st.y; cb.y = st.z;
            if (FP16_TARGET) ca.y = st.w; else T.y = st.w;
        }
    }
    if (!FP16_TARGET) {  // the pixel test reads liveness from T: pixels off the image never blend
        if (!in0) T.x = -1.0f;
        if (!in1) T.y = -1.0f;
    }
    bool live0 = in0 && (FP16_TARGET ? ca.x < 1.0f : T.x >= t_min);
    bool live1 = in1 && (FP16_TARGET ? ca.y < 1.0f : T.y >= t_min);
    bool wave_live = __any(live0 || live1);

    const uint32_t n = range.y - range.x;
    // batches: the longest segment's (every pair runs the same barriers)
    const uint32_t nmax = SEG > 1 ? (range0.y - range0.x + nseg - 1) / nseg : n;
    const uint32_t nb = (nmax + kCompBatch - 1) / kCompBatch;
    float4 ga, gb;  // the next batch's records in flight: geometry only (colour at park time)
    uint32_t gs_ = 0;
    bool gv = false;
    // the batch's slot ids are loaded one batch ahead of its records, so the record loads of batch
    // b + 1 do not wait for a tile-list load first
    uint32_t sl_next = 0;
    auto load_slots = [&](uint32_t batch) {
        const uint32_t e = range.x + batch * kCompBatch + ptid;
        if (e < range.y) sl_next = tvals[e];
    };
    auto gather = [&](uint32_t batch) {
        const uint32_t e = range.x + batch * kCompBatch + ptid;
        gv = e < range.y;
        if (gv) {
            gs_ = sl_next;
            const float4* r = rec + 3 * (uint64_t)gs_;
            ga = r[0];
            gb = r[1];
        }
        if (batch + 1 < nb) load_slots(batch + 1);
    };
    auto park = [&](int buf) {
        // offsets of the axes' linear forms at the tile origin (explicit roundings, see blend)
        const float4 gc = gv ? rec[3 * (uint64_t)gs_ + 2] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float cxr = ga.x - (float)tx0, cyr = ga.y - (float)ty0;
        const float c0u = -__builtin_fmaf(cxr, ga.z, cyr * ga.w);
        const float c0v = -__builtin_fmaf(cxr, gb.x, cyr * gb.y);
        // staged as [b, a, d, c] [r, c0u, g, c0v] [b, log2 op, slot, key]: every value a packed
        // op broadcasts sits in the low half of an aligned register pair (no moves in the blend;
        // log2 op is broadcast from a high half by op_sel)
        sR[sg][buf][ptid][0] = make_float4(ga.w, ga.z, gb.y, gb.x);
        sR[sg][buf][ptid][1] = make_float4(gc.x, c0u, gc.y, c0v);
        sR[sg][buf][ptid][2] = make_float4(gc.z, gb.z, __uint_as_float(gs_), gc.w);
        // the splat's pixel columns within each quarter's 8 rows (ellipse; the binning's margins),
        // against both column halves: 4 lists, each compacted per producing wave by a ballot; the
        // slots past a list's end hold the null record
        const Ellipse el = ellipse_of(ga, gb);
#pragma unroll
        for (int hy = 0; hy < kBands; ++hy) {
            uint32_t ul = 0u, uh = 0u;
            // rows relative to the centre from the tile-relative centre (literal row offsets: no
            // per-tile float constants held across the blend loop)
            const bool cols = gv && ellipse_cols_dy(el, (0.5f + (float)(kBandRows * hy)) - cyr,
                                                    ((float)kBandRows - 0.5f + (float)(kBandRows * hy)) - cyr, ul, uh);
#pragma unroll
            for (int hx = 0; hx < 2; ++hx) {
                const int qx = tx0 + hx * 8;
                const bool hit = cols && (int)ul <= qx + 7 && (int)uh >= qx;
                const uint64_t b = __ballot(hit);
                const uint32_t cnt = (uint32_t)__popcll(b);
                uint16_t* Lq = &sL[sg][buf][hx][hy][h * 64];
                if (hit) Lq[__popcll(b & lanemask_lt())] = (uint16_t)((((sg * 2 + buf) * (kCompBatch + 1) + ptid) * 3) * 16);
                if ((uint32_t)lane >= cnt) Lq[lane] = (uint16_t)kNullOff;
                if (lane == 0) sN[sg][buf][hx][hy][h] = cnt;
            }
        }
    };
    const char* const sRb = (const char*)&sR[0][0][0][0];
    auto blend = [&](uint32_t off) {
        const float4 A = *(const float4*)(sRb + off);
        const float4 B = *(const float4*)(sRb + off + 16);
        const float4 C = *(const float4*)(sRb + off + 32);
        // staged as [b, a, d, c] [r, c0u, g, c0v] [b, log2 op, slot, key]: each colour channel a
        // packed fma broadcasts is the low half of an aligned register pair (no moves)
        const float c0u = B.y, c0v = B.w, l2op = C.y, kr = B.x, kg = B.z, kb = C.x;
        // every rounding is spelled out (explicit fma or contraction off), so each inlined copy of
        // this blend rounds identically and the image cannot depend on where batches split
        const f2 u = __builtin_elementwise_fma(ly, (f2)A.x, (f2)__builtin_fmaf(lx, A.y, c0u));
        const f2 v = __builtin_elementwise_fma(ly, (f2)A.z, (f2)__builtin_fmaf(lx, A.w, c0v));
        const f2 qd = __builtin_elementwise_fma(u, u, v * v);
        const f2 e = (f2)l2op - qd;
        const float a0 = __builtin_amdgcn_exp2f(e.x), a1 = __builtin_amdgcn_exp2f(e.y);
        // FP16_TARGET: lane masks (live from dst.a).  FP32: one sign per pixel,
        // z = min(L - max(|u|,|v|), a - amin, T - t_min) >= 0 — each difference is exact in sign, so
        // this is the box, alpha and liveness test bit for bit (pixels off the image hold T = -1) —
        // and the accepted alpha is selected by z's sign bit with a bitfield insert, not through
        // lane masks combined on the scalar unit (whose VCC round trips cost wait states)
        const float z0 = fminf(fminf(L - fmaxf(fabsf(u.x), fabsf(v.x)), a0 - amin), T.x - t_min);
        const float z1 = fminf(fminf(L - fmaxf(fabsf(u.y), fabsf(v.y)), a1 - amin), T.y - t_min);
        const bool hit0 = FP16_TARGET ? live0 && fmaxf(fabsf(u.x), fabsf(v.x)) <= L && a0 >= amin : z0 >= 0.0f;
        const bool hit1 = FP16_TARGET ? live1 && fmaxf(fabsf(u.y), fabsf(v.y)) <= L && a1 >= amin : z1 >= 0.0f;
#ifdef GS_COMP_STATS
        {
            const uint64_t b0 = __ballot(hit0), b1 = __ballot(hit1);
            dg[0] += 1;
            dg[1] += __popcll(__ballot(live0)) + __popcll(__ballot(live1));
            dg[2] += __popcll(b0) + __popcll(b1);
            const uint64_t hb = b0 | b1;  // lanes 0-31: top quarter, 32-63: bottom quarter
            dg[3] += hb == 0;
            dg[4] += (hb & 0xffffffffull) != 0 && (hb >> 32) == 0;
            dg[5] += (hb & 0xffffffffull) == 0 && (hb >> 32) != 0;
            const float r = e.x > e.y ? e.x : e.y;  // best of the pair, ignoring the quad box
            dg[6] += __popcll(__ballot(r >= -7.99f));
        }
#endif
        if (FP16_TARGET) {
#pragma clang fp contract(off)
            // the blend unit: src * (1 - dst.a) + dst, stored as fp16 (as the oracle does it)
            if (hit0) {
                const float om = 1.0f - ca.x;
                cr.x = (float)(_Float16)((kr * a0) * om + cr.x);
                cg.x = (float)(_Float16)((kg * a0) * om + cg.x);
                cb.x = (float)(_Float16)((kb * a0) * om + cb.x);
                ca.x = (float)(_Float16)(a0 * om + ca.x);
                live0 = ca.x < 1.0f;  // dst.a == 1: later blends add exactly zero
            }
            if (hit1) {
                const float om = 1.0f - ca.y;
                cr.y = (float)(_Float16)((kr * a1) * om + cr.y);
                cg.y = (float)(_Float16)((kg * a1) * om + cg.y);
                cb.y = (float)(_Float16)((kb * a1) * om + cb.y);
                ca.y = (float)(_Float16)(a1 * om + ca.y);
                live1 = ca.y < 1.0f;
            }
        } else {
#pragma clang fp contract(off)
            // (no contraction: T - am T must not become one fma, k_composite_q rounds it twice)
            const f2 am = {hit0 ? a0 : 0.0f, hit1 ? a1 : 0.0f};
            const f2 s2 = am * T;  // = hit ? a T : 0 (T is finite and >= 0)
            cr = __builtin_elementwise_fma((f2)kr, s2, cr);
            cg = __builtin_elementwise_fma((f2)kg, s2, cg);
            cb = __builtin_elementwise_fma((f2)kb, s2, cb);
            T = T - s2;
            live0 = T.x >= t_min;  // (pixels off the image: T = -1)
            live1 = T.y >= t_min;
        }
    };
#ifdef GS_COMP_DIAG
    if (tid == 0) dg[7] = n;
#endif
    if (ptid == 0) s_sat[sg] = 0;
    if (ptid < 3) sR[sg][1][kCompBatch][ptid] = make_float4(0.0f, ptid == 2 ? -INFINITY : 0.0f, 0.0f, 0.0f);
#ifdef GS_COMP_PHASE
    const unsigned long long cp_start = clock64();
#endif
    if (nb > 0) {
        load_slots(0);
        gather(0);
        park(0);
    }
    __syncthreads();
#ifdef GS_COMP_PHASE
    dg[0] += clock64() - cp_start;
#endif
    for (uint32_t b = 0; b < nb; ++b) {
        const int cur = b & 1;
        {
            CP_T0(cg0);
            if (b + 1 < nb) gather(b + 1);  // in flight while this batch is blended
            CP_ADD(4, cg0);
        }
        CP_T0(cw0);
        if (wave_live) {
            for (int seg = 0; seg < 2 && wave_live; ++seg) {
                // both quarters' lists of this producing wave, in lockstep (the shorter one's tail
                // is the null record)
                uint32_t cmax = sN[sg][cur][h][0][seg];
#pragma unroll
                for (int bb = 1; bb < kBands; ++bb) cmax = max(cmax, sN[sg][cur][h][bb][seg]);
                const int cnt = (int)cmax;
                const uint16_t* list = &sL[sg][cur][h][qr][seg * 64];  // this lane's band
                // the depth key bounding where this lane's band died (the wave died at or before
                // step k): the band's entry at k, or past its list's end the band's last entry (the
                // lockstep lists differ: the other band's entry at k may be nearer than this band's
                // end).  The next frame's per-tile cut relies on it being an upper bound.
                auto sat_key = [&](uint32_t off) -> uint32_t {
                    if (off != kNullOff) return *(const uint32_t*)(sRb + off + 44);
                    const uint32_t nq = sN[sg][cur][h][qr][seg];
                    return nq ? *(const uint32_t*)(sRb + list[nq - 1] + 44) : 0u;
                };
                int k = 0;
                for (; k + 3 < cnt; k += 4) {  // saturation checked every 4 steps
                    const uint32_t o3 = list[k + 3];
                    blend(list[k]);
                    blend(list[k + 1]);
                    blend(list[k + 2]);
                    blend(o3);
                    if (!__any(live0 || live1)) {
                        wave_live = false;
                        if (m == 0) atomicMax(&s_sat[sg], sat_key(o3));
                        break;
                    }
                }
                for (; wave_live && k < cnt; ++k) {
                    const uint32_t ok = list[k];
                    blend(ok);
                    if (!__any(live0 || live1)) {
                        wave_live = false;
                        if (m == 0) atomicMax(&s_sat[sg], sat_key(ok));
                    }
                }
            }
        }
        CP_ADD(1, cw0);
        {
            CP_T0(cp0);
            if (b + 1 < nb) park(cur ^ 1);
            CP_ADD(2, cp0);
        }
        CP_T0(cb0);
        const bool go_on = block_any<NT>(wave_live, s_any[b & 1]);
        CP_ADD(3, cb0);
        if (!go_on) break;
    }
#ifdef GS_COMP_DIAG
    if (sg == 0 && lane == 0 && tile < 16384)
        for (int i = 0; i < 8; ++i) g_comp_cnt[tile][h][i] = dg[i];
    __shared__ uint32_t s_blends;
    if (tid == 0) s_blends = 0;
    __syncthreads();
    if (lane == 0 && sg == 0) atomicAdd(&s_blends, (uint32_t)dg[0]);
    __syncthreads();
    if (tid == 0 && tile < 16384) {
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_comp_time[tile][0] = (t_begin & 0xffffffffffull) | ((unsigned long long)min(n, 0xffffffu) << 40);
        g_comp_time[tile][1] = (wall_clock64() & 0xffffffffffull) | ((unsigned long long)min(s_blends, 0xffffffu) << 40);
        g_comp_time[tile][2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    }
#endif
    if (SEG > 1 && nseg > 1) {
        // the segments' (C, T) through LDS (each pair's own staging area, dead now), merged by
        // pair 0 in list order
        f2* sM = (f2*)&sR[sg][0][0][0];  // [4][128]: r, g, b, T of the pair's pixel pairs
        __syncthreads();                  // (every pair's walk has read its staging area)
        if (sg > 0 && sg < (int)nseg) {
            sM[0 * 128 + ptid] = cr;
            sM[1 * 128 + ptid] = cg;
            sM[2 * 128 + ptid] = cb;
            sM[3 * 128 + ptid] = T;
            if (ptid == 0 && s_sat[sg] == 0 && n > 0)  // never saturated alone: its last splat's key
                s_sat[sg] = __float_as_uint(rec[3 * (uint64_t)tvals[range.y - 1] + 2].w);
        }
        if (tid == 0) s_qsat = 0;
        __syncthreads();
        if (sg == 0) {
            int q0 = 0, q1 = 0;  // the segment in which each pixel's merged T fell below t_min
            for (uint32_t q = 1; q < nseg; ++q) {
                const f2* mq = (const f2*)&sR[q][0][0][0];
                const f2 qr_ = mq[0 * 128 + ptid], qg = mq[1 * 128 + ptid], qb = mq[2 * 128 + ptid];
                const f2 qt = mq[3 * 128 + ptid];
                if (T.x >= t_min) {
                    cr.x = __builtin_fmaf(T.x, qr_.x, cr.x);
                    cg.x = __builtin_fmaf(T.x, qg.x, cg.x);
                    cb.x = __builtin_fmaf(T.x, qb.x, cb.x);
                    T.x = T.x * qt.x;
                    if (T.x < t_min) q0 = (int)q;
                }
                if (T.y >= t_min) {
                    cr.y = __builtin_fmaf(T.y, qr_.y, cr.y);
                    cg.y = __builtin_fmaf(T.y, qg.y, cg.y);
                    cb.y = __builtin_fmaf(T.y, qb.y, cb.y);
                    T.y = T.y * qt.y;
                    if (T.y < t_min) q1 = (int)q;
                }
            }
            live0 = T.x >= t_min;
            live1 = T.y >= t_min;
            const int qm = max(q0, q1);
            if (qm > 0) atomicMax(&s_qsat, (uint32_t)qm);
        }
    }
    const bool tile_done = !block_any<NT>(sg == 0 && (live0 || live1), s_any[2]);
    if (SEG > 1 && sg != 0) return;
    if (tid == 0) {
        const bool sat = tile_done && range0.y > range0.x;
        const uint32_t key = SEG > 1 && nseg > 1 ? s_sat[s_qsat] : s_sat[0];
        if (sat) {  // saturation statistics for the chunk controller
            StatShard* sh = p.stats + tile % kStatShards;
            atomicAdd(&sh->sat_hist[sat_bucket(key, p.sat_base)], 1u);
            atomicMax(&sh->sat_key, key);
        }
        // the next frame's per-tile cut: the depth at which this tile saturated (none: no cut)
        if (p.tile_sat) p.tile_sat[(uint32_t)tile + (uint32_t)p.tile_row_begin * (uint32_t)p.tiles_x] = sat ? key : kSentinel;
    }
    if (p.mode == kCompFirst) {
        if (!tile_done) {  // park the pixels for chunk 1
            if (in0) p.state[pix_late(0)] = make_float4(cr.x, cg.x, cb.x, FP16_TARGET ? ca.x : T.x);
            if (in1) p.state[pix_late(1)] = make_float4(cr.y, cg.y, cb.y, FP16_TARGET ? ca.y : T.y);
            if (tid == 0) {
                p.done[tile] = 0;
                const uint32_t at = atomicAdd(&p.ctl->not_done, 1u);
                if (p.c1tiles) p.c1tiles[at] = (uint32_t)tile;  // chunk 1's tile list
                if (p.umask) umask_set(p, tile);
            }
            return;
        }
        if (tid == 0) p.done[tile] = 1;
    }
    if (!FP16_TARGET) ca = (f2)1.0f - T;
    int ox, oy;
    lane_pix(ox, oy);
    const uint64_t o0 = (uint64_t)(oy - p.row0) * p.W + ox, o1 = o0 + (uint64_t)p.W;
    if (p.out_f16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        if (in0) ((h4*)p.out)[o0] = h4{(_Float16)cr.x, (_Float16)cg.x, (_Float16)cb.x, (_Float16)ca.x};
        if (in1) ((h4*)p.out)[o1] = h4{(_Float16)cr.y, (_Float16)cg.y, (_Float16)cb.y, (_Float16)ca.y};
    } else {
        if (in0) ((float4*)p.out)[o0] = make_float4(cr.x, cg.x, cb.x, ca.x);
        if (in1) ((float4*)p.out)[o1] = make_float4(cr.y, cg.y, cb.y, ca.y);
    }
}


// One tile per workgroup.  XCD-aware order: blocks b and b + 8 share an XCD (round-robin
// dispatch), so XCD b % 8 gets the contiguous band of tiles [(b % 8) per, (b % 8 + 1) per): a
// splat's neighbouring tiles then read its record through one L2.  Measured alternatives (8160
// tiles, 2560 resident workgroups; the last partly filled round costs ~25 % of the span): a
// resident grid with per-band ticket counters (278 us), an equal static share per workgroup
// (285 us) and one ticket counter for all bands (352 us) were all slower than this (230 us).
template <bool FP16_TARGET, int SEG, int BANDS = kBands>
__global__ __launch_bounds__(128 * SEG, SEG == 1 ? GS_COMP_WAVES : (SEG == 2 ? 5 : 2)) void k_composite(CompositeParams p) {
    __shared__ CompShared<SEG, BANDS> S;
    const int per = (p.n_tiles + 7) >> 3;
    const int j = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // XCD band, position
    if (j < p.n_tiles) composite_tile<FP16_TARGET, SEG, BANDS>(p, p.order ? (int)p.order[j] : j, S);
}

// Chunk 0's per-tile sort and composite as one launch (the sort's 128-thread shape is the
// composite's): the workgroup sorts its tile's list, then composites it from the list it just
// wrote, in the same LDS.  The frame's chain then ends with the emission, one launch earlier.
template <bool FP16_TARGET, int BANDS = kBands>
__global__ __launch_bounds__(128, GS_COMP_WAVES) void k_composite_ts(CompositeParams p, TileSortParams tp) {
    static_assert(TsSmall::NT == 128, "the sort's shape is the composite's");
    constexpr size_t kLds = sizeof(CompShared<1, BANDS>) > sizeof(TsSharedT<TsSmall>) ? sizeof(CompShared<1, BANDS>)
                                                                                      : sizeof(TsSharedT<TsSmall>);
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const int per = (p.n_tiles + 7) >> 3;
    const int j = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // XCD band, position
    if (j >= p.n_tiles) return;
    const int tile = p.order ? (int)p.order[j] : j;
    tile_sort_tile<TsSmall>(tp, tile, *reinterpret_cast<TsSharedT<TsSmall>*>(lds));
    __syncthreads();  // (the sorted list: this workgroup's stores, through its CU's L1; the LDS reused)
    // an opaque copy of the tile: nothing of the composite is computed before the sort and held
    // across it (one such address was spilled to scratch)
    int tc;
    asm volatile("s_mov_b32 %0, %1" : "=s"(tc) : "s"(tile));
    composite_tile<FP16_TARGET, 1, BANDS>(p, tc, *reinterpret_cast<CompShared<1, BANDS>*>(lds));
}

// Chunk 1 (kCompSecond): workgroup j takes entry j of the compact list of the tiles chunk 0 left
// unsaturated; the rest return at once.  (A grid of a few workgroups per CU striding the list was
// slower: orbit frames' chunk-1 composite 69 -> 87 us, k_composite_q 71 -> 100 us; up to ~2600
// tiles are listed, most with few chunk-1 entries, and a strided workgroup walks its share of
// them one after another.)
template <bool FP16_TARGET, int SEG>
__global__ __launch_bounds__(128 * SEG, 2) void k_composite_c1(CompositeParams p) {
    __shared__ CompShared<SEG, kBands> S;
    if (blockIdx.x >= p.ctl->not_done) return;
    composite_tile<FP16_TARGET, SEG, kBands>(p, __builtin_amdgcn_readfirstlane((int)p.c1tiles[blockIdx.x]), S);
}

// Quarter variant for frames with few tiles (row strips): 4 waves per tile, wave q owns the 8x8
// quarter (q & 1, q >> 1) at one pixel per lane, and each splat is listed only for the quarters
// its ellipse reaches (columns within the quarter's rows).  Per pixel it performs the same
// operations in the same order as k_composite, so the image is bit-identical; it shortens the
// slowest tile's chain when there are too few tiles to fill the chip.
constexpr int kCompBatchQ = 256;

struct CompQShared {
    float4 sR[2][kCompBatchQ][3];
    uint16_t sL[2][4][kCompBatchQ];  // per quarter: LDS byte offsets of the records in sR, segment = producing wave
    uint32_t sN[2][4][4];           // per quarter, per producing wave: list length
    uint32_t s_sat;
    uint32_t any[3][4];             // block_any flags: batches by parity, the tile's end
};

template <bool FP16_TARGET>
__device__ __forceinline__ void composite_q_tile(const CompositeParams& p, const int tile, CompQShared& S);
#ifdef GS_CQ_TIME
__device__ unsigned long long g_cq_time[16384][3];
__device__ unsigned long long g_cq_phase[16384][4][4];  // per tile, wave: start clock, walk, park, barrier cycles
#endif

// Workgroup item vb -> tile: XCD-banded (through the tile order when set), or chunk 1's compact
// list of the tiles chunk 0 left unsaturated (kCompSecond with c1tiles).
template <bool FP16_TARGET>
__device__ __forceinline__ void composite_q_body(const CompositeParams& p, uint32_t vb, CompQShared& S) {
    int tile;
    if (p.mode == kCompSecond && p.c1tiles) {
        if (vb >= p.ctl->not_done) return;
        tile = __builtin_amdgcn_readfirstlane((int)p.c1tiles[vb]);
    } else {
        const int per = (p.n_tiles + 7) >> 3;
        const int j = (int)(vb & 7) * per + (int)(vb >> 3);  // XCD band, position
        if (j >= p.n_tiles) return;
        tile = p.order ? (int)p.order[j] : j;
        if (p.mode == kCompSecond && p.done[tile]) return;
    }
#ifdef GS_CQ_TIME  // diagnostics builds only: chunk 1's composite per listed tile (tile | n << 32, start, end)
    const unsigned long long t0 = wall_clock64();
#endif
    composite_q_tile<FP16_TARGET>(p, tile, S);  // one inlined copy
#ifdef GS_CQ_TIME
    if (threadIdx.x == 0 && p.mode == kCompSecond && vb < 16384) {
        g_cq_time[vb][0] = (unsigned long long)tile | ((unsigned long long)(p.ranges[tile].y - p.ranges[tile].x) << 32);
        g_cq_time[vb][1] = t0;
        g_cq_time[vb][2] = wall_clock64();
    }
#endif
}

template <bool FP16_TARGET>
__device__ __forceinline__ void composite_q_tile(const CompositeParams& p, const int tile, CompQShared& S) {
    auto& sR = S.sR;
    auto& sL = S.sL;
    auto& sN = S.sN;
    uint32_t& s_sat = S.s_sat;
    const int tid = threadIdx.x;
#ifdef GS_C1_PRINT
    if (tid == 0 && p.mode == kCompSecond) printf("C1T %d %u\n", tile, p.ranges[tile].y - p.ranges[tile].x);
#endif
    const int qw = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int tx = tile % p.tiles_x, ty = tile / p.tiles_x + p.tile_row_begin;
    const int tx0 = tx * kTile, ty0 = ty * kTile;
    const int px = tx0 + (qw & 1) * 8 + (lane & 7), py = ty0 + (qw >> 1) * 8 + (lane >> 3);
    const bool in = px < p.W && py < p.H;
    const float lx = (float)(px - tx0) + 0.5f, ly = (float)(py - ty0) + 0.5f;
    const uint2 range = p.ranges[tile];
    const float4* __restrict__ rec = p.rec;
    const uint32_t* __restrict__ tvals = p.tvals;
    const float L = 2.0f * kSqrtLog2e, amin = 1.0f / 255.0f, t_min = p.t_min;
    const uint64_t pix = (uint64_t)py * p.W + px;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f, T = 1.0f, ca = 0.0f;
    if (p.mode == kCompSecond && in) {
        const float4 st = p.state[pix];
        cr = st.x; cg = st.y; cb = st.z;
        if (FP16_TARGET) ca = st.w; else T = st.w;
    }
    if (!FP16_TARGET && !in) T = -1.0f;  // FP32: the pixel test reads liveness from T (as k_composite)
    bool live = in && (FP16_TARGET ? ca < 1.0f : T >= t_min);
    bool wave_live = __any(live);

    const uint32_t n = range.y - range.x;
    const uint32_t nb = (n + kCompBatchQ - 1) / kCompBatchQ;
    float4 ga, gb, gc;
    uint32_t gs_ = 0;
    bool gv = false;
    // the batch's slot ids are loaded one batch ahead of its records, so the record loads of batch
    // b + 1 do not wait for a tile-list load first
    uint32_t sl_next = 0;
    auto load_slots = [&](uint32_t batch) {
        const uint32_t e = range.x + batch * kCompBatchQ + tid;
        if (e < range.y) sl_next = tvals[e];
    };
    auto gather = [&](uint32_t batch) {
        const uint32_t e = range.x + batch * kCompBatchQ + tid;
        gv = e < range.y;
        if (gv) {
            gs_ = sl_next;
            const float4* r = rec + 3 * (uint64_t)gs_;
            ga = r[0];
            gb = r[1];
            gc = r[2];
        }
        if (batch + 1 < nb) load_slots(batch + 1);
    };
    auto park = [&](int buf) {
        const float cxr = ga.x - (float)tx0, cyr = ga.y - (float)ty0;
        const float c0u = -__builtin_fmaf(cxr, ga.z, cyr * ga.w);
        const float c0v = -__builtin_fmaf(cxr, gb.x, cyr * gb.y);
        sR[buf][tid][0] = make_float4(ga.w, ga.z, gb.y, gb.x);  // as k_composite
        sR[buf][tid][1] = make_float4(gc.x, c0u, gc.y, c0v);
        sR[buf][tid][2] = make_float4(gc.z, gb.z, __uint_as_float(gs_), gc.w);
        const Ellipse el = ellipse_of(ga, gb);
#pragma unroll
        for (int hy = 0; hy < 2; ++hy) {  // the splat's columns within the quarter row band
            uint32_t ul = 0u, uh = 0u;
            const bool cols = gv && ellipse_cols_band(el, (uint32_t)(ty0 + 8 * hy), (uint32_t)(ty0 + 8 * hy + 7), ul, uh);
#pragma unroll
            for (int hx = 0; hx < 2; ++hx) {
                const int q = hy * 2 + hx, qx = tx0 + hx * 8;
                const bool hit = cols && (int)ul <= qx + 7 && (int)uh >= qx;
                const uint64_t b = __ballot(hit);
                if (hit) sL[buf][q][qw * 64 + __popcll(b & lanemask_lt())] = (uint16_t)(((buf * kCompBatchQ + tid) * 3) * 16);
                if (lane == 0) sN[buf][q][qw] = (uint32_t)__popcll(b);
            }
        }
    };
    const char* const sRb = (const char*)&sR[0][0][0];
    auto blend = [&](uint32_t off) {
        const float4 A = *(const float4*)(sRb + off);
        const float4 B = *(const float4*)(sRb + off + 16);
        const float4 C = *(const float4*)(sRb + off + 32);
        // staged as [b, a, d, c] [r, c0u, g, c0v] [b, log2 op, slot, key]: each colour channel a
        // packed fma broadcasts is the low half of an aligned register pair (no moves)
        const float c0u = B.y, c0v = B.w, l2op = C.y, kr = B.x, kg = B.z, kb = C.x;
        // the same roundings as k_composite's packed pair
        const float u = __builtin_fmaf(ly, A.x, __builtin_fmaf(lx, A.y, c0u));
        const float v = __builtin_fmaf(ly, A.z, __builtin_fmaf(lx, A.w, c0v));
        const float qd = __builtin_fmaf(u, u, v * v);
        const float e = l2op - qd;
        const float a = __builtin_amdgcn_exp2f(e);
        // FP32: one sign, z = min(L - max(|u|,|v|), a - amin, T - t_min) >= 0, each difference exact
        // in sign (k_composite's test, bit for bit the box, alpha and liveness tests)
        const bool hit = FP16_TARGET ? live && fmaxf(fabsf(u), fabsf(v)) <= L && a >= amin
                                     : fminf(fminf(L - fmaxf(fabsf(u), fabsf(v)), a - amin), T - t_min) >= 0.0f;
        if (FP16_TARGET) {
#pragma clang fp contract(off)
            if (hit) {
                const float om = 1.0f - ca;
                cr = (float)(_Float16)((kr * a) * om + cr);
                cg = (float)(_Float16)((kg * a) * om + cg);
                cb = (float)(_Float16)((kb * a) * om + cb);
                ca = (float)(_Float16)(a * om + ca);
                live = ca < 1.0f;
            }
        } else {
            const float s = hit ? a * T : 0.0f;
            cr = __builtin_fmaf(kr, s, cr);
            cg = __builtin_fmaf(kg, s, cg);
            cb = __builtin_fmaf(kb, s, cb);
            T = T - s;
            live = T >= t_min;  // (pixels off the image: T = -1)
        }
    };
#ifdef GS_CQ_TIME
    unsigned long long q_walk = 0, q_park = 0, q_bar = 0;
    const unsigned long long q_start = clock64();
#endif
    if (tid == 0) s_sat = 0;
    if (nb > 0) {
        load_slots(0);
        gather(0);
        park(0);
    }
    __syncthreads();
    for (uint32_t b = 0; b < nb; ++b) {
        const int cur = b & 1;
#ifdef GS_CQ_TIME
        const unsigned long long q_t0 = clock64();
#endif
        if (b + 1 < nb) gather(b + 1);
        if (wave_live) {
            for (int seg = 0; seg < 4 && wave_live; ++seg) {
                const int cnt = (int)sN[cur][qw][seg];
                const uint16_t* list = &sL[cur][qw][seg * 64];
                int k = 0;
                for (; k + 3 < cnt; k += 4) {
                    const uint32_t o3 = list[k + 3];
                    blend(list[k]);
                    blend(list[k + 1]);
                    blend(list[k + 2]);
                    blend(o3);
                    if (!__any(live)) {
                        wave_live = false;
                        if (lane == 0) atomicMax(&s_sat, *(const uint32_t*)(sRb + o3 + 44));
                        break;
                    }
                }
                for (; wave_live && k < cnt; ++k) {
                    const uint32_t ok = list[k];
                    blend(ok);
                    if (!__any(live)) {
                        wave_live = false;
                        if (lane == 0) atomicMax(&s_sat, *(const uint32_t*)(sRb + ok + 44));
                    }
                }
            }
        }
#ifdef GS_CQ_TIME
        const unsigned long long q_t1 = clock64();
#endif
        if (b + 1 < nb) park(cur ^ 1);
#ifdef GS_CQ_TIME
        const unsigned long long q_t2 = clock64();
#endif
        const bool q_go = block_any<256>(wave_live, S.any[b & 1]);
#ifdef GS_CQ_TIME
        q_walk += q_t1 - q_t0;
        q_park += q_t2 - q_t1;
        q_bar += clock64() - q_t2;
#endif
        if (!q_go) break;
    }
#ifdef GS_CQ_TIME
    if (p.mode == kCompSecond && lane == 0) {  // per wave: start clock, walks, parks, barriers (shader cycles)
        g_cq_phase[tile & 16383][qw][0] = q_start;
        g_cq_phase[tile & 16383][qw][1] = q_walk;
        g_cq_phase[tile & 16383][qw][2] = q_park;
        g_cq_phase[tile & 16383][qw][3] = q_bar;
    }
#endif
    const bool tile_done = !block_any<256>(live, S.any[2]);
    if (tile_done && tid == 0 && n > 0) {
        StatShard* sh = p.stats + tile % kStatShards;
        atomicAdd(&sh->sat_hist[sat_bucket(s_sat, p.sat_base)], 1u);
        atomicMax(&sh->sat_key, s_sat);
    }
    if (tid == 0 && p.tile_sat)  // the next frame's per-tile cut (as composite_tile)
        p.tile_sat[(uint32_t)tile + (uint32_t)p.tile_row_begin * (uint32_t)p.tiles_x] = tile_done && n > 0 ? s_sat : kSentinel;
    if (p.mode == kCompFirst) {
        if (!tile_done) {
            if (in) p.state[pix] = make_float4(cr, cg, cb, FP16_TARGET ? ca : T);
            if (tid == 0) {
                p.done[tile] = 0;
                const uint32_t at = atomicAdd(&p.ctl->not_done, 1u);
                if (p.c1tiles) p.c1tiles[at] = (uint32_t)tile;  // chunk 1's tile list
                if (p.umask) umask_set(p, tile);
            }
            return;
        }
        if (tid == 0) p.done[tile] = 1;
    }
    if (!FP16_TARGET) ca = 1.0f - T;
    const uint64_t o = (uint64_t)(py - p.row0) * p.W + px;
    if (!in) return;
    if (p.out_f16) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        ((h4*)p.out)[o] = h4{(_Float16)cr, (_Float16)cg, (_Float16)cb, (_Float16)ca};
    } else {
        ((float4*)p.out)[o] = make_float4(cr, cg, cb, ca);
    }
}

template <bool FP16_TARGET>
__global__ __launch_bounds__(256) void k_composite_q(CompositeParams p) {
    __shared__ CompQShared S;
    composite_q_body<FP16_TARGET>(p, blockIdx.x, S);
}

// ============================================================================ k_chunk1
// Chunk 1 as ONE launch.  It has work only in frames where chunk 0 left a tile unsaturated, so
// its usual cost is this launch returning at once (eight gated launches cost ~35 us of floors).
// When it runs, it is the chunk-0 pipeline's phases in order, separated by grid barriers, on a
// grid of one 256-thread workgroup per CU (every workgroup co-resident): the partitions that may
// hold chunk-1 splats (c1_parts_body, against the unsaturated-tile bits the chunk-0 composite
// set) -> their chunk-1 slots
// (c1_records_body) -> bin count -> column scan -> tile scan -> emission ->
// per-tile sort -> composite (kCompSecond) of the unsaturated tiles.

// Grid barrier: bar[0] counts arrivals, bar[1] is a generation word that is never reset.  A
// workgroup reads the generation, arrives; the last arriver zeroes the count and then bumps the
// generation (release), the others spin until the generation moves (acquire).  The count is zero
// again whenever every workgroup has left a barrier, so no one resets it while another workgroup may
// still be polling (a reset at the frame's end raced with the last barrier's stragglers).  Agent
// scope (cdna_hip_programming.md Guideline 16).
// Residency: the grid is at most occupancy x CUs of k_chunk1 alone (queried at context creation,
// chunk1_occupancy; the context refuses a device where it is not) and no kernel beside it waits
// for it, so once the kernels launched before and beside it drain, every workgroup is resident.
// Bounded spin: `spin_ticks` of the 100 MHz wall clock (~200 ms, set by the host from the
// device's clock rate; far above any one kernel's duration, so only a grid that can never become
// resident times out).  A timeout sets kErrBarrier: a synchronous gs_render fails its own frame,
// gs_render_device reports it on its next call, and the host zeroes bar[] before the set's next launch.
__device__ __forceinline__ void grid_sync(uint32_t* bar, FrameCtl* ctl, uint64_t spin_ticks) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave drains its stores
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t gen = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t t0 = wall_clock64();
        for (uint32_t spins = 0; __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen;) {
            if ((++spins & 63u) == 0u && wall_clock64() - t0 > spin_ticks) {
                atomicOr(&ctl->err, kErrBarrier);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

constexpr size_t kBinLdsWords = kBandTiles + (kBinMaxUnits + 1) + 4 + kWideQueue + 3 + kBandTiles / 2 + kCutMaxBlocks;  // (s_nw, s_chk[2], cut)
constexpr size_t kChunk1Lds = std::max(std::max(kBinLdsWords * 4, sizeof(TsShared)), sizeof(CompQShared));

#ifdef GS_C1_TIME
// diagnostics builds only (make diag DIAGFLAGS=-DGS_C1_TIME): wall clock at k_chunk1's start and
// after each of its grid barriers (workgroup 0), the last frame with chunk-1 work
__device__ unsigned long long g_c1_time[16];
#define C1_MARK(k) do { if (blockIdx.x == 0 && threadIdx.x == 0) g_c1_time[k] = wall_clock64(); } while (0)
#else
#define C1_MARK(k) do { } while (0)
#endif

template <bool FP16_TARGET>
__device__ __forceinline__ void chunk1_phases(const Chunk1Params& c, uint8_t* lds) {  // inlined: a
// reference to the kernel argument must not force a copy of it into scratch
    FrameCtl* ctl = c.cp.ctl;
    const uint32_t G = gridDim.x, b = blockIdx.x;
    C1_MARK(0);
    const uint32_t* um = umask_lds(c.pp, (uint32_t*)lds, (uint32_t)(kChunk1Lds / 4));
    C1_MARK(1);
    c1_parts_body(c.pp, b, G, um);
    grid_sync(c.bar, ctl, c.spin_ticks);
    C1_MARK(2);
    c1_records_body(c.pp, b, G, um);
    grid_sync(c.bar, ctl, c.spin_ticks);  // (and every wave is done with the bits in LDS)
    C1_MARK(3);
    uint32_t* s_a = (uint32_t*)lds;
    uint32_t* s_pref = s_a + kBandTiles;
    uint32_t* s_tmp = s_pref + kBinMaxUnits + 1;
    uint32_t* s_wide = s_tmp + 4;
    uint32_t* s_nw = s_wide + kWideQueue;
    const uint32_t nbin = c.bp.nparts * bin_bands(c.bp.n_tiles, c.bp.band_tiles);
    for (uint32_t vb = b; vb < nbin; vb += G) {
        if (c.bp.cut) bin_count_body<256, false, true>(c.bp, vb, s_a, s_pref, s_tmp, s_wide, s_nw);
        else bin_count_body<256, false, false>(c.bp, vb, s_a, s_pref, s_tmp, s_wide, s_nw);
    }
    grid_sync(c.bar, ctl, c.spin_ticks);
    C1_MARK(4);
    const uint32_t ncol = (c.bp.n_tiles + kColTiles - 1) / kColTiles;
    for (uint32_t vb = b; vb < ncol; vb += G) colscan_body<4>(c.bp, vb, (uint32_t(*)[kColTiles])lds);
    grid_sync(c.bar, ctl, c.spin_ticks);
    C1_MARK(5);
    if (b == 0) tile_scan_body<256>(c.bp, s_a);
    grid_sync(c.bar, ctl, c.spin_ticks);
    C1_MARK(6);
    for (uint32_t vb = b; vb < nbin; vb += G) {
        if (c.bp.cut) bin_emit_body<256, false, false, true>(c.bp, vb, s_a, s_pref, s_tmp, s_wide, s_nw);
        else bin_emit_body<256, false, false, false>(c.bp, vb, s_a, s_pref, s_tmp, s_wide, s_nw);
    }
    grid_sync(c.bar, ctl, c.spin_ticks);
    C1_MARK(7);
    // (chunk 1's tiles: the compact list when the first pass kept one, else every tile)
    // each listed tile sorted and composited by one workgroup (c1tiles: both map item vb to the
    // same tile; the sorted list is the workgroup's own writes)
    const uint32_t ntb = ctl->not_done;
    for (uint32_t vb = b; vb < ntb; vb += G) {
        tile_sort_body<TsBig>(c.tp, vb, *(TsShared*)lds);
        __syncthreads();
        composite_q_body<FP16_TARGET>(c.cp, vb, *(CompQShared*)lds);
        __syncthreads();
    }
    grid_sync(c.bar, ctl, c.spin_ticks);
    C1_MARK(9);  // every phase done before the frame's end reads FrameCtl
}

template <bool FP16_TARGET>
__global__ __launch_bounds__(256) void k_chunk1(Chunk1Params c) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kChunk1Lds];
    FrameCtl* ctl = c.cp.ctl;
    const uint32_t G = gridDim.x, b = blockIdx.x;
    FE_MARK(5);
    if (c.two_chunks && ctl->not_done != 0) chunk1_phases<FP16_TARGET>(c, lds);  // else: chunk 0 saturated every tile
    // the frame's end (one wave): FrameCtl is read by no workgroup after this point
    if (b == 0 && threadIdx.x < 64) frame_end_body(ctl, c.stats, c.host_ctl, c.host_seq, c.seq, (uint32_t*)lds);
    (void)G;
}


// Chunk 1 as separate launches, for frames the host expects to leave tiles unsaturated (a recent
// frame did): the phases of chunk1_phases at full occupancy with a kernel boundary (~1.5 us) in
// place of each grid barrier; every launch returns at once when chunk 0 saturated every tile.
// Binning, per-tile sort and composite are the chunk-0 kernels with chunk-1 parameters.  The two
// projection-side launches test rectangles against an LDS copy of the unsaturated-tile bits.
// (dynamic LDS: the bits' words when they fit kUmaskLdsWords, else none)
__global__ __launch_bounds__(256) void k_c1_parts(ProjParams p) {
    extern __shared__ uint32_t s_um[];
    if (p.ctl->not_done == 0) return;
    c1_parts_body(p, blockIdx.x, gridDim.x, umask_lds(p, s_um, kUmaskLdsWords));
}
__global__ __launch_bounds__(256) void k_c1_records(ProjParams p) {
    extern __shared__ uint32_t s_um[];
    if (p.ctl->not_done == 0) return;
    c1_records_body(p, blockIdx.x, gridDim.x, umask_lds(p, s_um, kUmaskLdsWords));
}
// Chunk 1's per-tile sort and composite as one launch: workgroup j sorts entry j of the compact
// list of unsaturated tiles and composites it from the list it just wrote (the tile's chain is its
// own sort then its blend walk, not the slowest sort then the slowest walk; one launch fewer).
union C1TileShared {
    TsShared ts;
    CompQShared cq;
};
template <bool FP16_TARGET>
__global__ __launch_bounds__(256, 2) void k_c1_tiles(TileSortParams tp, CompositeParams cp) {
    __shared__ C1TileShared S;
    if (blockIdx.x >= cp.ctl->not_done) return;
    tile_sort_body<TsBig>(tp, blockIdx.x, S.ts);
    __syncthreads();  // (the sorted list: this workgroup's stores, through its CU's L1)
    composite_q_body<FP16_TARGET>(cp, blockIdx.x, S.cq);
}
__global__ __launch_bounds__(64) void k_frame_end(Chunk1Params c) {
    __shared__ uint32_t lds[kStatShards * ((sizeof(StatShard) / 4) | 1u)];
#ifdef GS_C1_PRINT  // diagnostics builds only: the chunk-1 workload of each frame
    if (threadIdx.x == 0 && c.cp.ctl->not_done)
        printf("C1F not_done %u c1_parts %u\n", c.cp.ctl->not_done, c.cp.ctl->c1_parts);
#endif
    frame_end_body(c.cp.ctl, c.stats, c.host_ctl, c.host_seq, c.seq, lds);
}

// ============================================================================ ref_quirks
// The reference's init-sort pass runs dispatchWorkgroups(max(N/8, 8)) workgroups of 8 threads
// (src/renderer.ts:306; src/shaders.ts:42-73): with WebIDL truncation only the first
// nk = trunc(max(N/8, 8)) * 8 slots get (depth key, index); slots nk..N-1 keep the (key, value)
// the previous frame's in-place radix sort left there (zero on the first frame).  The sort then
// orders all N slots (stable: ties by slot) and instance i draws Gaussian value[i], so a
// Gaussian can be drawn twice (or not at all).  Here: the N slots are keyed (k_quirk_keys),
// sorted by the device radix sort, and the draw list is gathered into a scene copy in draw order
// (k_quirk_gather) whose "reference index" is the draw rank; the frame then runs on that copy
// with every slot's depth key set to 0, so each tile's list is in draw-rank order.

// inv[orig[j]] = j: storage slot of each reference index.
__global__ __launch_bounds__(256) void k_inverse(const uint32_t* __restrict__ orig, uint64_t n,
                                                 uint32_t* __restrict__ inv) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < n) inv[orig[j]] = (uint32_t)j;
}

// Slots of the init-sort pass: slot g < nk = (sortable((V [p,1]).z), g) of Gaussian g (stored at
// storage slot j, orig[j] = g; the key bit-identical to k_cull's), slot s >= nk = the state.
__global__ __launch_bounds__(256) void k_quirk_keys(const float4* __restrict__ cull, const uint32_t* __restrict__ orig,
                                                    uint32_t n, uint32_t nk, float4 vrow,
                                                    const uint32_t* __restrict__ qk, const uint32_t* __restrict__ qv,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
#pragma clang fp contract(off)
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint32_t g = orig[j];
    if (g < nk) {
        const float4 c = cull[j];
        const float vz = ((vrow.x * c.x + vrow.y * c.y) + vrow.z * c.z) + vrow.w * 1.0f;  // src/shaders.ts:66-68
        keys[g] = sortable_key(vz);
        vals[g] = g;
    }
    if (j >= nk) {
        keys[j] = qk[j];
        vals[j] = qv[j];
    }
}

// Draw entry i = Gaussian svals[i]: its geometry, cull plane and SH copied to row i of the
// draw-ordered copy, dorig[i] = i; the sorted slots >= nk become the next frame's state.
__global__ __launch_bounds__(256) void k_quirk_gather(const uint32_t* __restrict__ skeys,
                                                      const uint32_t* __restrict__ svals,
                                                      const uint32_t* __restrict__ inv, uint32_t n, uint32_t nk,
                                                      uint32_t shq, const float4* __restrict__ geo,
                                                      const float4* __restrict__ shade, const float4* __restrict__ cull,
                                                      float4* __restrict__ dgeo, float4* __restrict__ dshade,
                                                      float4* __restrict__ dcull, uint32_t* __restrict__ dorig,
                                                      uint32_t* __restrict__ qk, uint32_t* __restrict__ qv) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = svals[i];
    const uint64_t j = inv[g < n ? g : 0];
    for (int k = 0; k < 3; ++k) dgeo[3 * (uint64_t)i + k] = geo[3 * j + k];
    for (uint32_t k = 0; k < shq; ++k) dshade[(uint64_t)i * shq + k] = shade[j * shq + k];
    dcull[i] = cull[j];
    dorig[i] = i;
    if (i >= nk) {
        qk[i] = skeys[i];
        qv[i] = g;
    }
}

// ============================================================================ k_present
// PostProcessRenderer.fragmentMain (src/post_process_render.ts:62-77) per pixel: the sampler
// reads texel (x, H-1-y) at its centre (exact), a' = saturate(1.5 a), a' = a'^4 (as (a'^2)^2,
// gs_present's rounding) when a' < 0.99; stored as f32, f16 (the rgba16float canvas) or unorm8.
__global__ __launch_bounds__(256) void k_present(const void* __restrict__ in, int in_f16, int W, int H,
                                                 int out_kind, void* __restrict__ out) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const uint64_t npx = (uint64_t)W * H;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < npx; i += (uint64_t)gridDim.x * 256ull) {
        const uint32_t y = (uint32_t)(i / (uint32_t)W), x = (uint32_t)(i % (uint32_t)W);
        const uint64_t src = (uint64_t)(H - 1 - y) * W + x;
        float4 c;
        if (in_f16) {
            const h4 v = ((const h4*)in)[src];
            c = make_float4((float)v.x, (float)v.y, (float)v.z, (float)v.w);
        } else {
            c = ((const float4*)in)[src];
        }
        float a = fminf(fmaxf(c.w * 1.5f, 0.0f), 1.0f);
        if (a < 0.99f) {
            const float a2 = a * a;
            a = a2 * a2;
        }
        c.w = a;
        if (out_kind == GS_PRESENT_RGBA_F32) {
            ((float4*)out)[i] = c;
        } else if (out_kind == GS_PRESENT_RGBA_F16) {
            ((h4*)out)[i] = h4{(_Float16)c.x, (_Float16)c.y, (_Float16)c.z, (_Float16)c.w};
        } else {
            auto u8 = [](float v) { return (uint32_t)rintf(fminf(fmaxf(v, 0.0f), 1.0f) * 255.0f); };
            ((uint32_t*)out)[i] = u8(c.x) | (u8(c.y) << 8) | (u8(c.z) << 16) | (u8(c.w) << 24);
        }
    }
}

}  // namespace

// ============================================================================ launchers
void launch_present(const void* in, int in_f16, int W, int H, int out_kind, void* out, hipStream_t s) {
    const uint64_t npx = (uint64_t)W * H;
    if (!npx) return;
    const unsigned grid = (unsigned)std::min<uint64_t>(8192, (npx + 255) / 256);
    hipLaunchKernelGGL(k_present, dim3(grid), dim3(256), 0, s, in, in_f16, W, H, out_kind, out);
}
void launch_bbox(const uint8_t* aos, uint64_t n, uint32_t rb, uint32_t* bbox, hipStream_t s) {
    if (!n) return;
    const unsigned grid = (unsigned)std::min<uint64_t>(256, (n + 255) / 256);
    hipLaunchKernelGGL(k_bbox, dim3(grid), dim3(256), 0, s, aos, n, rb, bbox);
}
void launch_morton(const uint8_t* aos, uint64_t n, uint32_t rb, const uint32_t* bbox, uint32_t* keys,
                   uint32_t* vals, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_morton, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, aos, n, rb, bbox, keys, vals);
}
void launch_transpose(const uint8_t* aos, uint64_t n, int n_sh, const uint32_t* perm, float4* geo, float4* shade,
                      float4* cull, uint32_t* orig, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_transpose, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, aos, n, n_sh, perm,
                       geo, shade, cull, orig);
}
void launch_part_bounds(const float4* cull, uint64_t n, PartBound* out, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_part_bounds, dim3(proj_parts(n)), dim3(256), 0, s, cull, n, out);
}
void launch_block_bounds(const float4* cull, uint64_t n, PartBound* out, hipStream_t s) {
    if (!n) return;
    const uint64_t blocks = (n + kCullBlock - 1) / kCullBlock;
    hipLaunchKernelGGL(k_block_bounds, dim3((unsigned)((blocks + 3) / 4)), dim3(256), 0, s, cull, n, out);
}
void launch_inverse(const uint32_t* orig, uint64_t n, uint32_t* inv, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_inverse, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, orig, n, inv);
}
void launch_quirk_keys(const float4* cull, const uint32_t* orig, uint32_t n, uint32_t nk, float4 vrow,
                       const uint32_t* qk, const uint32_t* qv, uint32_t* keys, uint32_t* vals, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_quirk_keys, dim3((n + 255) / 256), dim3(256), 0, s, cull, orig, n, nk, vrow, qk, qv, keys,
                       vals);
}
void launch_quirk_gather(const uint32_t* skeys, const uint32_t* svals, const uint32_t* inv, uint32_t n, uint32_t nk,
                         uint32_t shq, const float4* geo, const float4* shade, const float4* cull, float4* dgeo,
                         float4* dshade, float4* dcull, uint32_t* dorig, uint32_t* qk, uint32_t* qv, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_quirk_gather, dim3((n + 255) / 256), dim3(256), 0, s, skeys, svals, inv, n, nk, shq, geo,
                       shade, cull, dgeo, dshade, dcull, dorig, qk, qv);
}
void launch_project(const ProjParams& p, hipStream_t s) {
    const uint32_t parts = proj_parts(p.n);
    if (!parts) return;
#ifndef GS_CULL_GRID
#define GS_CULL_GRID 2048
#endif
    // k_cull's unit shard = blockIdx.x % kUnitShards holds at most unit_shard_cap units only when the
    // grid is a multiple of kUnitShards or has one partition per workgroup (grid = parts)
    static_assert(GS_CULL_GRID % kUnitShards == 0, "GS_CULL_GRID must be a multiple of kUnitShards");
#ifndef GS_PROJ_GRID
#define GS_PROJ_GRID 1536
#endif
    hipLaunchKernelGGL(k_part_list, dim3((parts + 255) / 256), dim3(256), 0, s, p);
    const uint64_t cg = p.cull_grid && p.cull_grid % kUnitShards == 0 ? p.cull_grid : GS_CULL_GRID;  // (a multiple of kUnitShards)
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(cg, parts));
    if (p.cut)
        hipLaunchKernelGGL(k_cull<true>, dim3(grid), dim3(kProjThreads), 0, s, p);
    else
        hipLaunchKernelGGL(k_cull<false>, dim3(grid), dim3(kProjThreads), 0, s, p);
    const uint64_t pg = p.proj_grid ? p.proj_grid : GS_PROJ_GRID;
    const unsigned ugrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(pg, (uint64_t)parts * kProjRounds));
    if (p.shq == 12)
        hipLaunchKernelGGL(k_project<true>, dim3(ugrid), dim3(kProjThreads), 0, s, p);
    else
        hipLaunchKernelGGL(k_project<false>, dim3(ugrid), dim3(kProjThreads), 0, s, p);
}
void launch_seed(const ProjParams& p, hipStream_t s) {
    const uint32_t nrun = (p.n + kSeedRun - 1) / kSeedRun;
    const uint32_t nsr = (nrun + p.seed_stride - 1) / std::max(1u, p.seed_stride);
    if (nsr) hipLaunchKernelGGL(k_seed_hist, dim3(std::min<uint32_t>(4096, (nsr + 15) / 16)), dim3(256), 0, s, p);
    hipLaunchKernelGGL(k_seed_pick, dim3(1), dim3(1024), 0, s, p);
}
void launch_records(const ProjParams& p, hipStream_t s) {
    if (!p.n) return;
    const uint32_t grid = std::min<uint32_t>((p.n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_records, dim3(grid), dim3(256), 0, s, p);
}

template <int IPT>
static void sort_pass_ipt(const SortPass& p, hipStream_t s) {
    const unsigned grid = std::min<uint32_t>(p.parts_max, kMaxGrid);
    if (!p.part_count)  // else k_project produced the counts (first depth pass of chunk 0)
        hipLaunchKernelGGL(k_radix_upsweep<IPT>, dim3(grid), dim3(kSortThreads), 0, s, p);
    const uint32_t m = p.part_count ? std::max(1, std::min(p.merge, kMaxMerge)) : 1;
    const unsigned dgrid = std::min<uint32_t>((p.parts_max + m - 1) / m, kMaxGrid);
    hipLaunchKernelGGL(k_radix_downsweep<IPT>, dim3(dgrid), dim3(kSortThreads), 0, s, p);
}

void launch_sort_pass(const SortPass& p, hipStream_t s) {
    if (!p.parts_max) return;
    switch (p.ipt) {
        case 4: sort_pass_ipt<4>(p, s); break;
        case 8: sort_pass_ipt<8>(p, s); break;
        default: sort_pass_ipt<16>(p, s); break;
    }
}
void launch_bin(const BinParams& p0, hipStream_t s) {
    if (p0.n_tiles == 0) return;
    static const bool lds_ok = [] {  // dynamic LDS past the default 64 KB
        const int mx = (int)(kBinLdsMaxWords * 4);
        for (const void* f : {(const void*)k_bin_count<true, false>, (const void*)k_bin_count<false, false>,
                              (const void*)k_bin_emit<true, false>, (const void*)k_bin_emit<false, false>,
                              (const void*)k_bin_count<true, true>, (const void*)k_bin_count<false, true>,
                              (const void*)k_bin_emit<true, true>, (const void*)k_bin_emit<false, true>})
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess) return false;
        return true;
    }();
    (void)lds_ok;
    BinParams p = p0;
    if ((p.nparts != (uint32_t)kBinParts && p.nparts != kBinPartsSmall) ||
        (uint64_t)p.parts * kProjRounds > (uint64_t)kBinMaxUnits * p.nparts) {
        std::fprintf(stderr, "gsplat: launch_bin with %u binning partitions for %u units\n", p.nparts, p.parts * (uint32_t)kProjRounds);
        std::abort();  // (the host never asks)
    }
    static const uint32_t min_bands = [] {  // (A/B runs: GS_BIN_BANDS, a smaller band per workgroup)
        const char* e = std::getenv("GS_BIN_BANDS");
        return e ? (uint32_t)std::max(1, std::min(4, std::atoi(e))) : 1u;
    }();
    const uint32_t bands = std::max(min_bands, (p.n_tiles + kBandTilesMax - 1) / kBandTilesMax);
    p.band_tiles = (p.n_tiles + bands - 1) / bands;  // equal bands
    // units of one binning partition: at most ceil(all units / nparts)
    p.pref_words = std::min<uint32_t>(kBinMaxUnits, (p.parts * (uint32_t)kProjRounds + p.nparts - 1) / p.nparts) + 1;
    // wide-splat queue: larger frames hold more splats that cover many tiles (near splats at 4K);
    // a splat past the queue is walked by its own thread
    // the unit entries cached in LDS beside their prefix when that leaves the minimum wide queue
    const uint32_t cut = p.cut ? cut_blocks(p.tiles_x, p.rows) : 0u;
    if (p.cut && (p.n_tiles > (uint32_t)kCutMaxTiles || cut > (uint32_t)kCutMaxBlocks || !p.cutb)) {
        std::fprintf(stderr, "gsplat: per-tile cut on a frame of %u tiles (%u blocks)\n", p.n_tiles, cut);  // (the host never asks)
        std::abort();
    }
    p.uid_lds = p.units && bin_lds_words(p.band_tiles, 2 * p.pref_words, kWideQueue, cut) <= kBinLdsMaxWords ? 1u : 0u;
    const uint32_t pw = p.pref_words * (p.uid_lds ? 2u : 1u);
    const uint32_t room = (uint32_t)(kBinLdsMaxWords - bin_lds_words(p.band_tiles, pw, 0, cut));
    p.wide_cap = p.wlist ? 0u : std::min(room, std::max(kWideQueue, std::min(kWideQueueMax, p.n_tiles / 4)));
    const size_t lds = bin_lds_words(p.band_tiles, pw, p.wide_cap, cut) * 4;
    const unsigned grid = p.nparts * bin_bands(p.n_tiles, p.band_tiles);
    if (!p.bchk || grid > bin_chk_words(p.n_tiles)) {
        std::fprintf(stderr, "gsplat: launch_bin without room for its %u workgroups' checksums\n", grid);
        std::abort();
    }
    auto count = p.units ? (cut ? k_bin_count<true, true> : k_bin_count<true, false>)
                         : (cut ? k_bin_count<false, true> : k_bin_count<false, false>);
    hipLaunchKernelGGL(count, dim3(grid), dim3(kBinThreads), lds, s, p);
    hipLaunchKernelGGL(k_bin_colscan, dim3((p.n_tiles + kColTiles - 1) / kColTiles), dim3(512), 0, s, p);
    auto emit = p.units ? (cut ? k_bin_emit<true, true> : k_bin_emit<true, false>)  // (each workgroup
                        : (cut ? k_bin_emit<false, true> : k_bin_emit<false, false>);  // scans the tile totals)
    hipLaunchKernelGGL(emit, dim3(grid), dim3(kBinThreads), lds, s, p);
}
void launch_tile_sort(const TileSortParams& p, hipStream_t s) {
    if (p.n_tiles <= 0) return;
    const unsigned grid = 8u * (unsigned)((p.n_tiles + 7) / 8);
    if (p.big == 2 && !p.done) {  // chunk-0 lists of thousands (one-chunk frames at 4K)
        hipLaunchKernelGGL(k_tile_sort_huge, dim3(grid), dim3(TsHuge::NT), 0, s, p);
        if (p.long_tiles && p.long_n && p.long_grid) {  // the lists past one LDS round: linear, 256 threads
            TileSortParams q = p;
            q.c1tiles = p.long_tiles;
            q.c1_n = p.long_n;
            q.long_tiles = nullptr;
            q.stats = nullptr;
            hipLaunchKernelGGL(k_tile_sort_list, dim3(std::min<uint32_t>(p.long_grid, grid)), dim3(TsBig::NT), 0, s, q);
        }
    } else if (p.done || p.big)  // chunk 1 (the unsaturated tiles' long lists), or long chunk-0 lists
        hipLaunchKernelGGL(k_tile_sort_big, dim3(grid), dim3(TsBig::NT), 0, s, p);
    else
        hipLaunchKernelGGL(k_tile_sort, dim3(grid), dim3(TsSmall::NT), 0, s, p);
}
void launch_chunk1(const Chunk1Params& c0, int grid, int accum_fp16, hipStream_t s) {
    if (!c0.two_chunks || c0.cp.n_tiles <= 0) grid = 1;  // the frame's end only
    Chunk1Params c = c0;  // k_chunk1's binning phases: static LDS, 8192-tile bands
    c.bp.band_tiles = kBandTiles;
    c.bp.pref_words = kBinMaxUnits + 1;
    c.bp.wide_cap = kWideQueue;
    c.bp.uid_lds = 0;  // (static LDS sized without the entries)
    if (accum_fp16)
        hipLaunchKernelGGL(k_chunk1<true>, dim3(grid), dim3(256), 0, s, c);
    else
        hipLaunchKernelGGL(k_chunk1<false>, dim3(grid), dim3(256), 0, s, c);
}
int chunk1_occupancy() {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_chunk1<false>, 256, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_chunk1<true>, 256, 0) != hipSuccess)
        return 0;
    return std::min(a, b);
}
void launch_chunk1_split(const Chunk1Params& c, int accum_fp16, hipStream_t s) {
    if (c.two_chunks && c.cp.n_tiles > 0) {
        const unsigned parts = proj_parts(c.pp.n);
        const unsigned items = c.pp.bbounds ? (unsigned)((c.pp.n + kCullBlock - 1) / kCullBlock) : parts;
        const uint32_t uw = (uint32_t)c.bp.rows * c.pp.umask_w;
        const size_t ulds = uw <= kUmaskLdsWords ? (size_t)uw * 4 : 0;
        hipLaunchKernelGGL(k_c1_parts, dim3(std::max(1u, (items + 255) / 256)), dim3(256), ulds, s, c.pp);
        hipLaunchKernelGGL(k_c1_records, dim3(kMaxGrid), dim3(256), ulds, s, c.pp);
        launch_bin(c.bp, s);
        // the unsaturated tiles only, each with a long list: 4 waves per tile at any frame size;
        // workgroup j takes entry j of the compact tile list (c1tiles), the rest return at once
        // (list split: the 4-pair half-tile kernel, the long lists cut into segments)
        const unsigned cgrid = 8u * (unsigned)((c.cp.n_tiles + 7) / 8);
        if (c.cp.seg > 1 && !accum_fp16) {
            launch_tile_sort(c.tp, s);
            hipLaunchKernelGGL((k_composite_c1<false, 4>), dim3(cgrid), dim3(512), 0, s, c.cp);
        } else if (accum_fp16) {
            hipLaunchKernelGGL(k_c1_tiles<true>, dim3(cgrid), dim3(256), 0, s, c.tp, c.cp);
        } else {
            hipLaunchKernelGGL(k_c1_tiles<false>, dim3(cgrid), dim3(256), 0, s, c.tp, c.cp);
        }
    }
    hipLaunchKernelGGL(k_frame_end, dim3(1), dim3(64), 0, s, c);
}
int composite_quarter_tiles() { return kQuarterTiles; }
void launch_composite(const CompositeParams& p, int accum_fp16, hipStream_t s, const TileSortParams* ts) {
    if (p.n_tiles <= 0) return;
    const unsigned grid = 8u * (unsigned)((p.n_tiles + 7) / 8);  // see k_composite's tile order
    if (ts) {  // the per-tile sort in the same launch (the host checked composite_sorts)
        if (accum_fp16)
            hipLaunchKernelGGL((k_composite_ts<true, 2>), dim3(grid), dim3(128), 0, s, p, *ts);
        else if (p.bands == 4)
            hipLaunchKernelGGL((k_composite_ts<false, 4>), dim3(grid), dim3(128), 0, s, p, *ts);
        else
            hipLaunchKernelGGL((k_composite_ts<false, 2>), dim3(grid), dim3(128), 0, s, p, *ts);
        return;
    }
    if (p.n_tiles <= kQuarterTiles) {  // (see kQuarterTiles)
        if (accum_fp16)
            hipLaunchKernelGGL(k_composite_q<true>, dim3(grid), dim3(256), 0, s, p);
        else
            hipLaunchKernelGGL(k_composite_q<false>, dim3(grid), dim3(256), 0, s, p);
    } else if (accum_fp16) {
        hipLaunchKernelGGL((k_composite<true, 1>), dim3(grid), dim3(128), 0, s, p);
    } else if (p.seg <= 1 && p.bands == 4) {  // (see CompositeParams::bands)
        hipLaunchKernelGGL((k_composite<false, 1, 4>), dim3(grid), dim3(128), 0, s, p);
    } else if (p.seg >= 4) {
        hipLaunchKernelGGL((k_composite<false, 4>), dim3(grid), dim3(512), 0, s, p);
    } else if (p.seg == 2) {
        hipLaunchKernelGGL((k_composite<false, 2>), dim3(grid), dim3(256), 0, s, p);
    } else {
        hipLaunchKernelGGL((k_composite<false, 1>), dim3(grid), dim3(128), 0, s, p);
    }
}

}  // namespace gs

#ifdef GS_CQ_TIME
extern "C" int gs_diag_cq_phase(unsigned long long* out) {  // out: 16384 x 4 x 4
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_cq_phase), sizeof(gs::g_cq_phase)) == hipSuccess ? 0 : -1;
}
extern "C" int gs_diag_cq_times(unsigned long long* out, int n) {  // out: n x 3 (read and zeroed)
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_cq_time), (size_t)n * 24) != hipSuccess) return -1;
    std::vector<unsigned long long> z((size_t)n * 3, 0ull);
    return hipMemcpyToSymbol(HIP_SYMBOL(gs::g_cq_time), z.data(), (size_t)n * 24) == hipSuccess ? 0 : -1;
}
#endif
#ifdef GS_C1_TIME
extern "C" int gs_diag_c1_times(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_c1_time), 16 * 8) == hipSuccess ? 0 : -1;
}
#endif
#ifdef GS_KTIME
extern "C" int gs_diag_kt(unsigned long long* out) {  // out: 2 x 8192 x 6
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_kt), sizeof(gs::g_kt)) == hipSuccess ? 0 : -1;
}
extern "C" int gs_diag_fe(unsigned long long* out) {  // out: 8
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_fe), sizeof(gs::g_fe)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef GS_TS_TIME
extern "C" int gs_diag_ts_time(unsigned long long* out) {  // out: 8 (read and zeroed)
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_ts_time), 64) != hipSuccess) return -1;
    const unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(gs::g_ts_time), z, 64) == hipSuccess ? 0 : -1;
}
#endif
#ifdef GS_COMP_DIAG
extern "C" int gs_diag_comp_times(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_comp_time), (size_t)n * 24) == hipSuccess ? 0 : -1;
}
extern "C" int gs_diag_comp_counters(unsigned long long* out, int n_tiles) {  // out: n_tiles x 2 x 8
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_comp_cnt), (size_t)n_tiles * 128) == hipSuccess ? 0 : -1;
}
#endif
