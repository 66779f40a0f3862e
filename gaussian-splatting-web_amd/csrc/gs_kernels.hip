// gs_kernels.hip — CDNA4 (gfx950) kernels of the splat forward path.
//
//   k_transpose   scene upload: reference AoS record (src/ply.ts:249-257) -> SoA planes
//   k_project     per Gaussian: depth key (src/shaders.ts:36-68) + vs_points projection
//                 (src/simple_render.ts:217-332) + SH colour (:26-66) + tile rectangle;
//                 streaming, one pass over the SoA planes; fuses the radix histograms.
//   k_sort_pass   one stable 8-bit LSD radix pass, Onesweep style (partition ticket +
//                 decoupled look-back); replaces webgpu-radix-sort's 16 x 2-bit passes (RS:621-654).
//   k_bin         per depth-sorted splat: (tile, splat) pairs emitted in depth order
//                 (order-preserving exclusive scan with look-back, wave64 ballot ranks).
//   k_ranges      per tile: [begin, end) of its list after the stable tile-id sort.
//   k_composite   16x16 tile workgroup: front-to-back "under" blending of fs_main's alpha
//                 (src/simple_render.ts:169-200, blend state :455-471), splat batches staged in LDS.
//
// Inter-workgroup hand-offs (look-back words) follow cdna_hip_programming.md Guideline 16 R2:
// the data word is the flag (one relaxed agent-scope store / load), state re-zeroed every call.
#include <algorithm>

#include "gs_device.h"

namespace gs {
namespace {

constexpr uint32_t kFlagAgg = 1u << 30, kFlagInc = 2u << 30, kValMask = (1u << 30) - 1;
constexpr unsigned long long kFlagAgg64 = 1ull << 62, kFlagInc64 = 2ull << 62,
                             kValMask64 = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

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

// Exclusive scan over a 256-thread block; returns exclusive prefix, *total = block sum.
// `tmp` = 4 words of LDS.  Contains __syncthreads().
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* tmp, uint32_t* total) {
    const uint32_t incl = wave_incl_scan(v);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 63) tmp[w] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < w; ++i) base += tmp[i];
    *total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    __syncthreads();
    return base + incl - v;
}

__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_relaxed64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ============================================================================ k_transpose
__global__ __launch_bounds__(256) void k_transpose(const uint8_t* __restrict__ aos, uint64_t n,
                                                   int n_sh, float* __restrict__ planes,
                                                   uint64_t stride) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* r = (const float*)(aos + i * (uint64_t)(64 + 16 * n_sh));
    // planes: 0-2 pos, 3-5 scale, 6-9 rot, 10 opacity logit, 11.. sh[k][c] at 11 + 3k + c
    planes[0 * stride + i] = r[0];
    planes[1 * stride + i] = r[1];
    planes[2 * stride + i] = r[2];
    planes[3 * stride + i] = r[4];
    planes[4 * stride + i] = r[5];
    planes[5 * stride + i] = r[6];
    planes[6 * stride + i] = r[8];
    planes[7 * stride + i] = r[9];
    planes[8 * stride + i] = r[10];
    planes[9 * stride + i] = r[11];
    planes[10 * stride + i] = r[12];
    for (int k = 0; k < n_sh; ++k)
        for (int c = 0; c < 3; ++c) planes[(uint64_t)(11 + 3 * k + c) * stride + i] = r[16 + 4 * k + c];
}

// ============================================================================ k_project
// SH evaluation, src/simple_render.ts:26-66, one colour channel; coefficients beyond the
// record's degree are absent (treated as 0; the reference draw shader assumes 16).
__device__ __forceinline__ float sh_channel(const float* __restrict__ planes, uint64_t S, uint32_t i,
                                            int c, int n_sh, float x, float y, float z) {
    auto C = [&](int k) { return planes[(uint64_t)(11 + 3 * k + c) * S + i]; };
    const float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
    float result = SH_C0 * C(0);
    if (n_sh > 1) result = result + SH_C1 * (-y * C(1) + z * C(2) - x * C(3));
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
    if (n_sh > 4)
        result = result + 1.0925484305920792f * xy * C(4) + -1.0925484305920792f * yz * C(5) +
                 0.31539156525252005f * (2.0f * zz - xx - yy) * C(6) +
                 -1.0925484305920792f * xz * C(7) + 0.5462742152960396f * (xx - yy) * C(8);
    if (n_sh > 9)
        result = result + -0.5900435899266435f * y * (3.0f * xx - yy) * C(9) +
                 2.890611442640554f * xy * z * C(10) +
                 -0.4570457994644658f * y * (4.0f * zz - xx - yy) * C(11) +
                 0.3731763325901154f * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * C(12) +
                 -0.4570457994644658f * x * (4.0f * zz - xx - yy) * C(13) +
                 1.445305721320277f * z * (xx - yy) * C(14) +
                 -0.5900435899266435f * x * (xx - 3.0f * yy) * C(15);
    result = result + 0.5f;
    return fmaxf(result, 0.0f);
}

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

__global__ __launch_bounds__(kProjThreads) void k_project(ProjParams p) {
    __shared__ uint32_t s_hist[4][256];
    __shared__ unsigned long long s_k;
    __shared__ uint32_t s_vis;
    for (int t = threadIdx.x; t < 1024; t += kProjThreads) (&s_hist[0][0])[t] = 0;
    if (threadIdx.x == 0) { s_k = 0; s_vis = 0; }
    __syncthreads();

    const uint64_t S = p.plane_stride;
    const float* __restrict__ P = p.planes;
    uint32_t my_vis = 0;
    unsigned long long my_k = 0;
    const int row_lo = p.tile_row_begin * kTile;
    const int row_hi = min(p.tile_row_end * kTile, p.H) - 1;

    for (uint32_t i = blockIdx.x * kProjThreads + threadIdx.x; i < p.n;
         i += gridDim.x * kProjThreads) {
        const float x = P[0 * S + i], y = P[1 * S + i], z = P[2 * S + i];
        const float sx = P[3 * S + i], sy = P[4 * S + i], sz = P[5 * S + i];
        const float qx = P[6 * S + i], qy = P[7 * S + i], qz = P[8 * S + i], qw = P[9 * S + i];
        const float logit = P[10 * S + i];

        float vz;
        float4 clip;
        Footprint f;
        project_footprint(p, x, y, z, sx, sy, sz, qx, qy, qz, qw, vz, clip, f);
        bool vis = (clip.w > 0.0f) && (clip.z >= 0.0f) && (clip.z <= clip.w);  // :230, near/far clip
        // sigmoid (:118-125)
        float op;
        if (logit >= 0.0f) {
            op = 1.0f / (1.0f + expf(-logit));
        } else {
            const float e = expf(logit);
            op = e / (1.0f + e);
        }
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

        uint32_t key = kSentinel;
        if (vis) {
            key = sortable_key(vz);
            // binning rectangle: quad box intersected with the alpha >= 1/255 disc box, widened by
            // a small margin so that float rounding can never drop a covered pixel
            const float R = sqrtf(fmaxf(logf(255.0f * op), 0.0f));
            float hx = fminf(qhx, R * sqrtf(f.e1x * f.e1x + f.e2x * f.e2x));
            float hy = fminf(qhy, R * sqrtf(f.e1y * f.e1y + f.e2y * f.e2y));
            hx = hx * 1.0001f + 0.02f;
            hy = hy * 1.0001f + 0.02f;
            float xl, xh, yl, yh;
            uint32_t ntiles = 0, rx = 0, ry = 0;
            if (pixel_rect(f.cx, f.cy, hx, hy, p.W, row_lo, row_hi, xl, xh, yl, yh)) {
                const int tx0 = (int)xl >> 4, tx1 = (int)xh >> 4, ty0 = (int)yl >> 4, ty1 = (int)yh >> 4;
                ntiles = (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1));
                rx = (uint32_t)tx0 | ((uint32_t)ty0 << 16);
                ry = (uint32_t)tx1 | ((uint32_t)ty1 << 16);
            }
            // colour (:321, dir = normalize(p - camPos))
            const float dx = x - p.cam[0], dy = y - p.cam[1], dz = z - p.cam[2];
            const float dl = sqrtf(dx * dx + dy * dy + dz * dz);
            const float X = dx / dl, Y = dy / dl, Z = dz / dl;
            const float cr = sh_channel(P, S, i, 0, p.n_sh, X, Y, Z);
            const float cg = sh_channel(P, S, i, 1, p.n_sh, X, Y, Z);
            const float cb = sh_channel(P, S, i, 2, p.n_sh, X, Y, Z);
            const float n1 = f.e1x * f.e1x + f.e1y * f.e1y, n2 = f.e2x * f.e2x + f.e2y * f.e2y;
            float4* r = p.rec + 4 * (uint64_t)i;
            r[0] = make_float4(f.cx, f.cy, f.e1x / n1, f.e1y / n1);
            r[1] = make_float4(f.e2x / n2, f.e2y / n2, op, cr);
            r[2] = make_float4(cg, cb, __uint_as_float(rx), __uint_as_float(ry));
            r[3] = make_float4(__uint_as_float(key), __uint_as_float(ntiles), 0.0f, 0.0f);
            atomicAdd(&s_hist[0][key & 255], 1u);
            atomicAdd(&s_hist[1][(key >> 8) & 255], 1u);
            atomicAdd(&s_hist[2][(key >> 16) & 255], 1u);
            atomicAdd(&s_hist[3][key >> 24], 1u);
            ++my_vis;
            my_k += ntiles;
        }
        p.keys_out[i] = key;
    }
    if (my_vis) {
        atomicAdd(&s_vis, my_vis);
        atomicAdd(&s_k, my_k);
    }
    __syncthreads();
    uint32_t* gh = p.hist + (blockIdx.x % kHistShards) * 1024;
    for (int t = threadIdx.x; t < 1024; t += kProjThreads) {
        const uint32_t c = (&s_hist[0][0])[t];
        if (c) atomicAdd(gh + t, c);
    }
    if (threadIdx.x == 0 && s_vis) {
        atomicAdd(p.counters + 0, (unsigned long long)s_vis);
        atomicAdd(p.counters + 1, s_k);
    }
}

// ============================================================================ histograms
// Digit histograms of an arbitrary key array (used by the standalone sort entry point).
__global__ __launch_bounds__(256) void k_hist_keys(const uint32_t* __restrict__ keys, uint32_t n,
                                                   int begin_bit, int end_bit, int npass,
                                                   uint32_t* hist) {
    __shared__ uint32_t s_hist[4][256];
    for (int t = threadIdx.x; t < 1024; t += 256) (&s_hist[0][0])[t] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint32_t k = keys[i];
        for (int ps = 0; ps < npass; ++ps) {
            const int sh = begin_bit + 8 * ps;
            const uint32_t mask = (1u << min(8, end_bit - sh)) - 1u;
            atomicAdd(&s_hist[ps][(k >> sh) & mask], 1u);
        }
    }
    __syncthreads();
    uint32_t* gh = hist + (blockIdx.x % kHistShards) * (npass * 256);
    for (int t = threadIdx.x; t < npass * 256; t += 256) {
        const uint32_t c = (&s_hist[0][0])[t];
        if (c) atomicAdd(gh + t, c);
    }
}

// ============================================================================ k_sort_pass
// One stable LSD pass.  Partition = 4096 consecutive elements, owned by the workgroup that drew
// its ticket (so every predecessor it waits on is already running).  Per partition:
//   1. wave-ordered stable ranking: element order inside the partition is (wave, item, lane);
//      peers with the same digit are found with 8 ballots, counts kept per wave in LDS;
//   2. digit counts published as an aggregate, decoupled look-back for the exclusive prefix;
//   3. scatter through an LDS staging area so global writes of one digit run are contiguous.
__global__ __launch_bounds__(kSortThreads) void k_sort_pass(SortPass p) {
    __shared__ uint32_t s_wave_hist[4][256];
    __shared__ uint32_t s_digit_start[256];
    __shared__ uint32_t s_global[256];
    __shared__ uint32_t s_keys[kSortTile];
    __shared__ uint32_t s_vals[kSortTile];
    __shared__ uint32_t s_tmp[8];
    __shared__ uint32_t s_part;

    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    if (tid == 0) s_part = atomicAdd(p.ticket, 1u);
    for (int t = tid; t < 1024; t += kSortThreads) (&s_wave_hist[0][0])[t] = 0;
    // global digit base for this pass: exclusive scan over bins of the sharded histogram
    uint32_t gcount = 0;
    for (int sh = 0; sh < kHistShards; ++sh) gcount += p.hist[sh * p.hist_stride + tid];
    uint32_t gtotal;
    const uint32_t gbase = block_excl_scan256(gcount, s_tmp, &gtotal);  // has __syncthreads
    const uint32_t part = s_part;
    const uint64_t base = (uint64_t)part * kSortTile;

    uint32_t keys[kSortIPT], vals[kSortIPT], rank[kSortIPT];
    const uint64_t wbase = base + (uint64_t)w * (kSortIPT * 64);
#pragma unroll
    for (int it = 0; it < kSortIPT; ++it) {
        const uint64_t idx = wbase + it * 64 + lane;
        const bool in = idx < p.n;
        keys[it] = in ? p.keys_in[idx] : kSentinel;
        vals[it] = in ? (p.vals_in ? p.vals_in[idx] : (uint32_t)idx) : 0u;
        // valid marker folded into rank's top bit until ranked
        const bool valid = in && !(p.filter_sentinel && keys[it] == kSentinel);
        rank[it] = valid ? 0u : 0x80000000u;
    }
#pragma unroll
    for (int it = 0; it < kSortIPT; ++it) {
        const bool valid = (rank[it] & 0x80000000u) == 0u;
        const uint32_t digit = (keys[it] >> p.shift) & p.mask;
        uint64_t peers = __ballot(valid);
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

    // per digit (thread = digit): wave offsets, partition count, publish, look-back
    const int d = tid;
    const uint32_t c0 = s_wave_hist[0][d], c1 = s_wave_hist[1][d], c2 = s_wave_hist[2][d],
                   c3 = s_wave_hist[3][d];
    const uint32_t cnt = c0 + c1 + c2 + c3;
    uint32_t* st = p.status + (uint64_t)part * 256;
    st_relaxed(st + d, (part == 0 ? kFlagInc : kFlagAgg) | cnt);
    uint32_t excl = 0;
    if (part > 0) {
        int64_t q = (int64_t)part - 1;
        uint32_t spins = 0;
        while (q >= 0) {
            const uint32_t s = ld_relaxed(p.status + (uint64_t)q * 256 + d);
            const uint32_t flag = s & ~kValMask;
            if (flag == 0u) {
                if (++spins > kSpinLimit) { atomicOr(p.err, kErrSpinSort); break; }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += s & kValMask;
            if (flag == kFlagInc) break;
            --q;
        }
        st_relaxed(st + d, kFlagInc | (excl + cnt));
    }
    uint32_t tile_total;
    const uint32_t dstart = block_excl_scan256(cnt, s_tmp, &tile_total);  // has __syncthreads
    s_digit_start[d] = dstart;
    s_global[d] = gbase + excl;
    s_wave_hist[0][d] = 0;
    s_wave_hist[1][d] = c0;
    s_wave_hist[2][d] = c0 + c1;
    s_wave_hist[3][d] = c0 + c1 + c2;
    __syncthreads();

#pragma unroll
    for (int it = 0; it < kSortIPT; ++it) {
        if ((rank[it] & 0x80000000u) == 0u) {
            const uint32_t digit = (keys[it] >> p.shift) & p.mask;
            const uint32_t pos = s_digit_start[digit] + s_wave_hist[w][digit] + rank[it];
            s_keys[pos] = keys[it];
            s_vals[pos] = vals[it];
        }
    }
    __syncthreads();
    for (uint32_t q = tid; q < tile_total; q += kSortThreads) {
        const uint32_t k = s_keys[q];
        const uint32_t digit = (k >> p.shift) & p.mask;
        const uint32_t dest = s_global[digit] + (q - s_digit_start[digit]);
        p.keys_out[dest] = k;
        p.vals_out[dest] = s_vals[q];
    }
}

// ============================================================================ k_bin
__global__ __launch_bounds__(kBinThreads) void k_bin(BinParams p) {
    __shared__ uint32_t s_off[kBinTile + 1];
    __shared__ uint32_t s_j[kBinTile];
    __shared__ uint2 s_rect[kBinTile];
    __shared__ uint32_t s_hist[2][256];
    __shared__ uint32_t s_tmp[8];
    __shared__ uint32_t s_part;
    __shared__ unsigned long long s_base;

    const int tid = threadIdx.x;
    if (tid == 0) s_part = atomicAdd(p.ticket, 1u);
    s_hist[0][tid] = 0;
    s_hist[1][tid] = 0;
    __syncthreads();
    const uint32_t part = s_part;
    const uint64_t base = (uint64_t)part * kBinTile;
    const uint32_t nitems = (uint32_t)min((uint64_t)kBinTile, (uint64_t)p.n_vis - base);

    uint32_t cnt[kBinIPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < kBinIPT; ++k) {
        const uint32_t li = tid * kBinIPT + k;
        cnt[k] = 0;
        if (li < nitems) {
            const uint32_t j = p.sorted_vals[base + li];
            const float4 c = p.rec[4 * (uint64_t)j + 2];
            const uint32_t rx = __float_as_uint(c.z), ry = __float_as_uint(c.w);
            cnt[k] = __float_as_uint(p.rec[4 * (uint64_t)j + 3].y);  // 0: no pixel reaches 1/255
            s_j[li] = j;
            s_rect[li] = make_uint2(rx, ry);
        }
        tsum += cnt[k];
    }
    uint32_t total;
    uint32_t run = block_excl_scan256(tsum, s_tmp, &total);
#pragma unroll
    for (int k = 0; k < kBinIPT; ++k) {
        s_off[tid * kBinIPT + k] = run;
        run += cnt[k];
    }
    if (tid == 0) {
        unsigned long long* st = p.status + part;
        st_relaxed64(st, (part == 0 ? kFlagInc64 : kFlagAgg64) | (unsigned long long)total);
        unsigned long long excl = 0;
        if (part > 0) {
            int64_t q = (int64_t)part - 1;
            uint32_t spins = 0;
            while (q >= 0) {
                const unsigned long long s = ld_relaxed64(p.status + q);
                const unsigned long long flag = s & ~kValMask64;
                if (flag == 0ull) {
                    if (++spins > kSpinLimit) { atomicOr(p.err, kErrSpinBin); break; }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += s & kValMask64;
                if (flag == kFlagInc64) break;
                --q;
            }
            st_relaxed64(st, kFlagInc64 | (excl + total));
        }
        s_base = excl;
    }
    __syncthreads();
    const unsigned long long obase = s_base;
    if (obase + total > p.capacity) {
        if (tid == 0) atomicOr(p.err, kErrOverflow);
        return;
    }
    // cooperative, coalesced emission of this partition's entries (depth order preserved)
    for (uint32_t e = tid; e < total; e += kBinThreads) {
        int lo = 0, hi = (int)nitems - 1;
        while (lo < hi) {  // largest s with s_off[s] <= e
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= e) lo = mid; else hi = mid - 1;
        }
        const uint2 rc = s_rect[lo];
        const uint32_t k = e - s_off[lo];
        const uint32_t w = (rc.y & 0xffffu) - (rc.x & 0xffffu) + 1u;
        const uint32_t tx = (rc.x & 0xffffu) + k % w;
        const uint32_t ty = (rc.x >> 16) + k / w;
        const uint32_t tile = (ty - (uint32_t)p.tile_row_begin) * (uint32_t)p.tiles_x + tx;
        p.tkeys[obase + e] = tile;
        p.tvals[obase + e] = s_j[lo];
        atomicAdd(&s_hist[0][tile & 255], 1u);
        atomicAdd(&s_hist[1][(tile >> 8) & 255], 1u);
    }
    __syncthreads();
    uint32_t* gh = p.hist + (blockIdx.x % kHistShards) * 512;
    for (int t = tid; t < 512; t += kBinThreads) {
        const uint32_t c = (&s_hist[0][0])[t];
        if (c) atomicAdd(gh + t, c);
    }
}

// ============================================================================ k_ranges
__global__ __launch_bounds__(256) void k_ranges(const uint32_t* __restrict__ tkeys, uint64_t k,
                                                uint2* __restrict__ ranges) {
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < k;
         q += (uint64_t)gridDim.x * 256) {
        const uint32_t t = tkeys[q];
        if (q == 0 || tkeys[q - 1] != t) ranges[t].x = (uint32_t)q;
        if (q == k - 1 || tkeys[q + 1] != t) ranges[t].y = (uint32_t)(q + 1);
    }
}

// ============================================================================ k_composite
// One workgroup per 16x16 tile, one pixel per thread.  Splats of the tile's list (depth order)
// are staged 256 at a time in LDS; every pixel evaluates fs_main's alpha at its centre and
// blends front to back with the reference's blend state:
//   dst.rgb = (col*alpha)*(1-dst.a) + dst.rgb ; dst.a = alpha*(1-dst.a) + dst.a
// A pixel is done once dst.a == 1 (nothing can change it) or 1-dst.a < t_min; the workgroup
// leaves as soon as every pixel is done.
template <bool FP16_TARGET>
__global__ __launch_bounds__(256) void k_composite(CompositeParams p) {
    __shared__ float4 s_a[256];
    __shared__ float4 s_b[256];
    __shared__ float2 s_c[256];
    const int tid = threadIdx.x;
    const int tile = blockIdx.x;
    const int tx = tile % p.tiles_x, ty = tile / p.tiles_x + p.tile_row_begin;
    const int px = tx * kTile + (tid & 15), py = ty * kTile + (tid >> 4);
    const bool inside = px < p.W && py < p.H;
    const float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
    const uint2 range = p.ranges[tile];
    float cr = 0.0f, cg = 0.0f, cb = 0.0f, ca = 0.0f;
    bool done = !inside;
    for (uint32_t b0 = range.x; b0 < range.y; b0 += 256) {
        const uint32_t e = b0 + tid;
        if (e < range.y) {
            const uint32_t j = p.tvals[e];
            const float4* r = p.rec + 4 * (uint64_t)j;
            s_a[tid] = r[0];
            s_b[tid] = r[1];
            const float4 c = r[2];
            s_c[tid] = make_float2(c.x, c.y);
        }
        __syncthreads();
        const int cnt = (int)min(256u, range.y - b0);
        if (!done) {
            for (int k = 0; k < cnt; ++k) {
                const float4 A = s_a[k];
                const float dx = fx - A.x, dy = fy - A.y;
                const float u = dx * A.z + dy * A.w;
                const float4 B = s_b[k];
                const float v = dx * B.x + dy * B.y;
                if (fabsf(u) <= 2.0f && fabsf(v) <= 2.0f) {
                    const float alpha = fminf(__expf(-(u * u + v * v)) * B.z, 1.0f);
                    if (alpha >= 1.0f / 255.0f) {
                        const float2 C = s_c[k];
                        const float om = 1.0f - ca;
                        cr = (B.w * alpha) * om + cr;
                        cg = (C.x * alpha) * om + cg;
                        cb = (C.y * alpha) * om + cb;
                        ca = alpha * om + ca;
                        if (FP16_TARGET) {
                            cr = (float)(_Float16)cr;
                            cg = (float)(_Float16)cg;
                            cb = (float)(_Float16)cb;
                            ca = (float)(_Float16)ca;
                        }
                        if (ca >= 1.0f || 1.0f - ca < p.t_min) { done = true; break; }
                    }
                }
            }
        }
        if (__syncthreads_count(!done) == 0) break;
    }
    if (inside) {
        const uint64_t o = (uint64_t)(py - p.row0) * p.W + px;
        if (p.out_f16) {
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            h4 h = {(_Float16)cr, (_Float16)cg, (_Float16)cb, (_Float16)ca};
            ((h4*)p.out)[o] = h;
        } else {
            ((float4*)p.out)[o] = make_float4(cr, cg, cb, ca);
        }
    }
}

}  // namespace

// ============================================================================ launchers
void launch_transpose(const uint8_t* aos, uint64_t n, int n_sh, float* planes, uint64_t stride,
                      hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_transpose, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, aos, n, n_sh,
                       planes, stride);
}
void launch_project(const ProjParams& p, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_project, dim3(grid), dim3(kProjThreads), 0, s, p);
}
void launch_hist_keys(const uint32_t* keys, uint32_t n, int begin_bit, int end_bit, int npass,
                      uint32_t* hist, hipStream_t s) {
    const unsigned grid = (unsigned)std::min<uint64_t>(1024, (n + 255) / 256 + 1);
    hipLaunchKernelGGL(k_hist_keys, dim3(grid), dim3(256), 0, s, keys, n, begin_bit, end_bit, npass,
                       hist);
}
void launch_sort_pass(const SortPass& p, hipStream_t s) {
    const uint32_t parts = sort_parts(p.n);
    if (!parts) return;
    hipLaunchKernelGGL(k_sort_pass, dim3(parts), dim3(kSortThreads), 0, s, p);
}
void launch_bin(const BinParams& p, hipStream_t s) {
    const uint32_t parts = bin_parts(p.n_vis);
    if (!parts) return;
    hipLaunchKernelGGL(k_bin, dim3(parts), dim3(kBinThreads), 0, s, p);
}
void launch_ranges(const uint32_t* tkeys, uint64_t k, uint2* ranges, hipStream_t s) {
    if (!k) return;
    const unsigned grid = (unsigned)std::min<uint64_t>(8192, (k + 255) / 256);
    hipLaunchKernelGGL(k_ranges, dim3(grid), dim3(256), 0, s, tkeys, k, ranges);
}
void launch_composite(const CompositeParams& p, int accum_fp16, hipStream_t s) {
    if (p.n_tiles <= 0) return;
    if (accum_fp16)
        hipLaunchKernelGGL(k_composite<true>, dim3(p.n_tiles), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL(k_composite<false>, dim3(p.n_tiles), dim3(256), 0, s, p);
}

}  // namespace gs
