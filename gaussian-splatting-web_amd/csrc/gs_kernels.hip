// gs_kernels.hip — CDNA4 (gfx950) kernels of the splat forward path.
//
//   k_transpose   scene upload: reference AoS record (src/ply.ts:249-257) -> SoA planes
//   k_project     per Gaussian: depth key (src/shaders.ts:36-68) + vs_points projection
//                 (src/simple_render.ts:217-332) + SH colour (:26-66) + tile rectangle;
//                 streaming, one pass over the SoA planes; fuses the radix histograms.
//   k_radix_*     one stable 8-bit LSD radix pass (upsweep / scan / downsweep); replaces
//                 webgpu-radix-sort's 16 x 2-bit passes (RS:621-654).
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
    __shared__ unsigned long long s_k;
    __shared__ uint32_t s_vis;
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

        uint32_t key = kSentinel, prect = kRectEmpty;
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
            uint32_t ntiles = 0, rx = 0, ry = 0, bbx = 0xFFFFu, bby = 0xFFFFu;  // empty box
            if (pixel_rect(f.cx, f.cy, hx, hy, p.W, row_lo, row_hi, xl, xh, yl, yh)) {
                bbx = (uint32_t)xl | ((uint32_t)xh << 16);
                bby = (uint32_t)yl | ((uint32_t)yh << 16);
                const uint32_t tx0 = (uint32_t)xl >> 4, tx1 = (uint32_t)xh >> 4,
                               ty0 = (uint32_t)yl >> 4, ty1 = (uint32_t)yh >> 4;
                ntiles = (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
                rx = tx0 | (ty0 << 16);
                ry = tx1 | (ty1 << 16);
                prect = (tx1 - tx0 < 16 && ty1 - ty0 < 16)
                            ? (tx0 | (ty0 << 12) | ((tx1 - tx0) << 24) | ((ty1 - ty0) << 28))
                            : kRectLarge;
            }
            // colour (:321, dir = normalize(p - camPos))
            const float dx = x - p.cam[0], dy = y - p.cam[1], dz = z - p.cam[2];
            const float dl = sqrtf(dx * dx + dy * dy + dz * dz);
            const float X = dx / dl, Y = dy / dl, Z = dz / dl;
            const float cr = sh_channel(P, S, i, 0, p.n_sh, X, Y, Z);
            const float cg = sh_channel(P, S, i, 1, p.n_sh, X, Y, Z);
            const float cb = sh_channel(P, S, i, 2, p.n_sh, X, Y, Z);
            // composite record: u' = d.(e1/|e1|^2)*sqrt(log2 e), so u'^2+v'^2 = (u^2+v^2) log2 e and
            // alpha = op * exp(-(u^2+v^2)) = exp2(log2(op) - (u'^2+v'^2))
            const float k1 = kSqrtLog2e / (f.e1x * f.e1x + f.e1y * f.e1y);
            const float k2 = kSqrtLog2e / (f.e2x * f.e2x + f.e2y * f.e2y);
            float4* r = p.rec + 4 * (uint64_t)i;
            r[0] = make_float4(f.cx, f.cy, f.e1x * k1, f.e1y * k1);
            r[1] = make_float4(f.e2x * k2, f.e2y * k2, log2f(op), cr);
            r[2] = make_float4(cg, cb, __uint_as_float(bbx), __uint_as_float(bby));
            r[3] = make_float4(__uint_as_float(key), __uint_as_float(ntiles), __uint_as_float(rx),
                               __uint_as_float(ry));
            ++my_vis;
            my_k += ntiles;
        }
        p.keys_out[i] = key;
        p.rect_out[i] = prect;
    }
    if (my_vis) {
        atomicAdd(&s_vis, my_vis);
        atomicAdd(&s_k, my_k);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_vis) {
        atomicAdd(&p.ctl->n_vis, s_vis);
        atomicAdd(&p.ctl->k_total, s_k);
    }
}

// ============================================================================ radix pass
// One stable LSD pass = three launches, no inter-workgroup waiting:
//   k_radix_upsweep    per 4096-element partition: digit histogram -> counts[digit][part]
//   k_radix_scan       per digit: offsets[digit][part] = base[digit] + sum of earlier partitions
//   k_radix_downsweep  per partition: stable local ranks (wave ballots, element order inside the
//                      partition = (wave, item, lane)), LDS staging, contiguous writes per digit run
// This replaces webgpu-radix-sort's 16 x 2-bit passes (RS:621-654) with 8-bit digits.

__device__ __forceinline__ uint32_t radix_n(const SortPass& p) { return p.n_dev ? *p.n_dev : p.n; }
__device__ __forceinline__ bool radix_valid(const SortPass& p, uint32_t n, uint64_t idx, uint32_t key) {
    return idx < n && !(p.filter_sentinel && key == kSentinel);
}

__global__ __launch_bounds__(kSortThreads) void k_radix_upsweep(SortPass p) {
    __shared__ uint32_t s_hist[4][256];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t n = radix_n(p), parts = sort_parts(n);
    uint32_t total = 0;  // this workgroup's count of digit `tid` over all its partitions
    for (uint32_t part = blockIdx.x; part < parts; part += gridDim.x) {
        for (int t = tid; t < 1024; t += kSortThreads) (&s_hist[0][0])[t] = 0;
        __syncthreads();
        const uint64_t wbase = (uint64_t)part * kSortTile + (uint64_t)w * (kSortIPT * 64);
#pragma unroll 4
        for (int it = 0; it < kSortIPT; ++it) {
            const uint64_t idx = wbase + it * 64 + lane;
            const uint32_t key = idx < n ? p.keys_in[idx] : kSentinel;
            if (radix_valid(p, n, idx, key)) atomicAdd(&s_hist[w][(key >> p.shift) & p.mask], 1u);
        }
        __syncthreads();
        const uint32_t c = s_hist[0][tid] + s_hist[1][tid] + s_hist[2][tid] + s_hist[3][tid];
        p.offsets[(uint64_t)tid * p.parts_max + part] = c;  // digit-major
        total += c;
        __syncthreads();
    }
    // global digit histogram of this pass (kHistShards shards, zeroed with the frame)
    if (total) atomicAdd(&p.hist[(blockIdx.x % kHistShards) * 256 + tid], total);
}

// Block d scans column d over partitions and adds the global digit base (exclusive scan of the
// global histogram, which the producing kernel accumulated in kHistShards shards).
__global__ __launch_bounds__(256) void k_radix_scan(SortPass p) {
    __shared__ uint32_t s_tmp[8];
    __shared__ uint32_t s_base;
    const int d = blockIdx.x, tid = threadIdx.x;
    const uint32_t parts = sort_parts(radix_n(p));
    uint32_t tot = 0;
    for (int sh = 0; sh < kHistShards; ++sh) tot += p.hist[sh * 256 + tid];
    uint32_t gtotal;
    const uint32_t gbase = block_excl_scan256(tot, s_tmp, &gtotal);
    if (tid == d) s_base = gbase;
    __syncthreads();
    uint32_t* col = p.offsets + (uint64_t)d * p.parts_max;
    const uint32_t per = (parts + 255) / 256;
    const uint32_t b0 = min(parts, tid * per), b1 = min(parts, b0 + per);
    uint32_t sum = 0;
    for (uint32_t i = b0; i < b1; ++i) sum += col[i];
    uint32_t total;
    uint32_t run = s_base + block_excl_scan256(sum, s_tmp, &total);
    for (uint32_t i = b0; i < b1; ++i) {
        const uint32_t c = col[i];
        col[i] = run;
        run += c;
    }
}

__global__ __launch_bounds__(kSortThreads) void k_radix_downsweep(SortPass p) {
    __shared__ uint32_t s_wave_hist[4][256];
    __shared__ uint32_t s_digit_start[256];
    __shared__ uint32_t s_global[256];
    __shared__ uint32_t s_keys[kSortTile];
    __shared__ uint32_t s_vals[kSortTile];
    __shared__ uint32_t s_aux[kSortTile];
    __shared__ uint32_t s_tmp[8];

    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t n = radix_n(p), parts = sort_parts(n);
    const bool has_aux = p.aux_in != nullptr;
    for (uint32_t part = blockIdx.x; part < parts; part += gridDim.x) {
        for (int t = tid; t < 1024; t += kSortThreads) (&s_wave_hist[0][0])[t] = 0;
        s_global[tid] = p.offsets[(uint64_t)tid * p.parts_max + part];
        const uint64_t wbase = (uint64_t)part * kSortTile + (uint64_t)w * (kSortIPT * 64);

        uint32_t keys[kSortIPT], vals[kSortIPT], aux[kSortIPT], rank[kSortIPT];
#pragma unroll
        for (int it = 0; it < kSortIPT; ++it) {
            const uint64_t idx = wbase + it * 64 + lane;
            const bool in = idx < n;
            keys[it] = in ? p.keys_in[idx] : kSentinel;
            vals[it] = in ? (p.vals_in ? p.vals_in[idx] : (uint32_t)idx) : 0u;
            aux[it] = (in && has_aux) ? p.aux_in[idx] : 0u;
            rank[it] = radix_valid(p, n, idx, keys[it]) ? 0u : 0x80000000u;  // top bit: unsorted
        }
        __syncthreads();
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
        for (int it = 0; it < kSortIPT; ++it) {
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
    }
}

// ============================================================================ binning
// Chunk c covers depth ranks [r0, r1): chunk 0 = the first ceil(f * n_vis) ranks, chunk 1 = the
// rest, binned only into tiles that were not saturated by chunk 0 (empty when all are).
// Three launches per chunk, no inter-workgroup waiting: per-partition entry counts, one scan,
// then the emission in depth order (cooperative, coalesced) plus the tile-id digit histograms.
__device__ __forceinline__ void chunk_range(const BinParams& p, uint32_t& r0, uint32_t& r1) {
    const uint32_t n = p.ctl->n_vis;
    const uint32_t c0 = p.chunk_f >= 1.0f
                            ? n
                            : min(n, max(kMinChunk0, (uint32_t)ceilf(p.chunk_f * (float)n)));
    if (p.chunk == 0) {
        r0 = 0;
        r1 = c0;
    } else {
        r0 = c0;
        r1 = p.ctl->not_done ? n : c0;
    }
}

struct TileRect {
    uint32_t x0, y0, x1, y1;  // inclusive, absolute tile coordinates
};

__device__ __forceinline__ bool rect_unpack(const BinParams& p, uint32_t pr, uint32_t j, TileRect& r) {
    if (pr == kRectEmpty) return false;
    if (pr == kRectLarge) {
        const float4 m = p.rec[4 * (uint64_t)j + 3];
        const uint32_t rx = __float_as_uint(m.z), ry = __float_as_uint(m.w);
        r = {rx & 0xffffu, rx >> 16, ry & 0xffffu, ry >> 16};
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

// entries of one splat in this chunk (chunk 1: only unsaturated tiles)
__device__ __forceinline__ uint32_t rect_count(const BinParams& p, const TileRect& r) {
    if (p.chunk == 0) return (r.x1 - r.x0 + 1) * (r.y1 - r.y0 + 1);
    uint32_t c = 0;
    for (uint32_t ty = r.y0; ty <= r.y1; ++ty)
        for (uint32_t tx = r.x0; tx <= r.x1; ++tx) c += p.done[tile_id(p, tx, ty)] ? 0u : 1u;
    return c;
}

__global__ __launch_bounds__(kBinThreads) void k_bin_count(BinParams p) {
    __shared__ uint32_t s_tmp[8];
    uint32_t r0, r1;
    chunk_range(p, r0, r1);
    const uint32_t parts = bin_parts(r1 - r0);
    for (uint32_t part = blockIdx.x; part < parts; part += gridDim.x) {
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < kBinIPT; ++k) {
            const uint32_t r = r0 + part * kBinTile + threadIdx.x * kBinIPT + k;
            if (r < r1) {
                TileRect tr;
                if (rect_unpack(p, p.sorted_rect[r], p.sorted_vals[r], tr)) sum += rect_count(p, tr);
            }
        }
        uint32_t total;
        block_excl_scan256(sum, s_tmp, &total);
        if (threadIdx.x == 0) p.part_tot[part] = total;
    }
}

// single workgroup: exclusive scan of the partition totals (in place), entry count, capacity
__global__ __launch_bounds__(1024) void k_bin_scan(BinParams p) {
    __shared__ uint32_t s_w[16];
    uint32_t r0, r1;
    chunk_range(p, r0, r1);
    const uint32_t parts = bin_parts(r1 - r0);
    const uint32_t tid = threadIdx.x, per = (parts + 1023) / 1024;
    const uint32_t b0 = min(parts, tid * per), b1 = min(parts, b0 + per);
    unsigned long long sum = 0;
    for (uint32_t i = b0; i < b1; ++i) sum += p.part_tot[i];
    // 64-bit inclusive wave scan, then across the 16 waves
    unsigned long long incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long t = __shfl_up(incl, d, 64);
        if ((int)lane_id() >= d) incl += t;
    }
    __shared__ unsigned long long s_wsum[16];
    if (lane_id() == 63) s_wsum[tid >> 6] = incl;
    __syncthreads();
    unsigned long long base = 0, total = 0;
    for (uint32_t i = 0; i < 16; ++i) {
        if (i < (tid >> 6)) base += s_wsum[i];
        total += s_wsum[i];
    }
    unsigned long long run = base + incl - sum;
    for (uint32_t i = b0; i < b1; ++i) {
        const uint32_t c = p.part_tot[i];
        p.part_tot[i] = (uint32_t)min(run, (unsigned long long)p.capacity);
        run += c;
    }
    if (tid == 0) {
        p.ctl->k_chunk[p.chunk] = (uint32_t)min(total, (unsigned long long)p.capacity);
        if (total > p.capacity) atomicOr(&p.ctl->err, kErrOverflow);
    }
    (void)s_w;
}

__global__ __launch_bounds__(kBinThreads) void k_bin_emit(BinParams p) {
    __shared__ uint32_t s_off[kBinTile + 1];
    __shared__ uint32_t s_j[kBinTile];
    __shared__ TileRect s_rect[kBinTile];
    __shared__ uint32_t s_tmp[8];
    const int tid = threadIdx.x;
    uint32_t r0, r1;
    chunk_range(p, r0, r1);
    const uint32_t parts = bin_parts(r1 - r0);
    for (uint32_t part = blockIdx.x; part < parts; part += gridDim.x) {
        const uint32_t base_r = r0 + part * kBinTile;
        const uint32_t nitems = min((uint32_t)kBinTile, r1 - base_r);
        uint32_t cnt[kBinIPT];
        uint32_t tsum = 0;
#pragma unroll
        for (int k = 0; k < kBinIPT; ++k) {
            const uint32_t li = tid * kBinIPT + k;
            cnt[k] = 0;
            if (li < nitems) {
                const uint32_t j = p.sorted_vals[base_r + li];
                TileRect tr;
                if (rect_unpack(p, p.sorted_rect[base_r + li], j, tr)) cnt[k] = rect_count(p, tr);
                s_j[li] = j;
                s_rect[li] = tr;
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
        __syncthreads();
        const uint32_t obase = p.part_tot[part];
        if (p.chunk == 0) {
            // cooperative, coalesced emission (depth order preserved within every tile)
            for (uint32_t e = tid; e < total; e += kBinThreads) {
                if (obase + e >= p.capacity) break;
                int lo = 0, hi = (int)nitems - 1;
                while (lo < hi) {  // largest s with s_off[s] <= e
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_off[mid] <= e) lo = mid; else hi = mid - 1;
                }
                const TileRect tr = s_rect[lo];
                const uint32_t k = e - s_off[lo];
                const uint32_t w = tr.x1 - tr.x0 + 1;
                const uint32_t tile = tile_id(p, tr.x0 + k % w, tr.y0 + k / w);
                p.tkeys[obase + e] = tile;
                p.tvals[obase + e] = s_j[lo];
            }
        } else {
            // chunk 1 (few unsaturated tiles): every splat walks its own rectangle
#pragma unroll
            for (int k = 0; k < kBinIPT; ++k) {
                const uint32_t li = tid * kBinIPT + k;
                if (li >= nitems || cnt[k] == 0) continue;
                const TileRect tr = s_rect[li];
                uint32_t o = obase + s_off[li];
                for (uint32_t ty = tr.y0; ty <= tr.y1; ++ty)
                    for (uint32_t tx = tr.x0; tx <= tr.x1; ++tx) {
                        const uint32_t tile = tile_id(p, tx, ty);
                        if (p.done[tile]) continue;
                        if (o < p.capacity) {
                            p.tkeys[o] = tile;
                            p.tvals[o] = s_j[li];
                        }
                        ++o;
                    }
            }
        }
        __syncthreads();
    }
}

// ============================================================================ k_ranges
__global__ __launch_bounds__(256) void k_ranges(const uint32_t* __restrict__ tkeys,
                                                const uint32_t* __restrict__ k_dev,
                                                uint2* __restrict__ ranges) {
    const uint32_t k = *k_dev;
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < k; q += gridDim.x * 256) {
        const uint32_t t = tkeys[q];
        if (q == 0 || tkeys[q - 1] != t) ranges[t].x = q;
        if (q == k - 1 || tkeys[q + 1] != t) ranges[t].y = q + 1;
    }
}

// ============================================================================ k_composite
// Workgroup = one 16x16 tile; wave w owns the 8x8 quarter (w&1, w>>1), lane = one pixel.
// The tile's depth-ordered list is consumed in batches of 256 splats: every thread gathers one
// 48-B record into registers (next batch issued before the current one is blended) and parks it
// in a double-buffered LDS stage; each wave then walks the batch on its own, skips splats whose
// pixel box misses its quarter, and stops blending once its 64 pixels are saturated.  Per pixel,
// fs_main's alpha = saturate(op * exp(-dot(uv,uv))), discarded below 1/255 and outside
// |u|,|v| <= 2, is blended front to back with the reference's blend state
// (src/simple_render.ts:169-200, :455-471):
//   FP32        transmittance form: C += col * alpha * T, T *= 1 - alpha; no splat is accepted
//               once T < t_min;
//   FP16_TARGET dst = src * (1 - dst.a) + dst rounded to fp16 after every blend (rgba16float).
// Chunked frames: mode kCompFirst marks saturated tiles done (and writes them out) and parks the
// per-pixel state of the others; kCompSecond resumes those from the state with chunk 1's list.
template <bool FP16_TARGET>
__global__ __launch_bounds__(256) void k_composite(CompositeParams p) {
    __shared__ float4 sA[2][256];  // cx, cy, a, b
    __shared__ float4 sB[2][256];  // c, d, log2(op), r
    __shared__ float2 sC[2][256];  // g, b
    __shared__ uint2 sD[2][256];   // pixel box
    const int tid = threadIdx.x;
    const int tile = blockIdx.x;
    if (p.mode == kCompSecond && p.done[tile]) return;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int tx = tile % p.tiles_x, ty = tile / p.tiles_x + p.tile_row_begin;
    const int bx0 = tx * kTile + (w & 1) * 8, by0 = ty * kTile + (w >> 1) * 8;
    const int px = bx0 + (lane & 7), py = by0 + (lane >> 3);
    const bool inside = px < p.W && py < p.H;
    const float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
    const uint2 range = p.ranges[tile];
    const float4* __restrict__ rec = p.rec;
    const uint32_t* __restrict__ tvals = p.tvals;
    const float L = 2.0f * kSqrtLog2e, amin = 1.0f / 255.0f, t_min = p.t_min;
    const uint64_t pix = (uint64_t)py * p.W + px;  // image-row index (state buffer)
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    float T = 1.0f;   // FP32: transmittance
    float ca = 0.0f;  // FP16_TARGET: dst.a
    if (p.mode == kCompSecond && inside) {
        const float4 st = p.state[pix];
        cr = st.x;
        cg = st.y;
        cb = st.z;
        if (FP16_TARGET) ca = st.w; else T = st.w;
    }
    bool live = inside && (FP16_TARGET ? ca < 1.0f : T >= t_min);
    bool wave_live = __any(live);

    const uint32_t n = range.y - range.x;
    const uint32_t nb = (n + 255) / 256;
    float4 ga, gb, gc;
    auto gather = [&](uint32_t batch) {
        const uint32_t e = range.x + batch * 256 + tid;
        if (e < range.y) {
            const float4* r = rec + 4 * (uint64_t)tvals[e];
            ga = r[0];
            gb = r[1];
            gc = r[2];
        }
    };
    auto park = [&](int buf) {
        sA[buf][tid] = ga;
        sB[buf][tid] = gb;
        sC[buf][tid] = make_float2(gc.x, gc.y);
        sD[buf][tid] = make_uint2(__float_as_uint(gc.z), __float_as_uint(gc.w));
    };
    if (nb > 0) {
        gather(0);
        park(0);
    }
    __syncthreads();
    for (uint32_t b = 0; b < nb; ++b) {
        const int cur = b & 1;
        if (b + 1 < nb) gather(b + 1);  // in flight while this batch is blended
        if (wave_live) {
            const int cnt = (int)min(256u, n - b * 256);
            for (int k = 0; k < cnt; ++k) {
                const uint2 bb = sD[cur][k];
                if ((int)(bb.x & 0xffffu) > bx0 + 7 || (int)(bb.x >> 16) < bx0 ||
                    (int)(bb.y & 0xffffu) > by0 + 7 || (int)(bb.y >> 16) < by0)
                    continue;  // the splat misses this quarter (wave-uniform)
                const float4 A = sA[cur][k];
                const float4 B = sB[cur][k];
                const float dx = fx - A.x, dy = fy - A.y;
                const float u = dx * A.z + dy * A.w;
                const float v = dx * B.x + dy * B.y;
                const float q = u * u + v * v;
                const float alpha = __builtin_amdgcn_exp2f(B.z - q);
                const bool hit = live && fmaxf(fabsf(u), fabsf(v)) <= L && alpha >= amin;
                const float2 C = sC[cur][k];
                if (FP16_TARGET) {
                    if (hit) {
                        const float om = 1.0f - ca;
                        cr = (float)(_Float16)((B.w * alpha) * om + cr);
                        cg = (float)(_Float16)((C.x * alpha) * om + cg);
                        cb = (float)(_Float16)((C.y * alpha) * om + cb);
                        ca = (float)(_Float16)(alpha * om + ca);
                        live = ca < 1.0f;  // dst.a == 1: later blends add exactly zero
                    }
                } else {
                    const float s = hit ? alpha * T : 0.0f;
                    cr = B.w * s + cr;
                    cg = C.x * s + cg;
                    cb = C.y * s + cb;
                    T = T - s;
                    live = live && T >= t_min;
                }
                if (!__any(live)) {
                    wave_live = false;
                    break;
                }
            }
        }
        if (b + 1 < nb) park(cur ^ 1);
        if (__syncthreads_count(wave_live) == 0) break;
    }
    if (p.mode == kCompFirst) {
        const bool tile_done = __syncthreads_count(live) == 0;
        if (!tile_done) {  // park the pixels for chunk 1
            if (inside) p.state[pix] = make_float4(cr, cg, cb, FP16_TARGET ? ca : T);
            if (tid == 0) {
                p.done[tile] = 0;
                atomicAdd(&p.ctl->not_done, 1u);
            }
            return;
        }
        if (tid == 0) p.done[tile] = 1;
    }
    if (inside) {
        if (!FP16_TARGET) ca = 1.0f - T;
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
void launch_project(const ProjParams& p, hipStream_t s) {
    const unsigned grid = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>(kMaxGrid, (p.n + kProjThreads - 1) / kProjThreads));
    hipLaunchKernelGGL(k_project, dim3(grid), dim3(kProjThreads), 0, s, p);
}
void launch_sort_pass(const SortPass& p, hipStream_t s) {
    if (!p.parts_max) return;
    const unsigned grid = std::min<uint32_t>(p.parts_max, kMaxGrid);
    hipLaunchKernelGGL(k_radix_upsweep, dim3(grid), dim3(kSortThreads), 0, s, p);
    hipLaunchKernelGGL(k_radix_scan, dim3(256), dim3(256), 0, s, p);
    hipLaunchKernelGGL(k_radix_downsweep, dim3(grid), dim3(kSortThreads), 0, s, p);
}
void launch_bin(const BinParams& p, hipStream_t s) {
    const unsigned grid = std::max<uint32_t>(1, std::min<uint32_t>(bin_parts(p.n_max), kMaxGrid));
    hipLaunchKernelGGL(k_bin_count, dim3(grid), dim3(kBinThreads), 0, s, p);
    hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, s, p);
    hipLaunchKernelGGL(k_bin_emit, dim3(grid), dim3(kBinThreads), 0, s, p);
}
void launch_ranges(const uint32_t* tkeys, const uint32_t* k_dev, uint32_t k_max, uint2* ranges,
                   hipStream_t s) {
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(8192, (k_max + 255) / 256));
    hipLaunchKernelGGL(k_ranges, dim3(grid), dim3(256), 0, s, tkeys, k_dev, ranges);
}
void launch_composite(const CompositeParams& p, int accum_fp16, hipStream_t s) {
    if (p.n_tiles <= 0) return;
    if (accum_fp16)
        hipLaunchKernelGGL(k_composite<true>, dim3(p.n_tiles), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL(k_composite<false>, dim3(p.n_tiles), dim3(256), 0, s, p);
}

}  // namespace gs
