// gs_oracle.cpp — CPU restatement of the reference's Gaussian-splat forward path.
//
// TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP renderer in
// gaussian-splatting-web_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it; the product path never links or calls it.
//
// Parity status: the WGSL hot path of the reference cannot execute in this container
// (no WebGPU runtime).  This restatement follows the WGSL line by line (cited below) and is
// pinned by (a) the reference's own wgpu-matrix / packing code run under node 12
// (tests/golden/gen_ref_fixtures.py), (b) the depth-key known-answer table of SURVEY §8a/a4,
// (c) std::stable_sort as the exact oracle of webgpu-radix-sort (stable ascending LSD).
// Golden images are NOT produced by the reference itself ("image parity unpinned by a
// reference run").
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fopenmp).  Contraction is off so every
// float op below rounds exactly as written (WGSL evaluation order, left to right).
//
// Reference files (paths relative to /root/reference):
//   depth key ........ src/shaders.ts:36-40, :57-68
//   projection ....... src/simple_render.ts:97-117, :118-125, :205-216, :217-332
//   SH colour ........ src/simple_render.ts:5-67
//   fragment + blend . src/simple_render.ts:169-200, :455-471 (rgba16float target :499-505)
//   draw order ....... src/renderer.ts:301-330 (init-sort grid :306), RS stable radix sort
//   record layout .... src/ply.ts:249-257, src/packing.ts:146-291
//   uniform layout ... src/renderer.ts:24-33
//   present .......... src/post_process_render.ts:62-77

#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <numeric>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <parallel/algorithm>
#endif

namespace {

// ---------------------------------------------------------------- WGSL-like mat types
// WGSL matrices are column-major: c[col][row].  Constructors from scalars fill column 0 first.
struct v2 { float x, y; };
struct v3 { float x, y, z; };
struct v4 { float x, y, z, w; };
struct m3 { float c[3][3]; };
struct m4 { float c[4][4]; };

m3 m3_from9(float a0, float a1, float a2, float a3, float a4, float a5, float a6, float a7,
            float a8) {
    m3 m;
    m.c[0][0] = a0; m.c[0][1] = a1; m.c[0][2] = a2;
    m.c[1][0] = a3; m.c[1][1] = a4; m.c[1][2] = a5;
    m.c[2][0] = a6; m.c[2][1] = a7; m.c[2][2] = a8;
    return m;
}
m3 m3_cols(v3 a, v3 b, v3 c) { return m3_from9(a.x, a.y, a.z, b.x, b.y, b.z, c.x, c.y, c.z); }
m3 mul(const m3& A, const m3& B) {  // (A*B)[j][i] = sum_k A[k][i] * B[j][k]
    m3 R;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i)
            R.c[j][i] = A.c[0][i] * B.c[j][0] + A.c[1][i] * B.c[j][1] + A.c[2][i] * B.c[j][2];
    return R;
}
m3 transpose(const m3& A) {
    m3 R;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) R.c[j][i] = A.c[i][j];
    return R;
}
m4 m4_load(const float* f) {  // from a column-major Float32Array(16) (wgpu-matrix storage)
    m4 m;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) m.c[j][i] = f[4 * j + i];
    return m;
}
m4 mul(const m4& A, const m4& B) {
    m4 R;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i)
            R.c[j][i] = A.c[0][i] * B.c[j][0] + A.c[1][i] * B.c[j][1] + A.c[2][i] * B.c[j][2] +
                        A.c[3][i] * B.c[j][3];
    return R;
}
v4 mul(const m4& A, v4 v) {
    v4 r;
    r.x = A.c[0][0] * v.x + A.c[1][0] * v.y + A.c[2][0] * v.z + A.c[3][0] * v.w;
    r.y = A.c[0][1] * v.x + A.c[1][1] * v.y + A.c[2][1] * v.z + A.c[3][1] * v.w;
    r.z = A.c[0][2] * v.x + A.c[1][2] * v.y + A.c[2][2] * v.z + A.c[3][2] * v.w;
    r.w = A.c[0][3] * v.x + A.c[1][3] * v.y + A.c[2][3] * v.z + A.c[3][3] * v.w;
    return r;
}
float saturate(float x) { return std::min(std::max(x, 0.0f), 1.0f); }
v3 normalize3(v3 v) {
    float l = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    return {v.x / l, v.y / l, v.z / l};
}

// ---------------------------------------------------------------- fp16 round trip
// Emulates storing an f32 into an rgba16float render target (round to nearest even,
// overflow -> inf) and reading it back.
float to_half_and_back(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const bool neg = (x >> 31) != 0;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return f;                        // inf / NaN pass through
    if (ax >= 0x477ff000u) return neg ? -INFINITY : INFINITY;  // >= 65520 rounds to inf
    if (ax <= 0x33000000u) return neg ? -0.0f : 0.0f;          // <= 2^-25 rounds to zero
    const int e = (int)(ax >> 23) - 127;
    const int ulp_exp = e >= -14 ? e - 10 : -24;  // half normal / subnormal spacing
    const float r = std::nearbyint(std::ldexp(std::fabs(f), -ulp_exp));  // exact scale, RNE
    const float res = std::ldexp(r, ulp_exp);
    return neg ? -res : res;
}

}  // namespace

extern "C" {

// 160-B uniform block, src/renderer.ts:24-33 (offsets pinned by tests/golden/layout.json).
struct or_uniforms {
    float view[16];   // @0   column-major
    float proj[16];   // @64
    float campos[3];  // @128
    float tan_half_fov_x, tan_half_fov_y, focal_x, focal_y;  // @140..152 (unused by shaders)
    float scale_modifier;                                     // @156
};

// Per-Gaussian projected result (the oracle's view of vs_points + the key pass).
struct or_splat {
    uint32_t key;       // float_to_sortable_uint((V*[p,1]).z)
    int32_t visible;    // 1 if the splat can produce any fragment
    float clip[4];      // (P*V)*[p,1]
    float c[2];         // centre in framebuffer pixels (row 0 = top)
    float e1[2], e2[2]; // quad half-axes in framebuffer pixels (corner = c + u e1 + v e2, |u|,|v|<=2)
    float col[3];       // SH colour (+0.5, max 0)
    float op;           // sigmoid(opacity_logit)
    int32_t rect[4];    // inclusive pixel bbox [x0,y0,x1,y1] of candidate pixels (clipped)
    int32_t ntiles;     // 16x16 tiles overlapped by the survey's K-rectangle
    float view_z;       // (V*[p,1]).z
};

struct or_stats {
    uint64_t n, n_vis, k_tiles, blends;
};

// src/shaders.ts:36-40
uint32_t or_sortable_key(float f) {
    uint32_t fu;
    std::memcpy(&fu, &f, 4);
    int32_t fi = (int32_t)fu;
    uint32_t mask = (uint32_t)(-(fi >> 31)) | 0x80000000u;
    return fu ^ mask;
}

// Record layout (src/ply.ts:249-257 through src/packing.ts rules): position @0, scale @16,
// rot @32, opacityLogit @48, sh[k] @64 + 16k (vec3, 16-B stride).  Size 64 + 16*n_sh.
int or_record_bytes(int n_sh_coeffs) { return 64 + 16 * n_sh_coeffs; }

// Pixels whose centre (x+0.5, y+0.5) lies in [cx-hx, cx+hx] x [cy-hy, cy+hy], clipped to the
// image; false if none.  f32 arithmetic.
static bool pixel_rect(float cx, float cy, float hx, float hy, int W, int H, int out[4]) {
    const float xl = std::fmax(std::ceil(cx - hx - 0.5f), 0.0f);
    const float xh = std::fmin(std::floor(cx + hx - 0.5f), (float)(W - 1));
    const float yl = std::fmax(std::ceil(cy - hy - 0.5f), 0.0f);
    const float yh = std::fmin(std::floor(cy + hy - 0.5f), (float)(H - 1));
    if (!(xl <= xh) || !(yl <= yh)) return false;
    out[0] = (int)xl; out[1] = (int)yl; out[2] = (int)xh; out[3] = (int)yh;
    return true;
}

static void project_one(const float* rec, int n_sh, const or_uniforms& u, int W, int H,
                        or_splat& s) {
    std::memset(&s, 0, sizeof(s));
    const v3 pos = {rec[0], rec[1], rec[2]};
    const v3 scale = {rec[4], rec[5], rec[6]};
    const v4 rot = {rec[8], rec[9], rec[10], rec[11]};
    const float opacity_logit = rec[12];
    const m4 V = m4_load(u.view);
    const m4 P = m4_load(u.proj);

    // --- depth key, src/shaders.ts:67-68
    const v4 vp4 = mul(V, v4{pos.x, pos.y, pos.z, 1.0f});
    s.view_z = vp4.z;
    s.key = or_sortable_key(vp4.z);

    // --- vs_points, src/simple_render.ts:228 : (P*V)*[p,1], matrix product first
    const m4 PV = mul(P, V);
    const v4 clip = mul(PV, v4{pos.x, pos.y, pos.z, 1.0f});
    s.clip[0] = clip.x; s.clip[1] = clip.y; s.clip[2] = clip.z; s.clip[3] = clip.w;
    if (!(clip.w > 0.0f)) return;                       // :230-233 (NaN position)
    if (!(clip.z >= 0.0f && clip.z <= clip.w)) return;  // rasteriser near/far clip (all corners share z,w)

    // :97-117 CalcMatrixFromRotationScale
    const float mod = u.scale_modifier;
    const m3 ms = m3_from9(scale.x * mod, 0.0f, 0.0f, 0.0f, scale.y * mod, 0.0f, 0.0f, 0.0f,
                           scale.z * mod);
    const float x = rot.x, y = rot.y, z = rot.z, w = rot.w;
    const m3 mr = m3_from9(1.0f - 2.0f * (y * y + z * z), 2.0f * (x * y - w * z),
                           2.0f * (x * z + w * y), 2.0f * (x * y + w * z),
                           1.0f - 2.0f * (x * x + z * z), 2.0f * (y * z - w * x),
                           2.0f * (x * z - w * y), 2.0f * (y * z + w * x),
                           1.0f - 2.0f * (x * x + y * y));
    const m3 M = mul(mr, ms);
    const m3 sig = mul(M, transpose(M));  // :247
    v3 cov3d0 = {sig.c[0][0], sig.c[0][1], sig.c[0][2]};
    v3 cov3d1 = {sig.c[1][1], sig.c[1][2], sig.c[2][2]};
    const float splatScale2 = 1.0f;  // :252-255
    cov3d0 = {cov3d0.x * splatScale2, cov3d0.y * splatScale2, cov3d0.z * splatScale2};
    cov3d1 = {cov3d1.x * splatScale2, cov3d1.y * splatScale2, cov3d1.z * splatScale2};

    // :259-271 (the limx/limy clamp only reaches J's unused third row)
    v3 viewPos = {vp4.x, vp4.y, vp4.z};
    const float aspect = P.c[0][0] / P.c[1][1];
    const float tanFovX = 1.0f / P.c[0][0];
    const float tanFovY = 1.0f / (P.c[1][1] * aspect);
    const float limx = 1.3f * tanFovX, limy = 1.3f * tanFovY;
    const float txtz = viewPos.x / viewPos.z, tytz = viewPos.y / viewPos.z;
    viewPos.x = std::min(limx, std::max(-limx, txtz)) * viewPos.z;
    viewPos.y = std::min(limy, std::max(-limy, tytz)) * viewPos.z;

    // :273-298
    const float focal = (float)W * P.c[0][0] / 2.0f;
    const m3 J = m3_from9(focal / viewPos.z, 0.0f, -(focal * viewPos.x) / (viewPos.z * viewPos.z),
                          0.0f, focal / viewPos.z, -(focal * viewPos.y) / (viewPos.z * viewPos.z),
                          0.0f, 0.0f, 0.0f);
    const m3 W3 = m3_cols(v3{V.c[0][0], V.c[0][1], V.c[0][2]}, v3{V.c[1][0], V.c[1][1], V.c[1][2]},
                          v3{V.c[2][0], V.c[2][1], V.c[2][2]});
    const m3 T = mul(J, W3);
    const m3 Vrk = m3_from9(cov3d0.x, cov3d0.y, cov3d0.z, cov3d0.y, cov3d1.x, cov3d1.y, cov3d0.z,
                            cov3d1.y, cov3d1.z);
    m3 cov2d_mat = mul(T, mul(Vrk, transpose(T)));
    cov2d_mat.c[0][0] += 0.3f;
    cov2d_mat.c[1][1] += 0.3f;
    const float d1 = cov2d_mat.c[0][0], off = -cov2d_mat.c[0][1], d2 = cov2d_mat.c[1][1];

    // :305-314 eigen basis
    const float mid = 0.5f * (d1 + d2);
    const float ra = (d1 - d2) / 2.0f;
    const float radius = std::sqrt(ra * ra + off * off);
    const float lambda1 = mid + radius;
    const float lambda2 = std::max(mid - radius, 0.1f);
    // :205-216 safe_normalize_v2
    float nx = off, ny = lambda1 - d1;
    if (nx != 0.0f) nx = nx + 1e-10f;
    if (ny != 0.0f) ny = ny + 1e-10f;
    const float nl = std::sqrt(nx * nx + ny * ny);
    v2 dv = {nx / nl, ny / nl};
    dv.y = -dv.y;
    const float maxSize = 4096.0f;
    const float s1 = std::min(std::sqrt(2.0f * lambda1), maxSize);
    const float s2 = std::min(std::sqrt(2.0f * lambda2), maxSize);
    const v2 v1 = {s1 * dv.x, s1 * dv.y};
    const v2 v2_ = {s2 * dv.y, s2 * -dv.x};

    // Corner k: ndc = clip.xy/clip.w + q.x*v1*2/(W,H) + q.y*v2*2/(W,H)  (:316-320).
    // Framebuffer pixel (row 0 = top): x=(ndc.x+1)W/2, y=(1-ndc.y)H/2  =>
    //   corner_px = c + q.x*e1 + q.y*e2 with e = (v.x, -v.y), |q.x|,|q.y| <= 2.
    const float ndcx = clip.x / clip.w, ndcy = clip.y / clip.w;
    s.c[0] = (ndcx + 1.0f) * (float)W / 2.0f;
    s.c[1] = (1.0f - ndcy) * (float)H / 2.0f;
    s.e1[0] = v1.x; s.e1[1] = -v1.y;
    s.e2[0] = v2_.x; s.e2[1] = -v2_.y;
    for (float f : {s.c[0], s.c[1], s.e1[0], s.e1[1], s.e2[0], s.e2[1]})
        if (!std::isfinite(f)) return;  // NaN basis (off=0 and lambda1=d1) -> primitive dropped

    // :321 colour, :5-67
    {
        const v3 cp = {u.campos[0], u.campos[1], u.campos[2]};
        const v3 dir = normalize3(v3{pos.x - cp.x, pos.y - cp.y, pos.z - cp.z});
        const float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
        const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                -1.0925484305920792f, 0.5462742152960396f};
        const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                -0.5900435899266435f};
        float sh[16][3];
        for (int k = 0; k < 16; ++k)
            for (int c = 0; c < 3; ++c) sh[k][c] = k < n_sh ? rec[16 + 4 * k + c] : 0.0f;
        const float X = dir.x, Y = dir.y, Z = dir.z;
        const float xx = X * X, yy = Y * Y, zz = Z * Z, xy = X * Y, xz = X * Z, yz = Y * Z;
        for (int c = 0; c < 3; ++c) {
            float r = SH_C0 * sh[0][c];
            r = r + SH_C1 * (-Y * sh[1][c] + Z * sh[2][c] - X * sh[3][c]);
            r = r + SH_C2[0] * xy * sh[4][c] + SH_C2[1] * yz * sh[5][c] +
                SH_C2[2] * (2.0f * zz - xx - yy) * sh[6][c] + SH_C2[3] * xz * sh[7][c] +
                SH_C2[4] * (xx - yy) * sh[8][c];
            r = r + SH_C3[0] * Y * (3.0f * xx - yy) * sh[9][c] + SH_C3[1] * xy * Z * sh[10][c] +
                SH_C3[2] * Y * (4.0f * zz - xx - yy) * sh[11][c] +
                SH_C3[3] * Z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12][c] +
                SH_C3[4] * X * (4.0f * zz - xx - yy) * sh[13][c] +
                SH_C3[5] * Z * (xx - yy) * sh[14][c] + SH_C3[6] * X * (xx - 3.0f * yy) * sh[15][c];
            r = r + 0.5f;
            s.col[c] = std::max(r, 0.0f);
        }
    }
    // :118-125 sigmoid, :328
    if (opacity_logit >= 0.0f) {
        s.op = 1.0f / (1.0f + std::exp(-opacity_logit));
    } else {
        const float zz = std::exp(opacity_logit);
        s.op = zz / (1.0f + zz);
    }
    if (!(s.op >= 1.0f / 255.0f)) return;  // alpha <= op everywhere -> every fragment discarded

    // Visibility (SURVEY §8d "bbox ∩ screen"): the bounding box of the quad |u|,|v| <= 2 contains
    // at least one pixel centre of the image.  All in f32, the order the kernel uses.
    const float qx = 2.0f * (std::fabs(s.e1[0]) + std::fabs(s.e2[0]));
    const float qy = 2.0f * (std::fabs(s.e1[1]) + std::fabs(s.e2[1]));
    int qb[4];
    if (!pixel_rect(s.c[0], s.c[1], qx, qy, W, H, qb)) return;
    s.visible = 1;
    // K rectangle: the quad's box intersected with the box of the alpha >= 1/255
    // disc u^2+v^2 <= ln(255 op); it may be empty (a visible splat that binds no tile).
    const float R = std::sqrt(std::fmax(std::log(255.0f * s.op), 0.0f));
    const float hx = std::min(qx, R * std::sqrt(s.e1[0] * s.e1[0] + s.e2[0] * s.e2[0]));
    const float hy = std::min(qy, R * std::sqrt(s.e1[1] * s.e1[1] + s.e2[1] * s.e2[1]));
    int kb[4];
    if (pixel_rect(s.c[0], s.c[1], hx, hy, W, H, kb))
        s.ntiles = (kb[2] / 16 - kb[0] / 16 + 1) * (kb[3] / 16 - kb[1] / 16 + 1);
    // pixels the composite tests exactly: the quad box widened by one pixel
    s.rect[0] = std::max(qb[0] - 1, 0); s.rect[1] = std::max(qb[1] - 1, 0);
    s.rect[2] = std::min(qb[2] + 1, W - 1); s.rect[3] = std::min(qb[3] + 1, H - 1);
}

int or_project(const void* aos, uint64_t n, int n_sh, const void* uni160, int W, int H,
               or_splat* out) {
    if (!aos || !uni160 || !out || W <= 0 || H <= 0) return -1;
    if (n_sh != 1 && n_sh != 4 && n_sh != 9 && n_sh != 16) return -2;
    or_uniforms u;
    std::memcpy(&u, uni160, sizeof(u));
    const int stride = or_record_bytes(n_sh) / 4;
    const float* base = (const float*)aos;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) project_one(base + (size_t)i * stride, n_sh, u, W, H, out[i]);
    return 0;
}

// Oracle of webgpu-radix-sort (RS:541-654): stable ascending sort of u32 keys carrying u32
// values.
// A stable sort by key is a sort by (key, position): positions are distinct, so sorting the
// packed 64-bit (key << 32 | position) with any (parallel) sort gives exactly the stable order.
void or_stable_sort_pairs(uint32_t* keys, uint32_t* vals, uint64_t n) {
    if (n > 0xFFFFFFFFull) return;
    std::vector<uint64_t> kp(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) kp[i] = ((uint64_t)keys[i] << 32) | (uint64_t)i;
#ifdef _OPENMP
    __gnu_parallel::sort(kp.begin(), kp.end());
#else
    std::sort(kp.begin(), kp.end());
#endif
    std::vector<uint32_t> v2(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        keys[i] = (uint32_t)(kp[i] >> 32);
        v2[i] = vals[kp[i] & 0xFFFFFFFFull];
    }
    std::memcpy(vals, v2.data(), n * 4);
}

// Init-sort grid of the reference (src/renderer.ts:306): dispatchWorkgroups(max(N/8,8)) with
// WebIDL truncation, workgroup size 8 -> only the first trunc(max(N/8,8))*8 slots are keyed.
uint64_t or_keyed_slots(uint64_t n) {
    const double g = std::max((double)n / 8.0, 8.0);
    const uint64_t keyed = (uint64_t)std::trunc(g) * 8;
    return std::min(keyed, n);
}

// Draw order.  quirk=0: every Gaussian keyed (stated harness fix); quirk=1: reference
// behaviour, slots >= or_keyed_slots(n) keep the (key,value) the previous frame's in-place
// sort left there (zero on the first frame); state_* (n entries each) carry that state.
int or_draw_order(const or_splat* sp, uint64_t n, int quirk, uint32_t* state_keys,
                  uint32_t* state_vals, uint32_t* order_out) {
    std::vector<uint32_t> k(n), v(n);
    const uint64_t nk = quirk ? or_keyed_slots(n) : n;
    for (uint64_t s = 0; s < n; ++s) {
        if (s < nk) { k[s] = sp[s].key; v[s] = (uint32_t)s; }
        else { k[s] = state_keys[s]; v[s] = state_vals[s]; }
    }
    or_stable_sort_pairs(k.data(), v.data(), n);
    if (quirk) {
        std::memcpy(state_keys, k.data(), n * 4);
        std::memcpy(state_vals, v.data(), n * 4);
    }
    std::memcpy(order_out, v.data(), n * 4);
    return 0;
}

static int or_num_threads_internal() {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

// Fragment + blend (src/simple_render.ts:169-200, :455-471) over the draw order.
// accum_mode 0: fp32 dst; 1: dst rounded to fp16 after every blend (rgba16float target).
// t_min: a pixel stops accepting splats once (1 - dst.a) < t_min (0 = never).
// out: W*H*4 floats, premultiplied RGBA, row 0 = top (SimpleRender.framebuffer contents).
int or_composite(const or_splat* sp, const uint32_t* order, uint64_t n_order, int W, int H,
                 int accum_mode, float t_min, float* out, uint64_t* blends_out) {
    std::memset(out, 0, sizeof(float) * 4 * (size_t)W * H);
    const int TR = (H + 15) / 16;
    // per 16-row band: the draw positions whose pixel rect reaches it, in draw order (a band's
    // pixels see exactly the splats in this list, in the same order as a walk over all of them)
    std::vector<std::vector<uint32_t>> band_list(TR);
    {
        const int nth = or_num_threads_internal();
        std::vector<std::vector<std::vector<uint32_t>>> part(nth, std::vector<std::vector<uint32_t>>(TR));
        const uint64_t per = (n_order + nth - 1) / std::max(nth, 1);
#pragma omp parallel for schedule(static, 1)
        for (int t = 0; t < nth; ++t)
            for (uint64_t o = t * per; o < std::min<uint64_t>(n_order, (t + 1) * per); ++o) {
                const or_splat& s = sp[order[o]];
                if (!s.visible) continue;
                for (int b = s.rect[1] / 16; b <= std::min(s.rect[3] / 16, TR - 1); ++b) part[t][b].push_back((uint32_t)o);
            }
#pragma omp parallel for schedule(dynamic, 1)
        for (int b = 0; b < TR; ++b)
            for (int t = 0; t < nth; ++t) band_list[b].insert(band_list[b].end(), part[t][b].begin(), part[t][b].end());
    }
    uint64_t blends = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : blends)
    for (int band = 0; band < TR; ++band) {
        const int by0 = band * 16, by1 = std::min(by0 + 15, H - 1);
        for (const uint32_t o : band_list[band]) {
            const or_splat& s = sp[order[o]];
            const int y0 = std::max(s.rect[1], by0), y1 = std::min(s.rect[3], by1);
            if (y0 > y1) continue;
            const float e1n = s.e1[0] * s.e1[0] + s.e1[1] * s.e1[1];
            const float e2n = s.e2[0] * s.e2[0] + s.e2[1] * s.e2[1];
            for (int py = y0; py <= y1; ++py) {
                for (int px = s.rect[0]; px <= s.rect[2]; ++px) {
                    const float dx = ((float)px + 0.5f) - s.c[0];
                    const float dy = ((float)py + 0.5f) - s.c[1];
                    const float uu = (dx * s.e1[0] + dy * s.e1[1]) / e1n;
                    const float vv = (dx * s.e2[0] + dy * s.e2[1]) / e2n;
                    if (!(std::fabs(uu) <= 2.0f && std::fabs(vv) <= 2.0f)) continue;
                    // fs_main: alpha = saturate(exp(-dot(uv,uv)) * opacity); discard < 1/255
                    const float power = -(uu * uu + vv * vv);
                    const float alpha = saturate(std::exp(power) * s.op);
                    if (alpha < 1.0f / 255.0f) continue;
                    float* d = out + 4 * ((size_t)py * W + px);
                    const float oma = 1.0f - d[3];
                    if (oma < t_min) continue;
                    // blend: src*(1-dst.a) + dst, src = (col*alpha, alpha)
                    float r = (s.col[0] * alpha) * oma + d[0];
                    float g = (s.col[1] * alpha) * oma + d[1];
                    float b = (s.col[2] * alpha) * oma + d[2];
                    float a = alpha * oma + d[3];
                    if (accum_mode == 1) {
                        r = to_half_and_back(r); g = to_half_and_back(g);
                        b = to_half_and_back(b); a = to_half_and_back(a);
                    }
                    d[0] = r; d[1] = g; d[2] = b; d[3] = a;
                    ++blends;
                }
            }
        }
    }
    if (blends_out) *blends_out = blends;
    return 0;
}

// Whole frame: project -> key -> stable sort -> composite.  Statistics per SURVEY §8d.
int or_render(const void* aos, uint64_t n, int n_sh, const void* uni160, int W, int H,
              int accum_mode, float t_min, int quirk, uint32_t* state_keys, uint32_t* state_vals,
              float* out, or_stats* st) {
    std::vector<or_splat> sp(n);
    int rc = or_project(aos, n, n_sh, uni160, W, H, sp.data());
    if (rc) return rc;
    std::vector<uint32_t> order(n);
    std::vector<uint32_t> sk, sv;
    if (quirk && (!state_keys || !state_vals)) return -3;
    or_draw_order(sp.data(), n, quirk, state_keys, state_vals, order.data());
    uint64_t blends = 0;
    or_composite(sp.data(), order.data(), n, W, H, accum_mode, t_min, out, &blends);
    if (st) {
        st->n = n;
        st->n_vis = 0;
        st->k_tiles = 0;
        for (uint64_t i = 0; i < n; ++i)
            if (sp[i].visible) { st->n_vis++; st->k_tiles += (uint64_t)sp[i].ntiles; }
        st->blends = blends;
    }
    return 0;
}

// PostProcessRenderer fragmentMain (src/post_process_render.ts:62-77): the fragment at pixel
// centre (x+.5, y+.5) samples uv = fragCoord / (W, H) with uv.y = 1 - uv.y, i.e. the texel centre
// of row H-1-y (a sampler at a texel centre returns the texel), so the pass is a row flip; then
// color.a = saturate(color.a * 1.5) and, below 0.99, color.a = pow(color.a, 4).  pow is WGSL's
// builtin (exp2(4 log2 a) on most backends, a few ulp): restated with powf.
int or_present(const float* in, int W, int H, float* out) {
    if (!in || !out || W <= 0 || H <= 0) return -1;
    for (int y = 0; y < H; ++y) {
        const float* src = in + 4 * (size_t)(H - 1 - y) * W;
        float* dst = out + 4 * (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            dst[4 * x + 0] = src[4 * x + 0];
            dst[4 * x + 1] = src[4 * x + 1];
            dst[4 * x + 2] = src[4 * x + 2];
            float a = src[4 * x + 3] * 1.5f;
            a = a < 0.0f ? 0.0f : (a > 1.0f ? 1.0f : a);  // saturate
            if (a < 0.99f) a = std::pow(a, 4.0f);
            dst[4 * x + 3] = a;
        }
    }
    return 0;
}

int or_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

}  // extern "C"

extern "C" {
// Diagnostics for the tile compositor: per 16x16 tile, the list length (splats whose K-rectangle
// touches the tile) and the number of list entries consumed before all of the tile's pixels stop
// accepting splats (T < t_min), plus how many (8x8 quarter, entry) pairs overlap the splat box.
int or_tile_stats(const or_splat* sp, const uint32_t* order, uint64_t n_order, int W, int H,
                  float t_min, uint32_t* out_len, uint32_t* out_used, uint64_t* out_quarter_pairs) {
    const int TX = (W + 15) / 16, TY = (H + 15) / 16;
    std::vector<std::vector<uint32_t>> lists((size_t)TX * TY);
    for (uint64_t o = 0; o < n_order; ++o) {
        const or_splat& s = sp[order[o]];
        if (!s.visible) continue;
        for (int ty = s.rect[1] / 16; ty <= s.rect[3] / 16; ++ty)
            for (int tx = s.rect[0] / 16; tx <= s.rect[2] / 16; ++tx) lists[(size_t)ty * TX + tx].push_back(order[o]);
    }
    uint64_t qp = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : qp)
    for (int t = 0; t < TX * TY; ++t) {
        const int tx = t % TX, ty = t / TX;
        float T[256];
        for (int i = 0; i < 256; ++i) {
            const int px = tx * 16 + (i & 15), py = ty * 16 + (i >> 4);
            T[i] = (px < W && py < H) ? 1.0f : 0.0f;
        }
        uint32_t used = 0;
        for (uint32_t k = 0; k < lists[t].size(); ++k) {
            bool any = false;
            for (int i = 0; i < 256; ++i) any |= T[i] >= t_min && T[i] > 0.0f;
            if (!any) break;
            used = k + 1;
            const or_splat& s = sp[lists[t][k]];
            for (int qy = 0; qy < 2; ++qy)
                for (int qx = 0; qx < 2; ++qx) {
                    const int x0 = tx * 16 + qx * 8, y0 = ty * 16 + qy * 8;
                    if (s.rect[0] <= x0 + 7 && s.rect[2] >= x0 && s.rect[1] <= y0 + 7 && s.rect[3] >= y0) ++qp;
                }
            const float e1n = s.e1[0] * s.e1[0] + s.e1[1] * s.e1[1];
            const float e2n = s.e2[0] * s.e2[0] + s.e2[1] * s.e2[1];
            for (int i = 0; i < 256; ++i) {
                if (!(T[i] >= t_min && T[i] > 0.0f)) continue;
                const int px = tx * 16 + (i & 15), py = ty * 16 + (i >> 4);
                if (px < s.rect[0] || px > s.rect[2] || py < s.rect[1] || py > s.rect[3]) continue;
                const float dx = ((float)px + 0.5f) - s.c[0], dy = ((float)py + 0.5f) - s.c[1];
                const float uu = (dx * s.e1[0] + dy * s.e1[1]) / e1n, vv = (dx * s.e2[0] + dy * s.e2[1]) / e2n;
                if (!(std::fabs(uu) <= 2.0f && std::fabs(vv) <= 2.0f)) continue;
                const float a = saturate(std::exp(-(uu * uu + vv * vv)) * s.op);
                if (a < 1.0f / 255.0f) continue;
                T[i] *= 1.0f - a;
            }
        }
        out_len[t] = (uint32_t)lists[t].size();
        out_used[t] = used;
    }
    if (out_quarter_pairs) *out_quarter_pairs = qp;
    return 0;
}
}
