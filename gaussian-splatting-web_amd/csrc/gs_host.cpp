// gs_host.cpp — host-side pieces of the C ABI that need no GPU:
//   * camera / uniform producer with wgpu-matrix 2.9.1 semantics (every store rounds to f32, the
//     arithmetic in between is JS double): lookAt, perspective, inverse(view).translation as used
//     by src/camera.ts:101-138 and packed as src/renderer.ts:24-33 / :349-384;
//   * seeded synthetic scenes, written in the reference AoS layout;
//   * the present pass (src/post_process_render.ts:54-77).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/gsplat.h"

namespace {

inline float f32(double v) { return (float)v; }

// WM normalize$2 into a Float32Array (len computed in double from the f32 inputs).
void wm_normalize(const float v[3], float out[3]) {
    const double v0 = v[0], v1 = v[1], v2 = v[2];
    const double len = std::sqrt(v0 * v0 + v1 * v1 + v2 * v2);
    if (len > 0.00001) {
        out[0] = f32(v0 / len); out[1] = f32(v1 / len); out[2] = f32(v2 / len);
    } else {
        out[0] = out[1] = out[2] = 0.0f;
    }
}

// WM cross(a, b) with a given as doubles (JS array) or f32 (Float32Array)
void wm_cross(const double a[3], const double b[3], float out[3]) {
    const double t1 = a[2] * b[0] - a[0] * b[2];
    const double t2 = a[0] * b[1] - a[1] * b[0];
    out[0] = f32(a[1] * b[2] - a[2] * b[1]);
    out[1] = f32(t1);
    out[2] = f32(t2);
}

struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
    double normal() {  // Box-Muller, cosine branch
        const double u1 = uniform(), u2 = uniform();
        return std::sqrt(-2.0 * std::log(1.0 - u1)) * std::cos(6.283185307179586 * u2);
    }
};

}  // namespace

extern "C" {

int gs_look_at(const double eye[3], const double target[3], const double up[3], float out_view[16]);
int gs_perspective(double fovy, double aspect, double zn, double zf, float out_proj[16]);

// mat4.lookAt (WM:3619)
int gs_look_at(const double eye[3], const double target[3], const double up[3], float dst[16]) {
    if (!eye || !target || !up || !dst) return GS_ERR_INVALID;
    float z[3], x[3], y[3];
    const float zs[3] = {f32(eye[0] - target[0]), f32(eye[1] - target[1]), f32(eye[2] - target[2])};
    wm_normalize(zs, z);
    const double zd[3] = {z[0], z[1], z[2]};
    float xs[3];
    wm_cross(up, zd, xs);
    wm_normalize(xs, x);
    const double xd[3] = {x[0], x[1], x[2]};
    float ys[3];
    wm_cross(zd, xd, ys);
    wm_normalize(ys, y);
    dst[0] = x[0]; dst[1] = y[0]; dst[2] = z[0]; dst[3] = 0;
    dst[4] = x[1]; dst[5] = y[1]; dst[6] = z[1]; dst[7] = 0;
    dst[8] = x[2]; dst[9] = y[2]; dst[10] = z[2]; dst[11] = 0;
    dst[12] = f32(-((double)x[0] * eye[0] + (double)x[1] * eye[1] + (double)x[2] * eye[2]));
    dst[13] = f32(-((double)y[0] * eye[0] + (double)y[1] * eye[1] + (double)y[2] * eye[2]));
    dst[14] = f32(-((double)z[0] * eye[0] + (double)z[1] * eye[1] + (double)z[2] * eye[2]));
    dst[15] = 1;
    return GS_OK;
}

// mat4.perspective (WM:3325)
int gs_perspective(double fovy, double aspect, double zn, double zf, float dst[16]) {
    if (!dst || !(aspect != 0.0)) return GS_ERR_INVALID;
    const double f = std::tan(M_PI * 0.5 - 0.5 * fovy);
    std::memset(dst, 0, 64);
    dst[0] = f32(f / aspect);
    dst[5] = f32(f);
    dst[11] = -1;
    if (std::isfinite(zf)) {
        const double rangeInv = 1.0 / (zn - zf);
        dst[10] = f32(zf * rangeInv);
        dst[14] = f32(zf * zn * rangeInv);
    } else {
        dst[10] = -1;
        dst[14] = f32(-zn);
    }
    return GS_OK;
}

// Camera.getPosition (src/camera.ts:135-138) = translation of WM mat4.inverse (WM:3004).
int gs_camera_position(const float view[16], float out[3]) {
    if (!view || !out) return GS_ERR_INVALID;
    const double m00 = view[0], m01 = view[1], m02 = view[2], m03 = view[3];
    const double m10 = view[4], m11 = view[5], m12 = view[6], m13 = view[7];
    const double m20 = view[8], m21 = view[9], m22 = view[10], m23 = view[11];
    const double m30 = view[12], m31 = view[13], m32 = view[14], m33 = view[15];
    const double tmp0 = m22 * m33, tmp1 = m32 * m23, tmp2 = m12 * m33, tmp3 = m32 * m13;
    const double tmp4 = m12 * m23, tmp5 = m22 * m13, tmp6 = m02 * m33, tmp7 = m32 * m03;
    const double tmp8 = m02 * m23, tmp9 = m22 * m03, tmp10 = m02 * m13, tmp11 = m12 * m03;
    const double tmp12 = m20 * m31, tmp13 = m30 * m21, tmp14 = m10 * m31, tmp15 = m30 * m11;
    const double tmp16 = m10 * m21, tmp17 = m20 * m11, tmp18 = m00 * m31, tmp19 = m30 * m01;
    const double tmp20 = m00 * m21, tmp21 = m20 * m01, tmp22 = m00 * m11, tmp23 = m10 * m01;
    const double t0 = (tmp0 * m11 + tmp3 * m21 + tmp4 * m31) - (tmp1 * m11 + tmp2 * m21 + tmp5 * m31);
    const double t1 = (tmp1 * m01 + tmp6 * m21 + tmp9 * m31) - (tmp0 * m01 + tmp7 * m21 + tmp8 * m31);
    const double t2 = (tmp2 * m01 + tmp7 * m11 + tmp10 * m31) - (tmp3 * m01 + tmp6 * m11 + tmp11 * m31);
    const double t3 = (tmp5 * m01 + tmp8 * m11 + tmp11 * m21) - (tmp4 * m01 + tmp9 * m11 + tmp10 * m21);
    const double d = 1.0 / (m00 * t0 + m10 * t1 + m20 * t2 + m30 * t3);
    out[0] = f32(d * ((tmp14 * m22 + tmp17 * m32 + tmp13 * m12) - (tmp16 * m32 + tmp12 * m12 + tmp15 * m22)));
    out[1] = f32(d * ((tmp20 * m32 + tmp12 * m02 + tmp19 * m22) - (tmp18 * m22 + tmp21 * m32 + tmp13 * m02)));
    out[2] = f32(d * ((tmp18 * m12 + tmp23 * m32 + tmp15 * m02) - (tmp22 * m32 + tmp14 * m02 + tmp19 * m12)));
    return GS_OK;
}

// uniformLayout.pack (src/renderer.ts:24-33): 160 bytes.
int gs_pack_uniforms(const float view[16], const float proj[16], const float cam_pos[3], float thx,
                     float thy, float fx, float fy, float scale_modifier, void* out160) {
    if (!view || !proj || !cam_pos || !out160) return GS_ERR_INVALID;
    float u[40];
    std::memcpy(u, view, 64);
    std::memcpy(u + 16, proj, 64);
    std::memcpy(u + 32, cam_pos, 12);
    u[35] = thx;
    u[36] = thy;
    u[37] = fx;
    u[38] = fy;
    u[39] = scale_modifier;
    std::memcpy(out160, u, 160);
    return GS_OK;
}

// PostProcessRenderer fragmentMain (src/post_process_render.ts:62-77).
int gs_present(const float* in, int W, int H, float* out) {
    if (!in || !out || W <= 0 || H <= 0 || in == out) return GS_ERR_INVALID;
    for (int y = 0; y < H; ++y) {
        const float* src = in + 4 * (size_t)(H - 1 - y) * W;
        float* dst = out + 4 * (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            dst[4 * x + 0] = src[4 * x + 0];
            dst[4 * x + 1] = src[4 * x + 1];
            dst[4 * x + 2] = src[4 * x + 2];
            float a = std::fmin(std::fmax(src[4 * x + 3] * 1.5f, 0.0f), 1.0f);
            if (a < 0.99f) a = std::pow(a, 4.0f);
            dst[4 * x + 3] = a;
        }
    }
    return GS_OK;
}

// Synthetic scene, SURVEY §8d / BASELINE.md §4: camera lookAt([0,0,0],[0,0,-1],[0,1,0]), depth
// d ~ U(2,20), x ~ U(-1.1,1.1) d tan30 W/H, y ~ U(-1.1,1.1) d tan30, log-scale ~ U(-5.5,-3.5),
// quat (w,x,y,z) = normalize(N(0,1)^4), opacity logit ~ N(0,2), f_dc ~ N(0,1), f_rest ~ N(0,0.15).
// Gaussian i draws from its own splitmix64 stream (state = seed*phi + i*C) in the fixed order
// d, ux, uy, 3 log-scales, 4 quat, opacity, 3 dc, 45 rest (f_rest_0..44); values are then
// preprocessed exactly as PackedGaussians does (src/ply.ts:166-176, :202-218, :289-336).
int gs_synth_aos(uint64_t n, uint64_t seed, int W, int H, void* out_aos) {
    if ((!out_aos && n) || W <= 0 || H <= 0) return GS_ERR_INVALID;
    const double t30 = std::tan(M_PI / 6.0), aspect = (double)W / (double)H;
    float* base = (float*)out_aos;
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
        const uint64_t i = (uint64_t)ii;
        SplitMix64 r{seed * 0x9E3779B97F4A7C15ull + i * 0xD1B54A32D192ED03ull};
        float* rec = base + i * 80;
        std::memset(rec, 0, 320);
        const double d = 2.0 + 18.0 * r.uniform();
        const double x = (-1.1 + 2.2 * r.uniform()) * d * t30 * aspect;
        const double y = (-1.1 + 2.2 * r.uniform()) * d * t30;
        rec[0] = f32(x); rec[1] = f32(y); rec[2] = f32(-d);
        for (int k = 0; k < 3; ++k) rec[4 + k] = f32(std::fabs(std::exp(-5.5 + 2.0 * r.uniform())));
        double q[4];
        for (int k = 0; k < 4; ++k) q[k] = r.normal();  // (w,x,y,z) as rot_0..rot_3
        const double len = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        // normalise, swizzle to (x,y,z,w), negate xyz; `||= 0` maps NaN and -0 to +0
        const double qq[4] = {-(q[1] / len), -(q[2] / len), -(q[3] / len), q[0] / len};
        for (int k = 0; k < 4; ++k) rec[8 + k] = (qq[k] != 0.0 && !std::isnan(qq[k])) ? f32(qq[k]) : 0.0f;
        rec[12] = f32(2.0 * r.normal());
        for (int c = 0; c < 3; ++c) rec[16 + c] = f32(r.normal());
        double rest[45];
        for (int k = 0; k < 45; ++k) rest[k] = 0.15 * r.normal();
        for (int k = 1; k < 16; ++k)
            for (int c = 0; c < 3; ++c) rec[16 + 4 * k + c] = f32(rest[c * 15 + (k - 1)]);
    }
    return GS_OK;
}

}  // extern "C"
