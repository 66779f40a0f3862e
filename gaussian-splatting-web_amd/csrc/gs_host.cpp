// gs_host.cpp — host-side pieces of the C ABI that need no GPU:
//   * camera / uniform producer with wgpu-matrix 2.9.1 semantics (every store rounds to f32, the
//     arithmetic in between is JS double): lookAt, perspective, inverse(view).translation as used
//     by src/camera.ts:101-138 and packed as src/renderer.ts:24-33 / :349-384;
//   * seeded synthetic scenes, written in the reference AoS layout;
//   * the present pass (src/post_process_render.ts:54-77).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
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

// cameraFromJSON (src/camera.ts:476-503).  Every WM store rounds to f32; the arithmetic between
// stores is JS double.
int gs_camera_from_json(const double pos[3], const double rot[9], double fx, double fy, int W,
                        int H, float view[16], float proj[16], float focal[2]) {
    if (!pos || !rot || !view || !proj || W <= 0 || H <= 0) return GS_ERR_INVALID;
    // focal2fov (:463-465), getProjectionMatrix (:19-42): P row-major in f32, then transposed.
    const double fovx = 2.0 * std::atan((double)W / (2.0 * fx));
    const double fovy = 2.0 * std::atan((double)H / (2.0 * fy));
    const double zn = 0.2, zf = 100.0;
    const double top = std::tan(fovy / 2) * zn, bottom = -top;
    const double right = std::tan(fovx / 2) * zn, left = -right;
    float P[16] = {0};
    P[0] = f32((2.0 * zn) / (right - left));
    P[5] = f32((2.0 * zn) / (top - bottom));
    P[8] = f32((right + left) / (right - left));
    P[9] = f32((top + bottom) / (top - bottom));
    P[10] = f32(zf / (zf - zn));
    P[11] = f32(-(zf * zn) / (zf - zn));
    P[14] = 1.0f;
    P[15] = 0.0f;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) proj[4 * c + r] = P[4 * r + c];
    // worldToCamFromRT (:467-473): mat3.create(rows...) stores the nine values column by column
    // (WM create$3), fromMat3 widens to a mat4, translate(m, -t) in place (WM translate).
    const float m[12] = {f32(rot[0]), f32(rot[1]), f32(rot[2]), 0, f32(rot[3]), f32(rot[4]),
                         f32(rot[5]), 0, f32(rot[6]), f32(rot[7]), f32(rot[8]), 0};
    for (int c = 0; c < 3; ++c) {
        for (int r = 0; r < 3; ++r) view[4 * c + r] = m[4 * c + r];
        view[4 * c + 3] = 0.0f;
    }
    view[12] = view[13] = view[14] = 0.0f;
    view[15] = 1.0f;
    const double v0 = f32(pos[0] * -1.0), v1 = f32(pos[1] * -1.0), v2 = f32(pos[2] * -1.0);
    for (int r = 0; r < 4; ++r)
        view[12 + r] = f32((double)view[r] * v0 + (double)view[4 + r] * v1 + (double)view[8 + r] * v2 +
                           (double)view[12 + r]);
    if (focal) {
        focal[0] = f32(H);
        focal[1] = f32(W);
    }
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
            if (a < 0.99f) {  // pow(a, 4) as (a^2)^2: the device kernel rounds identically
                const float a2 = a * a;
                a = a2 * a2;
            }
            dst[4 * x + 3] = a;
        }
    }
    return GS_OK;
}

// ---- PNG (RGBA8, zlib stream of stored deflate blocks) -------------------------------------
static uint32_t crc32_update(uint32_t c, const uint8_t* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
            table[i] = v;
        }
        init = true;
    }
    c = ~c;
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

static uint64_t png_size(int W, int H) {
    const uint64_t raw = (uint64_t)H * (1 + 4 * (uint64_t)W);
    const uint64_t blocks = raw ? (raw + 65534) / 65535 : 1;
    return 8 + 25 + (12 + 2 + raw + 5 * blocks + 4) + 12;
}

int gs_encode_png(const uint8_t* rgba8, int W, int H, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    if (!out_len || W <= 0 || H <= 0 || (!rgba8 && out)) return GS_ERR_INVALID;
    const uint64_t need = png_size(W, H);
    *out_len = need;
    if (!out) return GS_OK;
    if (cap < need) return GS_ERR_INVALID;
    uint8_t* o = out;
    auto be32 = [&](uint32_t v) {
        o[0] = v >> 24; o[1] = (v >> 16) & 0xFF; o[2] = (v >> 8) & 0xFF; o[3] = v & 0xFF;
        o += 4;
    };
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    std::memcpy(o, sig, 8);
    o += 8;
    auto chunk = [&](const char* type, uint64_t len, auto&& body) {
        be32((uint32_t)len);
        uint8_t* start = o;
        std::memcpy(o, type, 4);
        o += 4;
        body();
        be32(crc32_update(0, start, (size_t)(o - start)));
    };
    chunk("IHDR", 13, [&] {
        be32((uint32_t)W);
        be32((uint32_t)H);
        *o++ = 8;  // bit depth
        *o++ = 6;  // colour type RGBA
        *o++ = 0; *o++ = 0; *o++ = 0;  // deflate, adaptive filtering, no interlace
    });
    const uint64_t row = 1 + 4 * (uint64_t)W, raw = (uint64_t)H * row;
    const uint64_t blocks = (raw + 65534) / 65535;
    chunk("IDAT", 2 + raw + 5 * blocks + 4, [&] {
        *o++ = 0x78;  // zlib: deflate, 32 K window
        *o++ = 0x01;
        uint32_t s1 = 1, s2 = 0;  // Adler-32
        uint64_t pos = 0;         // position in the filtered raw stream
        for (uint64_t b = 0; b < blocks; ++b) {
            const uint32_t len = (uint32_t)std::min<uint64_t>(65535, raw - pos);
            *o++ = b + 1 == blocks ? 1 : 0;  // BFINAL, BTYPE = stored
            *o++ = len & 0xFF; *o++ = len >> 8;
            *o++ = ~len & 0xFF; *o++ = (~len >> 8) & 0xFF;
            for (uint32_t k = 0; k < len; ++k, ++pos) {
                const uint64_t y = pos / row, c = pos % row;
                const uint8_t v = c == 0 ? 0 : rgba8[y * 4 * (uint64_t)W + (c - 1)];  // filter 0
                *o++ = v;
                s1 = (s1 + v) % 65521;
                s2 = (s2 + s1) % 65521;
            }
        }
        be32((s2 << 16) | s1);
    });
    chunk("IEND", 0, [] {});
    return (uint64_t)(o - out) == need ? GS_OK : GS_ERR_INTERNAL;
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


// ---- PLY ingest: PackedGaussians (src/ply.ts:54-355) restated in C++ ---------------------------
// Same header reading (50-byte chunks until "end_header", src/ply.ts:54-102), property order (a JS
// object: integer-like names first, then first-insertion order), only float / uchar properties
// advance the read offset (:104-123), SH feature order f_dc_c then f_rest_{c*K+i} (:222-232),
// rotation normalised in double, swizzled to (-x,-y,-z,w) with NaN/-0 -> 0 (:166-213, :289-297),
// scale = |exp(s)| (:214-218), every value rounded once to f32 when packed (src/packing.ts), and
// min_pos / max_pos by the running x+y+z comparison of src/mylib.ts:28-30 (:276-286).
namespace {

struct PlyProp {
    std::string name, type;
};

bool js_index_key(const std::string& k, uint64_t& v) {  // canonical array index -> ordered first
    if (k.empty() || k.size() > 10 || (k.size() > 1 && k[0] == '0')) return false;
    v = 0;
    for (char c : k) {
        if (c < '0' || c > '9') return false;
        v = v * 10 + (uint64_t)(c - '0');
    }
    return v < 4294967295ull;
}

bool is_word(char c) { return std::isalnum((unsigned char)c) || c == '_'; }

// first match of /(\w+)\s+(\w+)\s+(\w+)/ in line: (group2, group3)
bool match3(const std::string& l, std::string& g2, std::string& g3) {
    for (size_t st = 0; st < l.size(); ++st) {
        if (!is_word(l[st]) || (st > 0 && is_word(l[st - 1]) && false)) continue;
        size_t i = st;
        std::string g[3];
        bool ok = true;
        for (int k = 0; k < 3 && ok; ++k) {
            size_t b = i;
            while (i < l.size() && is_word(l[i])) ++i;
            if (i == b) { ok = false; break; }
            g[k] = l.substr(b, i - b);
            if (k < 2) {
                size_t ws = i;
                while (i < l.size() && std::isspace((unsigned char)l[i])) ++i;
                if (i == ws) ok = false;
            }
        }
        if (ok) {
            g2 = g[1];
            g3 = g[2];
            return true;
        }
    }
    return false;
}

std::string js_trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

struct PlyHeader {
    uint64_t count = 0;
    std::vector<PlyProp> props;  // JS key order
    uint64_t data_offset = 0;
};

int ply_header(const uint8_t* buf, uint64_t bytes, PlyHeader& h) {
    std::string text;
    uint64_t off = 0;
    for (;;) {
        if (off + 50 > bytes) return GS_ERR_INVALID;  // new Uint8Array(buf, off, 50) throws
        text.append((const char*)buf + off, 50);
        off += 50;
        if (text.find("end_header") != std::string::npos) break;
    }
    std::vector<std::string> order;
    std::map<std::string, std::string> types;
    size_t pos = 0;
    for (;;) {
        const size_t e = text.find('\n', pos);
        const std::string line = js_trim(text.substr(pos, e == std::string::npos ? std::string::npos : e - pos));
        if (line.rfind("element vertex", 0) == 0) {
            const size_t d = line.find_first_of("0123456789");
            if (d != std::string::npos) {
                size_t q = d;
                uint64_t v = 0;
                while (q < line.size() && std::isdigit((unsigned char)line[q])) v = v * 10 + (uint64_t)(line[q++] - '0');
                h.count = v;
            }
        } else if (line.rfind("property", 0) == 0) {
            std::string t, nm;
            if (match3(line, t, nm)) {
                if (!types.count(nm)) order.push_back(nm);
                types[nm] = t;
            }
        } else if (line == "end_header") {
            break;
        }
        if (e == std::string::npos) break;
        pos = e + 1;
    }
    // JS property enumeration order: integer-like keys ascending, then insertion order
    std::vector<std::pair<uint64_t, std::string>> idx;
    std::vector<std::string> rest;
    for (const auto& k : order) {
        uint64_t v;
        if (js_index_key(k, v)) idx.push_back({v, k}); else rest.push_back(k);
    }
    std::sort(idx.begin(), idx.end());
    for (const auto& k : idx) h.props.push_back({k.second, types[k.second]});
    for (const auto& k : rest) h.props.push_back({k, types[k]});
    h.data_offset = text.find("end_header") + std::string("end_header").size() + 1;
    return GS_OK;
}

// DataView.getFloat32 into a JS number: a signalling NaN comes back quiet (f32 -> f64 conversion)
inline float f32_from_le(const uint8_t* p) {
    uint32_t u;
    std::memcpy(&u, p, 4);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) u |= 0x00400000u;
    float v;
    std::memcpy(&v, &u, 4);
    return v;
}

}  // namespace

int gs_ply_parse(const void* ply, uint64_t bytes, gs_ply_info* info, void* out_aos, uint64_t out_bytes) {
    if (!ply || !info) return GS_ERR_INVALID;
    const uint8_t* buf = (const uint8_t*)ply;
    PlyHeader h;
    int rc = ply_header(buf, bytes, h);
    if (rc) return rc;
    // per-property byte offset within a vertex (float 4, uchar 1, anything else 0 and unread)
    std::map<std::string, int> col;       // name -> index into props
    std::vector<uint32_t> poff(h.props.size());
    uint64_t stride = 0;
    int n_rest = 0;
    for (size_t k = 0; k < h.props.size(); ++k) {
        col[h.props[k].name] = (int)k;
        poff[k] = (uint32_t)stride;
        if (h.props[k].type == "float") stride += 4;
        else if (h.props[k].type == "uchar") stride += 1;
        if (h.props[k].name.rfind("f_rest_", 0) == 0) ++n_rest;
    }
    const double per_color = n_rest / 3.0;
    const double deg = std::sqrt(per_color + 1.0) - 1.0;
    int n_sh;
    if (deg == 0.0) n_sh = 1;
    else if (deg == 1.0) n_sh = 4;
    else if (deg == 2.0) n_sh = 9;
    else if (deg == 3.0) n_sh = 16;
    else return GS_ERR_UNSUPPORTED;  // "Unsupported SH degree"
    const uint64_t rec = 64 + 16 * (uint64_t)n_sh;
    if (h.data_offset + h.count * stride > bytes && h.count > 0 && stride > 0) return GS_ERR_INVALID;
    if (h.count > 0 && stride == 0 && h.data_offset > bytes) return GS_ERR_INVALID;
    info->num_gaussians = h.count;
    info->sh_degree = (int32_t)deg;
    info->n_sh_coeffs = n_sh;
    info->record_bytes = rec;
    info->data_offset = h.data_offset;
    info->vertex_stride = stride;
    // value of property `name` of vertex v as JS sees it (missing -> NaN, as `undefined` packs)
    auto column = [&](const std::string& name) { auto it = col.find(name); return it == col.end() ? -1 : it->second; };
    const uint8_t* data = buf + h.data_offset;
    auto value = [&](uint64_t v, int c) -> double {
        if (c < 0) return NAN;
        const PlyProp& pr = h.props[c];
        const uint8_t* p = data + v * stride + poff[c];
        if (pr.type == "float") return (double)f32_from_le(p);
        if (pr.type == "uchar") return (double)p[0] / 255.0;
        return NAN;  // never read by the reference: undefined
    };
    const int cx = column("x"), cy = column("y"), cz = column("z");
    // bounding box, sequential as the reference (src/ply.ts:276-286, src/mylib.ts:28-30)
    double mx[3] = {-99999, -99999, -99999}, mn[3] = {99999, 99999, 99999};
    for (uint64_t v = 0; v < h.count; ++v) {
        const double x = value(v, cx), y = value(v, cy), z = value(v, cz);
        const double s = x + y + z;
        if (s > mx[0] + mx[1] + mx[2]) { mx[0] = x; mx[1] = y; mx[2] = z; }
        if (!(s > mn[0] + mn[1] + mn[2])) { mn[0] = x; mn[1] = y; mn[2] = z; }
    }
    for (int k = 0; k < 3; ++k) {
        info->min_pos[k] = (float)mn[k];
        info->max_pos[k] = (float)mx[k];
    }
    info->min_pos_d[0] = mn[0]; info->min_pos_d[1] = mn[1]; info->min_pos_d[2] = mn[2];
    info->max_pos_d[0] = mx[0]; info->max_pos_d[1] = mx[1]; info->max_pos_d[2] = mx[2];
    if (!out_aos) return GS_OK;
    if (out_bytes < h.count * rec) return GS_ERR_INVALID;
    std::vector<int> shc(3 * (size_t)n_sh);
    const int K = n_rest / 3;
    for (int c = 0; c < 3; ++c) shc[c] = column("f_dc_" + std::to_string(c));
    for (int i = 0; i < K && 1 + i < n_sh; ++i)
        for (int c = 0; c < 3; ++c) shc[3 * (1 + i) + c] = column("f_rest_" + std::to_string(c * K + i));
    const int cs[3] = {column("scale_0"), column("scale_1"), column("scale_2")};
    const int cr[4] = {column("rot_0"), column("rot_1"), column("rot_2"), column("rot_3")};
    const int co = column("opacity");
    uint8_t* out = (uint8_t*)out_aos;
    std::memset(out, 0, h.count * rec);
#pragma omp parallel for schedule(static)
    for (int64_t vv = 0; vv < (int64_t)h.count; ++vv) {
        const uint64_t v = (uint64_t)vv;
        float* r = (float*)(out + v * rec);
        r[0] = (float)value(v, cx);
        r[1] = (float)value(v, cy);
        r[2] = (float)value(v, cz);
        for (int k = 0; k < 3; ++k) r[4 + k] = (float)std::fabs(std::exp(value(v, cs[k])));
        const double q0 = value(v, cr[0]), q1 = value(v, cr[1]), q2 = value(v, cr[2]), q3 = value(v, cr[3]);
        const double len = std::sqrt(((q0 * q0 + q1 * q1) + q2 * q2) + q3 * q3);
        double qq[4] = {(q1 / len) * -1.0, (q2 / len) * -1.0, (q3 / len) * -1.0, q0 / len};
        for (double& x : qq)
            if (!(x != 0.0) || std::isnan(x)) x = 0.0;  // `qq[i] ||= 0`: NaN, 0 and -0 -> +0
        for (int k = 0; k < 4; ++k) r[8 + k] = (float)qq[k];
        r[12] = (float)value(v, co);
        for (int k = 0; k < n_sh; ++k)
            for (int c = 0; c < 3; ++c) r[16 + 4 * k + c] = (float)value(v, shc[3 * k + c]);
    }
    return GS_OK;
}

}  // extern "C"
