// Sanitizer driver: the host-side C ABI (gs_host.cpp: PLY ingest, camera / uniform
// producer, present, PNG, synthetic scenes) and the CPU oracle, built with
// -fsanitize=address,undefined, run over the golden PLYs, their truncations and header mutations,
// and small renders.  Exit status 0 = clean (the sanitizers abort on the first finding).
// Build and run: make -C tools/asan run  (tests/test_asan.py does this).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>
#include <array>

#include "../../include/gsplat.h"
#include "../../oracle/gs_oracle.cpp"  // the oracle TU itself, instrumented

static std::vector<uint8_t> read_file(const char* path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

// One parse into an exactly sized heap buffer (the sanitizer sees any write past it).
static int parse_exact(const std::vector<uint8_t>& b, gs_ply_info& info, std::vector<uint8_t>* keep) {
    // the input copied into an exactly sized allocation, so an over-read past the file is caught
    uint8_t* in = (uint8_t*)std::malloc(b.size() ? b.size() : 1);
    if (!b.empty()) std::memcpy(in, b.data(), b.size());
    int rc = gs_ply_parse(in, b.size(), &info, nullptr, 0);
    if (rc == GS_OK && info.num_gaussians * info.record_bytes < (64ull << 20)) {
        const uint64_t bytes = info.num_gaussians * info.record_bytes;
        uint8_t* out = (uint8_t*)std::malloc(bytes ? bytes : 1);
        rc = gs_ply_parse(in, b.size(), &info, out, bytes);
        if (rc == GS_OK && keep) keep->assign(out, out + bytes);
        // a buffer one record short must be refused, not overrun
        if (bytes >= info.record_bytes && info.record_bytes)
            (void)gs_ply_parse(in, b.size(), &info, out, bytes - info.record_bytes);
        std::free(out);
    }
    std::free(in);
    return rc;
}

int main(int argc, char** argv) {
    uint64_t parses = 0, ok = 0;
    std::vector<uint8_t> simple_aos;
    int simple_nsh = 0;
    uint64_t simple_n = 0;
    for (int a = 1; a < argc; ++a) {
        const std::vector<uint8_t> b = read_file(argv[a]);
        gs_ply_info info{};
        std::vector<uint8_t> aos;
        if (parse_exact(b, info, &aos) == GS_OK) ++ok;
        ++parses;
        if (std::strstr(argv[a], "simple.ply")) {
            simple_aos = aos;
            simple_nsh = info.n_sh_coeffs;
            simple_n = info.num_gaussians;
        }
        // truncations at ~64 points and single-byte header mutations
        size_t hdr = 0;
        for (size_t i = 0; i + 10 < b.size() && i < 4096; ++i)
            if (!std::memcmp(&b[i], "end_header", 10)) { hdr = i + 11; break; }
        for (size_t k = 0; k < 64 && !b.empty(); ++k) {
            std::vector<uint8_t> t(b.begin(), b.begin() + (b.size() * k) / 64);
            gs_ply_info ti{};
            parse_exact(t, ti, nullptr);
            ++parses;
        }
        const uint8_t vals[] = {'0', '9', ' ', '\n', 'x', 0, 0xff};
        for (size_t i = 0; i < hdr; i += 5)
            for (uint8_t v : vals) {
                std::vector<uint8_t> m = b;
                m[i] = v;
                gs_ply_info mi{};
                parse_exact(m, mi, nullptr);
                ++parses;
            }
    }
    // camera / uniform producer
    const double eye[3] = {0.3, -5.0, 3.0}, tgt[3] = {0.0, 0.1, -1.0}, up[3] = {0.0, 1.0, 0.0};
    float view[16], proj[16], pos[3], focal[2], uni[40];
    if (gs_look_at(eye, tgt, up, view) || gs_perspective(1.04719755, 16.0 / 9.0, 0.03, 1000.0, proj) ||
        gs_camera_position(view, pos) || gs_pack_uniforms(view, proj, pos, 0.5f, 0.3f, 100, 100, 1, uni))
        return 2;
    const double cp[3] = {-0.16, -1.97, 3.9}, rot[9] = {-0.99, 0.06, 0.07, 0.09, 0.6, 0.79, 0.005, 0.79, -0.6};
    if (gs_camera_from_json(cp, rot, 3104.3, 3106.0, 1920, 1080, view, proj, focal)) return 3;
    if (gs_camera_from_json(cp, rot, 3104.3, 3106.0, 0, 1080, view, proj, focal) != GS_ERR_INVALID) return 4;
    // present and PNG on odd sizes, exactly sized buffers
    for (int W = 1; W < 40; W += 13)
        for (int H = 1; H < 30; H += 7) {
            const size_t px = (size_t)W * H;
            float* fb = (float*)std::malloc(px * 16);
            float* out = (float*)std::malloc(px * 16);
            for (size_t i = 0; i < 4 * px; ++i) fb[i] = (float)((i * 2654435761u) % 1000) / 700.0f;
            if (gs_present(fb, W, H, out) || or_present(fb, W, H, out)) return 5;
            uint8_t* rgba = (uint8_t*)std::malloc(px * 4);
            for (size_t i = 0; i < 4 * px; ++i) rgba[i] = (uint8_t)(i * 7);
            uint64_t need = 0;
            if (gs_encode_png(rgba, W, H, nullptr, 0, &need)) return 6;
            uint8_t* png = (uint8_t*)std::malloc(need);
            uint64_t got = 0;
            if (gs_encode_png(rgba, W, H, png, need, &got) || got != need) return 7;
            if (gs_encode_png(rgba, W, H, png, need - 1, &got) != GS_ERR_INVALID) return 8;
            std::free(png); std::free(rgba); std::free(fb); std::free(out);
        }
    // synthetic scene, then the oracle on it and on simple.ply (both accumulation modes, quirks)
    const uint64_t n = 3000;
    std::vector<uint8_t> syn(n * 320);
    if (gs_synth_aos(n, 7, 96, 64, syn.data())) return 9;
    gs_look_at(std::array<double, 3>{0, 0, 0}.data(), std::array<double, 3>{0, 0, -1}.data(), up, view);
    gs_perspective(1.04719755, 96.0 / 64.0, 0.03, 1000.0, proj);
    gs_camera_position(view, pos);
    gs_pack_uniforms(view, proj, pos, 0, 0, 96, 64, 1, uni);
    for (int accum = 0; accum < 2; ++accum) {
        std::vector<float> img(96 * 64 * 4);
        or_stats st{};
        if (or_render(syn.data(), n, 16, uni, 96, 64, accum, 1e-4f, 0, nullptr, nullptr, img.data(), &st)) return 10;
        if (!simple_aos.empty()) {
            std::vector<uint32_t> sk(simple_n, 0), sv(simple_n, 0);
            for (int f = 0; f < 2; ++f)
                if (or_render(simple_aos.data(), simple_n, simple_nsh, uni, 96, 64, accum, 1e-4f, 1, sk.data(),
                              sv.data(), img.data(), &st))
                    return 11;
        }
    }
    std::printf("asan driver clean: %llu parses (%llu of the %d files accepted)\n", (unsigned long long)parses,
                (unsigned long long)ok, argc - 1);
    return 0;
}
