#!/usr/bin/env python3
"""Render a scene to PNG through the product path: gs_render_device (rgba16float framebuffer, as
the reference) -> gs_present_device (PostProcessRenderer: flip + alpha remap) -> RGBA8 ->
gs_encode_png.  For visual diffs.

    python tools/render_png.py --ply tests/golden/ply/simple.ply --width 512 --height 512 out.png
    python tools/render_png.py --synth 1000000 --width 1920 --height 1080 out.png
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--ply")
    src.add_argument("--synth", type=int)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--eye", type=float, nargs=3, default=None)
    ap.add_argument("--target", type=float, nargs=3, default=(0.0, 0.0, 0.0))
    ap.add_argument("--fit", action="store_true", help="aim at the PLY's bounding box (its centre, from -z)")
    ap.add_argument("out")
    a = ap.parse_args()
    W, H = a.width, a.height
    if a.ply:
        aos, info = gs.parse_ply(open(a.ply, "rb").read())
        n, nsh = info["numGaussians"], info["nShCoeffs"]
        eye, target = a.eye or (0.0, 0.0, -5.0), a.target  # Camera.default (src/camera.ts:101-111)
        if a.fit:
            lo, hi = np.array(info["min_pos"], float), np.array(info["max_pos"], float)
            target = tuple((lo + hi) / 2)
            eye = tuple(np.array(target) + (0.0, 0.0, -1.2 * float(np.linalg.norm(hi - lo)) - 1e-3))
        u = gs.pack_uniforms(gs.look_at(eye, target), gs.perspective(1.04719755, W / H, 0.03, 1000.0),
                             focal=(W, H))
    else:
        n, nsh = a.synth, 16
        aos = gs.synth_aos(n, a.seed, W, H)
        u = gs.bench_uniforms(W, H)
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, n, nsh)
        fb = gs.DeviceBuffer(W * H * 8)
        img = gs.DeviceBuffer(W * H * 4)
        sc.render_device(u, W, H, fb.ptr.value, fb.nbytes, opts=gs.make_opts(out_format=gs.GS_OUT_RGBA_F16))
        ctx.present_device(fb.ptr, gs.GS_OUT_RGBA_F16, W, H, gs.GS_PRESENT_RGBA8, img.ptr, img.nbytes)
        ctx.sync()
        rgba8 = np.empty((H, W, 4), np.uint8)
        img.to_host(rgba8)
        gs.write_png(a.out, rgba8)
        sc.close()
    print("wrote %s (%dx%d, %d Gaussians)" % (a.out, W, H, n))


if __name__ == "__main__":
    main()
