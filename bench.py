#!/usr/bin/env python3
"""Headline benchmark: Msplats/s (and fps) at 1920x1080 on a 6.1 M-Gaussian scene, 1..8 MI355X.

BASELINE.json metric "Msplats/s + frames/s at 1920x1080, 6 M Gaussians; 1/2/4/8 MI355X",
configs[3] ("INRIA bicycle ~6 M at 1920x1080, 1->8 MI355X row-strip + RCCL all-gather").  The
bicycle PLY is not in this image, so the workload is the seeded synthetic stand-in of SURVEY §8d
(seed 6, N = 6,100,000, SH degree 3) — reported in `data`/`config`.

A step = one frame: uniform upload -> project/key -> depth sort -> bin -> tile sort -> composite
(-> all-gather of the row strips at N > 1).  The scene is uploaded before timing (inputs resident
in HBM).  Launch:  python bench.py [--gpus 1 --steps 50 --warmup 5]
                   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Prints ONE JSON line (rank 0).
"""
import argparse
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))

import numpy as np  # noqa: E402

import gsplat_amd as gs  # noqa: E402
from gsplat_amd.strips import strip_geometry  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 4 cycles at 2.4 GHz
VALU_PEAK = 256 * 4 * 2.4e9 / 4  # wave instructions / s


def algorithmic_bytes(stage, n, n_vis, k, W, H, n_chunk0=None):
    """Bytes a kernel group must move per launch."""
    if stage == "project":
        # k_cull reads the 16-B cull plane of every Gaussian of a surviving partition (<= N);
        # each chunk-0 splat: its 48-B geometry record and 192-B SH read, 80 B of slot records
        # (composite record 48, sort key 8, storage index 4, rect 4, per-Gaussian r2 16) written
        return 16 * n + 320 * (n_vis if n_chunk0 is None else n_chunk0)
    if stage == "composite":
        # per (tile, splat) entry: the 4-B slot and the 48-B composite record; RGBA f16 out
        return 52 * k + 8 * W * H
    raise KeyError(stage)


def pmc_traffic(kernel):
    """HBM bytes per frame of `kernel` from the committed PMC profile of this bench command
    (profiles/<round>_pmc.json: FETCH_SIZE x2 (gfx950) + WRITE_SIZE, summed over the kernel's
    launches in a frame); None when no profile is committed."""
    names = {"composite": "k_composite<false>", "project": "k_project"}
    prof = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc.json")) \
        if os.path.isdir(os.path.join(ROOT, "profiles")) else []
    if not prof:
        return None, None
    d = json.load(open(os.path.join(ROOT, "profiles", prof[-1])))
    tot = 0.0
    for lab, e in d.items():
        if lab.startswith(names[kernel] + "#") and "traffic_bytes" in e:
            tot += e["traffic_bytes"]
    return (tot if tot else None), prof[-1]


def pmc_valu(kernel):
    """VALU wave instructions per frame of `kernel` from the committed PMC profile (SQ_INSTS_VALU)."""
    names = {"composite": "k_composite<false>", "project": "k_project"}
    prof = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc.json")) \
        if os.path.isdir(os.path.join(ROOT, "profiles")) else []
    if not prof:
        return None
    d = json.load(open(os.path.join(ROOT, "profiles", prof[-1])))
    tot = sum(e.get("SQ_INSTS_VALU", 0.0) for lab, e in d.items() if lab.startswith(names[kernel] + "#"))
    return tot or None


def frame_bytes(n, n_vis, k, W, H):
    """B = 236 N + 148 N_vis + 48 K + 16 W H."""
    return 236 * n + 148 * n_vis + 48 * k + 16 * W * H


def cpu_baseline(aos, n, W, H, u):
    """The oracle (CPU restatement of the reference semantics) on the same frame, host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as orc
    t0 = time.perf_counter()
    _, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    dt = time.perf_counter() - t0
    return {"value": n / dt / 1e6, "unit": "Msplats/s", "cores": orc.num_threads(), "kind": "port",
            "sample": "1 full frame of the same %d-Gaussian %dx%d workload (project, std::stable_sort, "
                      "composite; %.1f s wall)" % (n, W, H, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=6_100_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--seed", type=int, default=6)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus %d needs torch.distributed.run with %d processes" % (args.gpus, args.gpus))
    W, H, N = args.width, args.height, args.n

    launched = "WORLD_SIZE" in os.environ  # torch.distributed.run: the RCCL path, even at N = 1
    dist = None
    if launched:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    aos = gs.synth_aos(N, args.seed, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(local_rank)
    scene = gs.Scene(ctx, aos, N, 16)

    row0, rows_padded, t0, t1 = strip_geometry(H, rank, world)
    # output RGBA f16: the reference's framebuffer format (rgba16float, src/simple_render.ts:499-505);
    # accumulation stays fp32 (gs_opts.accum), rounded once at the store
    # timed loop: HIP events around the composite only (timing=2; an event record costs the stream a
    # few microseconds); a separate shorter loop with events between every stage (timing=1) gives
    # the stage breakdown
    opts_head = gs.make_opts(strip_index=rank, strip_count=world, timing=2, out_format=gs.GS_OUT_RGBA_F16)
    opts_stage = gs.make_opts(strip_index=rank, strip_count=world, timing=1, out_format=gs.GS_OUT_RGBA_F16)
    cur = {"opts": opts_head}
    strip_bytes = rows_padded * W * 8
    if launched:
        import torch
        from gsplat_amd.strips import StripPipeline
        stream = torch.cuda.current_stream()
        pipe = StripPipeline(rows_padded, W, dtype=torch.float16)  # gather t beside render t+1

        def frame():
            strip = pipe.next_strip()
            scene.render_device(u, W, H, strip.data_ptr(), strip_bytes, stream.cuda_stream, cur["opts"])
            pipe.submit()

        def sync():
            pipe.finish()
            torch.cuda.synchronize()
            dist.barrier()
    else:
        buf = gs.DeviceBuffer(H * W * 8)

        def frame():
            scene.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, cur["opts"])

        def sync():
            ctx.sync()

    for _ in range(args.warmup):
        frame()
    sync()
    ctx.timings_reset()
    sync()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        frame()
    sync()
    elapsed = time.perf_counter() - t_start
    ms_composite_live = ctx.timings()["ms_composite"]  # HIP events over the timed region
    # stage breakdown (not timed for `value`)
    cur["opts"] = opts_stage
    ctx.timings_reset()
    for _ in range(min(args.steps, 50)):
        frame()
    sync()
    st = ctx.timings()
    st["ms_composite_stage_pass"] = st["ms_composite"]
    st["ms_composite"] = ms_composite_live
    # one untimed one-chunk frame for the exact visible count and K of SURVEY 8d's byte model
    # (with a chunk split the pipeline never projects the splats past it)
    cur["opts"] = gs.make_opts(strip_index=rank, strip_count=world, chunk_fraction=1.0,
                               out_format=gs.GS_OUT_RGBA_F16)
    frame()
    sync()
    ex = ctx.timings()
    if launched:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tot = torch.tensor([ex["n_vis"], ex["k_total"], st["k_entries"]], dtype=torch.float64, device="cuda")
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        n_vis_all, k_all, k_binned = (int(x) for x in tot.tolist())
    else:
        n_vis_all, k_all, k_binned = ex["n_vis"], ex["k_total"], st["k_entries"]

    ms = elapsed / args.steps * 1e3
    fps = args.steps / elapsed
    value = N * args.steps / elapsed / 1e6

    # roofline of the dominant kernel (this rank's per-launch event time, HIP events on the
    # stream the kernel runs on; algorithmic bytes per launch of this rank)
    stages = {"project": st["ms_project"], "composite": st["ms_composite"]}
    dom = max(stages, key=stages.get)
    rows_here = max(0, min(t1 * 16, H) - row0)
    a_bytes = algorithmic_bytes(dom, N, ex["n_vis"], st["k_entries"], W, rows_here,
                                n_chunk0=int(round(st["chunk_fraction"] * st["n_vis"])))
    achieved = a_bytes / (stages[dom] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(dom)
    valu = pmc_valu(dom) if world == 1 else None
    fb = frame_bytes(N, n_vis_all, k_all, W, H)

    if rank == 0:
        out = {
            "metric": "Msplats/s at 1920x1080, 6.1 M Gaussians (synthetic bicycle stand-in)",
            "value": round(value, 3),
            "unit": "Msplats/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "fps": round(fps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (SURVEY §8d generator, splitmix64 seed %d; bicycle PLY absent); "
                    "output RGBA f16 (the reference's rgba16float framebuffer)" % args.seed,
            "config": {"workload": "configs[3]: %d Gaussians (SH deg 3) at %dx%d, lookAt([0,0,0],[0,0,-1]) "
                                   "perspective(60deg,W/H,0.03,1000)" % (N, W, H),
                       "n_gaussians": N, "width": W, "height": H,
                       "parallelism": "row-strips x%d + all-gather" % world if world > 1 else "single GPU"},
            # per-stage HIP-event times from the separate timing=1 loop (events between stages add
            # ~20 us to its frame), except ms_composite, timed live in the headline loop:
            # project = partition cull + cull + projection/colour, bin = count + scans + emission,
            # tile_sort = per-tile sort, chunk1 = the chunk-1 launch (returns at once when chunk 0
            # saturated every tile)
            "stages_ms": {"ms_total": round(st["ms_total"], 4), "ms_project": round(st["ms_project"], 4),
                          "ms_bin": round(st["ms_bin"], 4), "ms_tile_sort": round(st["ms_tile_sort"], 4),
                          "ms_composite": round(st["ms_composite"], 4), "ms_chunk1": round(st["ms_sort"], 4),
                          "ms_other": round(st["ms_other"], 4)},
            "n_vis": n_vis_all,         # exact, from the one-chunk frame
            "k_total": k_all,           # SURVEY's K (box tiles of the visible splats), same frame
            "k_binned": k_binned,       # (tile, splat) entries a timed frame binned (chunk 0)
            # chunk-0 splats of a timed frame over the exact visible count
            "chunk_fraction": round(st["chunk_fraction"] * st["n_vis"] / max(1, ex["n_vis"]), 4),
            "tiles_unsaturated": st["tiles_unsaturated"],
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved * 1e9 / HBM_PEAK, 4),
                         "traffic": int(traffic) if traffic else None,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": int(a_bytes),
                         "per": "frame (the kernel's launches in one frame, HIP events on the render stream)"},
            # the dominant kernel's real bound: VALU issue (PMC instruction count of this command's
            # committed profile / the live event-timed duration)
            "valu_roofline": ({"kernel": dom, "insts_per_launch": int(valu),
                               "achieved": round(valu / (stages[dom] * 1e-3) / 1e9, 1),
                               "peak": VALU_PEAK / 1e9, "unit": "G wave-instr/s",
                               "frac": round(valu / (stages[dom] * 1e-3) / VALU_PEAK, 4),
                               "source": traffic_src} if valu else None),
            "frame_roofline": {"bytes": int(fb), "frac": round(fb / (ms * 1e-3) / (world * HBM_PEAK), 4),
                               "compulsory_frac": round((236 * N + 16 * W * H) / (ms * 1e-3) / (world * HBM_PEAK), 4),
                               "formula": "236N + 148N_vis + 48K + 16WH (SURVEY 8d)"},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(aos, N, W, H, u)
        print(json.dumps(out), flush=True)

    scene.close()
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
