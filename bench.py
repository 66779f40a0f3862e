#!/usr/bin/env python3
"""Headline benchmark: Msplats/s (and fps) at 1920x1080 on a 6.1 M-Gaussian scene, 1..8 MI355X.

BASELINE.json metric "Msplats/s + frames/s at 1920x1080, 6 M Gaussians; 1/2/4/8 MI355X",
configs[3] ("INRIA bicycle ~6 M at 1920x1080, 1->8 MI355X row-strip + RCCL all-gather").  The
bicycle PLY is not in this image, so the workload is the seeded synthetic stand-in of SURVEY §8d
(seed 6, N = 6,100,000, SH degree 3) — reported in `data`/`config`.

A step = one frame: uniform upload -> project/key -> depth sort -> bin -> tile sort -> composite
(-> all-gather of the row strips at N > 1).  The scene is uploaded before timing (inputs resident
in HBM).  Launch:  python bench.py [--gpus N --steps 50 --warmup 5] [--config 4]
                   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Without torch.distributed.run, --gpus N > 1 starts the N ranks itself (one process per GPU, the
same environment torch.distributed.run gives them) before anything touches a GPU.
Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))

import numpy as np  # noqa: E402

import gsplat_amd as gs  # noqa: E402
from gsplat_amd.strips import strip_geometry  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMD-32s, one wave64 VALU instruction per SIMD every 2 cycles at
# 2.4 GHz once two or more waves share a SIMD (MI355X_MICROARCH.md "Wave scheduling", v_fma_f32 row);
# transcendentals (v_exp_f32) issue at a quarter of that rate
VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave instructions / s

CONFIGS = {  # BASELINE.json configs the bench can run (index: N, W, H, seed)
    3: (6_100_000, 1920, 1080, 6),   # the headline: bicycle ~6 M stand-in at 1080p
    4: (50_000_000, 3840, 2160, 50),  # synthetic 50 M at 4K (the HBM-roofline configuration)
}


def algorithmic_bytes(stage, n, n_vis, k, W, H, n_chunk0=None, sorts=False):
    """Bytes a kernel group must move per launch.  sorts: the composite sorts its
    tile's list in the same launch (a still camera's frames, k_composite_ts): 16 B more per entry
    (the unordered slot read, its 8-B sort key gathered, the ordered slot written)."""
    if stage == "project":
        # k_cull reads the 16-B cull plane of every Gaussian of a surviving partition (<= N);
        # each chunk-0 splat: its 48-B geometry record and 192-B SH read, 80 B of slot records
        # (composite record 48, sort key 8, storage index 4, rect 4, per-Gaussian r2 16) written
        return 16 * n + 320 * (n_vis if n_chunk0 is None else n_chunk0)
    if stage == "composite":
        # per (tile, splat) entry: the 4-B slot and the 48-B composite record; RGBA f16 out
        return (68 if sorts else 52) * k + 8 * W * H
    raise KeyError(stage)


def pmc_traffic(kernel):
    """HBM bytes per frame of `kernel` from the committed PMC profile of this bench command
    (profiles/<round>_pmc.json: FETCH_SIZE x2 (gfx950) + WRITE_SIZE, summed over the kernel's
    launches in a frame); None when no profile is committed."""
    prof = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc.json")) \
        if os.path.isdir(os.path.join(ROOT, "profiles")) else []
    if not prof:
        return None, None
    d = json.load(open(os.path.join(ROOT, "profiles", prof[-1])))
    tot = 0.0
    for lab, e in d.items():
        if _is_kernel(lab, kernel) and "traffic_bytes" in e:
            tot += e["traffic_bytes"]
    return (tot if tot else None), prof[-1]


def _is_kernel(label, kernel):
    """A PMC profile label ("k_composite<false, 1, 2>#0": kernel name, template arguments, launch
    position in the frame) of the chunk-0 composite (any of its template instances; not chunk 1's
    k_composite_q) or of the projection."""
    name = label.split("#")[0]
    if kernel == "composite":  # (k_composite_ts: with its tile's sort, a still camera's frames)
        return name.startswith("k_composite<false") or name.startswith("k_composite_ts<false")
    if kernel == "project":
        return name.startswith("k_project<")
    raise KeyError(kernel)


def pmc_valu(kernel):
    """VALU wave instructions per frame of `kernel` from the committed PMC profile (SQ_INSTS_VALU)."""
    prof = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc.json")) \
        if os.path.isdir(os.path.join(ROOT, "profiles")) else []
    if not prof:
        return None
    d = json.load(open(os.path.join(ROOT, "profiles", prof[-1])))
    tot = sum(e.get("SQ_INSTS_VALU", 0.0) for lab, e in d.items() if _is_kernel(lab, kernel))
    return tot or None


def pmc_frame():
    """HBM bytes of one whole frame (every kernel launch of a steady-state frame, FETCH_SIZE x2 +
    WRITE_SIZE) and the serialised kernel time, from the committed PMC profile of this bench command."""
    prof = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc.json")) \
        if os.path.isdir(os.path.join(ROOT, "profiles")) else []
    if not prof:
        return None
    d = json.load(open(os.path.join(ROOT, "profiles", prof[-1])))
    b = sum(e.get("traffic_bytes", 0.0) for e in d.values())
    us = sum(e.get("mean_us", 0.0) for e in d.values())
    return {"bytes": int(b), "kernel_us_serialised": round(us, 1), "source": prof[-1]} if b else None


def frame_bytes(n, n_vis, k, W, H):
    """B = 236 N + 148 N_vis + 48 K + 16 W H."""
    return 236 * n + 148 * n_vis + 48 * k + 16 * W * H


def cpu_baseline(aos, n, W, H, u, budget_s=10.0, max_frames=10):
    """The oracle (CPU restatement of the reference semantics) on the same frame, host cores:
    full frames until about `budget_s` of CPU wall time (at most max_frames), the median frame."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as orc
    times = []
    t_all = time.perf_counter()
    while len(times) < max_frames and (not times or time.perf_counter() - t_all < budget_s):
        t0 = time.perf_counter()
        orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    return {"value": n / dt / 1e6, "unit": "Msplats/s", "cores": orc.num_threads(), "kind": "port",
            "sample": "median of %d full frames of the same %d-Gaussian %dx%d workload (project, stable sort, "
                      "composite; %.2f s per frame, %.1f s total)" % (len(times), n, W, H, dt,
                                                                       time.perf_counter() - t_all)}


def node_fps(n, seed, W, H, frames=300):
    """The Node drop-in's frame rate (tools/node_fps.js: the reference's Renderer frame loop through
    the N-API addon, same scene and camera; device-resident frames and host readback), or None
    when node or the addon is absent."""
    import shutil
    import subprocess
    addon_path = os.path.join(ROOT, "gaussian-splatting-web_amd", "lib", "gsplat_napi.node")
    if not shutil.which("node") or not os.path.exists(addon_path):
        return None
    try:
        r = subprocess.run(["node", os.path.join(ROOT, "tools", "node_fps.js"), str(n), str(seed), str(W), str(H),
                            str(frames)], capture_output=True, text=True, timeout=180)
        if r.returncode != 0:
            return {"error": r.stderr[-300:]}
        d = json.loads(r.stdout.strip().splitlines()[-1])
        return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}
    except (subprocess.TimeoutExpired, ValueError) as e:
        return {"error": str(e)[:300]}


def orbit_uniforms(W, H, k, period=60):
    """The orbit loop's camera (gsplat_amd.orbit_uniforms: yaw +-25 deg, pitch +-8 deg)."""
    return gs.orbit_uniforms(W, H, k, period)


def spawn_ranks(n, cmd=None):
    """torch.distributed.run's job, for `python bench.py --gpus N`: N rank processes on this node
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), started before this process touches a GPU; rank
    0's JSON line is the output.  Returns the exit status (the worst rank's)."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i]: 3 = 6.1 M at 1080p (default), 4 = 50 M at 4K")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--prewarm", type=float, default=0.2,
                    help="seconds of untimed frames before the --warmup frames (the GPU's clocks and the "
                         "scene's first frames after its upload settle; 0: none)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the latency / orbit / stage loops")
    ap.add_argument("--list-split", type=int, default=0, choices=(0, 1),
                    help="gs_opts.list_split: one serial chain per tile (0, default: bit-identical across "
                         "chunk splits, strips and groups) or long tile lists of frames with few tiles over "
                         "several wave pairs (1)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    N0, W0, H0, S0 = CONFIGS[args.config]
    N = args.n or N0
    W, H = args.width or W0, args.height or H0
    seed = args.seed if args.seed is not None else S0

    # torch.distributed.run (or spawn_ranks): RCCL all-gather of the strips at N > 1; a single rank
    # renders the whole image, and gathers nothing
    launched = "WORLD_SIZE" in os.environ
    dist = None
    if launched:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    aos = gs.synth_aos(N, seed, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(local_rank)
    scene = gs.Scene(ctx, aos, N, 16)

    row0, rows_padded, t0, t1 = strip_geometry(H, rank, world)
    # output RGBA f16: the reference's framebuffer format (rgba16float, src/simple_render.ts:499-505);
    # accumulation stays fp32 (gs_opts.accum), rounded once at the store
    # timed loop: HIP events around the composite only (timing=2; an event record costs the stream a
    # few microseconds); a separate shorter loop with events between every stage (timing=1) gives
    # the stage breakdown
    opts_head = gs.make_opts(strip_index=rank, strip_count=world, list_split=args.list_split, timing=2, out_format=gs.GS_OUT_RGBA_F16)
    opts_stage = gs.make_opts(strip_index=rank, strip_count=world, list_split=args.list_split, timing=1, out_format=gs.GS_OUT_RGBA_F16)
    cur = {"opts": opts_head}
    strip_bytes = rows_padded * W * 8
    if launched:
        import torch
        from gsplat_amd.strips import StripPipeline
        # a stream of our own for the frames: the default stream's handle is 0, which the C ABI
        # reads as "the context's stream", and the strip pipeline's events must be recorded on the
        # stream the frame's composite actually ran on
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        pipe = StripPipeline(rows_padded, W, dtype=torch.float16)  # gather t beside render t+1

        def frame_u(uu, sc=None):
            strip = pipe.next_strip()
            (sc or scene).render_device(uu, W, H, strip.data_ptr(), strip_bytes, stream.cuda_stream, cur["opts"])
            pipe.submit()

        def frame():
            frame_u(u)

        def sync():
            pipe.finish()
            torch.cuda.synchronize()
            dist.barrier()
    else:
        buf = gs.DeviceBuffer(H * W * 8)

        def frame_u(uu, sc=None):
            (sc or scene).render_device(uu, W, H, buf.ptr.value, buf.nbytes, None, cur["opts"])

        def frame():
            frame_u(u)

        def sync():
            ctx.sync()

    # untimed: at least `prewarm` seconds of frames, then the W warmup frames (20 timed frames right
    # after the scene's upload and 5 warmup frames ran ~5 % below the steady rate:
    # tools/r05/benchsteps.sh)
    n_prewarm = 0
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < args.prewarm:
        frame()
        n_prewarm += 1
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
    extra = {}
    if not args.no_extra:
        # median single-frame time of 50 frames (each frame waited for, no overlap)
        cur["opts"] = gs.make_opts(strip_index=rank, strip_count=world, list_split=args.list_split, out_format=gs.GS_OUT_RGBA_F16)
        lat = []
        for _ in range(50):
            t0 = time.perf_counter()
            frame()
            sync()
            lat.append(time.perf_counter() - t0)
        extra["latency_ms_median"] = round(float(np.median(lat)) * 1e3, 4)
        # a moving camera: a new view every frame (frames in flight, like the headline loop)
        uo = [orbit_uniforms(W, H, k) for k in range(args.steps)]
        for k in range(args.warmup):
            frame_u(uo[k % len(uo)])
        sync()
        t0 = time.perf_counter()
        for k in range(args.steps):
            frame_u(uo[k])
        sync()
        el = time.perf_counter() - t0
        st_o = ctx.timings()
        if launched and world > 1:  # the slowest rank's times
            import torch
            tt = torch.tensor([el, extra["latency_ms_median"]], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el, extra["latency_ms_median"] = float(tt[0]), round(float(tt[1]), 4)
        extra["orbit"] = {"fps": round(args.steps / el, 2), "ms_per_step": round(el / args.steps * 1e3, 4),
                          "value_msplats": round(N * args.steps / el / 1e6, 3),
                          "tiles_unsaturated_last": st_o["tiles_unsaturated"], "k_chunk1_last": st_o["k_chunk1"],
                          "camera": "origin, yaw +-25 deg, pitch +-8 deg, period 60 frames"}
        # camera cuts: every frame a view far from the last one (gsplat_amd.COLD_VIEWS, a cycle of
        # 4), so no frame has saturation history from its own view: the chunk controller's cold path
        uc = [gs.cold_uniforms(W, H, k) for k in range(len(gs.COLD_VIEWS))]
        for k in range(args.warmup):
            frame_u(uc[k % len(uc)])
        sync()
        ctx.timings_reset()
        t0 = time.perf_counter()
        for k in range(args.steps):
            frame_u(uc[k % len(uc)])
        sync()
        el_c = time.perf_counter() - t0
        st_c = ctx.timings()
        lat_c = []
        for k in range(2 * len(uc)):  # each frame waited for: the worst single cold frame
            t0 = time.perf_counter()
            frame_u(uc[k % len(uc)])
            sync()
            lat_c.append(time.perf_counter() - t0)
        worst_c = max(lat_c)
        if launched and world > 1:
            import torch
            tt = torch.tensor([el_c, worst_c], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el_c, worst_c = float(tt[0]), float(tt[1])
        extra["cold"] = {"fps": round(args.steps / el_c, 2), "ms_per_step": round(el_c / args.steps * 1e3, 4),
                         "value_msplats": round(N * args.steps / el_c / 1e6, 3),
                         "worst_frame_ms": round(worst_c * 1e3, 4),
                         "median_frame_ms": round(float(np.median(lat_c)) * 1e3, 4),
                         "frames_cold": st_c["frames_seeded"], "frames": st_c["frames_rendered"],
                         "camera": "a cut every frame: cycle of %d views (gsplat_amd.COLD_VIEWS)" % len(uc)}
        # a scene whose tiles do not saturate (opacity logit ~ N(-4, 2)): every frame renders all
        # its visible splats as one chunk, as the reference renders every frame (src/renderer.ts:311-318)
        cur["opts"] = opts_head
        sparse = gs.Scene(ctx, gs.synth_aos_sparse(N, seed, W, H), N, 16)
        for _ in range(args.warmup):
            frame_u(u, sparse)
        sync()
        ctx.timings_reset()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            frame_u(u, sparse)
        sync()
        el_s = time.perf_counter() - t0
        st_s = ctx.timings()
        sat_frac = None
        if not launched:  # 16x16 tiles whose every pixel reached alpha = 1 (f16) in the last frame
            img = buf.to_host(np.empty((H, W, 4), np.float16))[:H // 16 * 16, :W // 16 * 16, 3]
            sat_frac = round(float((img.reshape(H // 16, 16, W // 16, 16) == 1.0).all(axis=(1, 3)).mean()), 4)
        if launched and world > 1:
            import torch
            tt = torch.tensor([el_s], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el_s = float(tt[0])
        extra["sparse"] = {"fps": round(args.steps / el_s, 2), "ms_per_step": round(el_s / args.steps * 1e3, 4),
                           "value_msplats": round(N * args.steps / el_s / 1e6, 3),
                           "n_vis": st_s["n_vis"], "k_binned": st_s["k_entries"],
                           "tiles_saturated_frac": sat_frac, "chunk_fraction": round(st_s["chunk_fraction"], 4),
                           "frames_chunked": st_s["frames_chunked"], "frames": st_s["frames_rendered"],
                           "ms_composite": round(st_s["ms_composite"], 4),
                           "scene": "SURVEY 8d generator, seed %d, opacity logit shifted by -%g (~N(-4,2))" % (
                               seed, gs.SPARSE_LOGIT_SHIFT)}
        sparse.close()
    # one untimed one-chunk frame for the exact visible count and K of SURVEY 8d's byte model
    # (with a chunk split the pipeline never projects the splats past it)
    cur["opts"] = gs.make_opts(strip_index=rank, strip_count=world, list_split=args.list_split, chunk_fraction=1.0,
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
    # (the per-tile sort ran inside the composite when its own stage is only the events' gap: a
    # separate sort takes >= 19 us at this size)
    sorts_in_composite = st["ms_tile_sort"] < 0.010
    a_bytes = algorithmic_bytes(dom, N, ex["n_vis"], st["k_entries"], W, rows_here,
                                n_chunk0=int(round(st["chunk_fraction"] * st["n_vis"])), sorts=sorts_in_composite)
    achieved = a_bytes / (stages[dom] * 1e-3) / 1e9
    # the committed PMC profile is of the default command (configs[3] on one GPU): its counters
    # only describe that workload
    profiled = world == 1 and args.config == 3 and (N, W, H) == (N0, W0, H0)
    traffic, traffic_src = pmc_traffic(dom) if profiled else (None, None)
    valu = pmc_valu(dom) if profiled else None
    fb = frame_bytes(N, n_vis_all, k_all, W, H)

    if rank == 0:
        out = {
            "metric": "Msplats/s at %dx%d, %s Gaussians (%s)" % (
                W, H, "%.1f M" % (N / 1e6), "synthetic bicycle stand-in" if args.config == 3 else "synthetic"),
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
            "data": "synthetic (SURVEY §8d generator, splitmix64 seed %d%s); "
                    "output RGBA f16 (the reference's rgba16float framebuffer)" % (
                        seed, "; bicycle PLY absent" if args.config == 3 else ""),
            "config": {"workload": "configs[%d]: %d Gaussians (SH deg 3) at %dx%d, lookAt([0,0,0],[0,0,-1]) "
                                   "perspective(60deg,W/H,0.03,1000)" % (args.config, N, W, H),
                       "n_gaussians": N, "width": W, "height": H, "list_split": args.list_split,
                       "prewarm": {"seconds": args.prewarm, "frames": n_prewarm},
                       "parallelism": "row-strips x%d + all-gather" % world if world > 1 else "single GPU"},
            # per-stage HIP-event times from the separate timing=1 loop (events between stages add
            # ~20 us to its frame), except ms_composite, timed live in the headline loop:
            # project = partition cull + cull + projection/colour, bin = count + scans + emission,
            # tile_sort = per-tile sort (a still camera: inside the composite's launch, this stage
            # then only the events' gap), chunk1 = the chunk-1 launch (returns at once when chunk 0
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
                         # (PMC counters cannot run inside the timed loop: the traffic figure is
                         # read from the committed profile of this same command, not this run)
                         "traffic_source": ("committed profile profiles/%s" % traffic_src) if traffic_src else None,
                         "algorithmic_bytes_per_launch": int(a_bytes),
                         "includes_tile_sort": bool(sorts_in_composite and dom == "composite"),
                         "per": "frame (the kernel's launches in one frame, HIP events on the render stream)"},
            # the dominant kernel's real bound: VALU issue (PMC instruction count of this command's
            # committed profile / the live event-timed duration)
            "valu_roofline": ({"kernel": dom, "insts_per_launch": int(valu),
                               "achieved": round(valu / (stages[dom] * 1e-3) / 1e9, 1),
                               "peak": VALU_PEAK / 1e9, "unit": "G wave-instr/s",
                               "frac": round(valu / (stages[dom] * 1e-3) / VALU_PEAK, 4),
                               "source": "committed profile profiles/%s (instruction count); "
                                         "duration live" % traffic_src} if valu else None),
            # SURVEY §8d's byte MODEL priced at the measured frame time.  Not bytes this design moves
            # (whole partitions past the chunk threshold cost 32 B, K is replaced by the chunk-0
            # entries; the measured bytes are frame_traffic), so its ratios can exceed 1 and are not
            # a roofline
            "survey_byte_model": {"bytes": int(fb),
                                  "model_bytes_frac": round(fb / (ms * 1e-3) / (world * HBM_PEAK), 4),
                                  "compulsory_model_bytes_frac": round((236 * N + 16 * W * H) / (ms * 1e-3) / (world * HBM_PEAK), 4),
                                  "formula": "236N + 148N_vis + 48K + 16WH (SURVEY 8d)"},
            # measured: the PMC bytes of every kernel of one frame over the live frame time
            "frame_traffic": None,
            "cpu_baseline": None,
        }
        pf = pmc_frame() if profiled else None
        if pf:
            pf["frac"] = round(pf["bytes"] / (ms * 1e-3) / HBM_PEAK, 4)
            pf["achieved_GBs"] = round(pf["bytes"] / (ms * 1e-3) / 1e9, 1)
            out["frame_traffic"] = pf
        out.update(extra)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(aos, N, W, H, u)

    scene.close()
    ctx.close()
    if rank == 0:
        if world == 1 and not args.no_extra and args.config == 3:
            out["node_fps"] = node_fps(N, seed, W, H)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
