"""N>1 path on CPU: row strips + one all-gather (gloo, world_size 2 and 3), checked against the
single-image render.  Each rank's strip renderer here is the oracle (no GPU in this container);
the partitioning and the collective are the code bench.py runs over RCCL."""
import json
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gaussian-splatting-web_amd"), os.path.join(root, "tests")]
    import gsplat_amd as gs
    import oracle_py as orc
    from gsplat_amd.strips import StripPipeline, assemble, gather_strips, strip_geometry
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 4000
    aos = gs.synth_aos(n, 17, W, H)
    u = gs.bench_uniforms(W, H)
    img, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H)
    row0, rows_padded, t0, t1 = strip_geometry(H, rank, world)
    strip = torch.zeros((rows_padded, W, 4), dtype=torch.float32)
    rows = max(0, min(t1 * 16, H) - row0)
    strip[:rows] = torch.from_numpy(img[row0:row0 + rows])
    full = gather_strips(strip)
    out = assemble(full, H).numpy()
    # the double-buffered pipeline bench.py uses (synchronous on CPU tensors), two frames
    pipe = StripPipeline(rows_padded, W, dtype=torch.float32, device="cpu")
    ok_pipe = True
    for _ in range(3):
        buf = pipe.next_strip()
        buf.zero_()
        buf[:rows] = torch.from_numpy(img[row0:row0 + rows])
        f = pipe.submit()
        pipe.finish()
        ok_pipe = ok_pipe and np.array_equal(assemble(f, H).numpy(), img)
    # K-balanced uneven strips: costs all-gathered, the same boundaries on every rank, the strips
    # (explicit tile rows, padded to a common height for the all-gather) assemble to the image
    from gsplat_amd.strips import assemble_uneven, balanced_bounds, even_bounds
    bounds = even_bounds(H, world)
    tr = (H + 15) // 16
    ok_bal = True
    for _ in range(4):
        mine = float((rank + 1) ** 3 * (bounds[rank + 1] - bounds[rank]))  # rank-dependent density
        nb = balanced_bounds(bounds, mine)
        chk = [torch.zeros(world + 1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(chk, torch.tensor(nb, dtype=torch.int64))
        ok_bal = ok_bal and all(c.tolist() == nb for c in chk) and nb[0] == 0 and nb[-1] == tr
        bounds = nb
    cap = 16 * max(b - a for a, b in zip(bounds[:-1], bounds[1:]))
    s = torch.zeros((cap, W, 4), dtype=torch.float32)
    r0, r1 = 16 * bounds[rank], min(16 * bounds[rank + 1], H)
    s[:r1 - r0] = torch.from_numpy(img[r0:r1])
    full = torch.zeros((world * cap, W, 4), dtype=torch.float32)
    dist.all_gather_into_tensor(full, s)
    ok_bal = ok_bal and np.array_equal(assemble_uneven(full, bounds, cap, H).numpy(), img)
    if 1 < world < tr:
        ok_bal = ok_bal and bounds != even_bounds(H, world)  # the costly last ranks' strips shrank
    if rank == 0:
        q.put(bool(np.array_equal(out, img)) and ok_pipe and ok_bal)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,size", [(1, (96, 50)), (2, (160, 120)), (3, (100, 37))])
def test_strip_allgather_gloo(world, size):
    W, H = size
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_bench_spawns_ranks(tmp_path):
    """`python bench.py --gpus N` without torch.distributed.run starts N rank processes with the
    launcher's environment (distinct RANK/LOCAL_RANK, one WORLD_SIZE, one 127.0.0.1 rendezvous) and
    returns the worst exit status."""
    import bench
    probe = ("import json, os, sys; json.dump({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', "
             "'MASTER_ADDR', 'MASTER_PORT')}, open(os.path.join(%r, 'r' + os.environ['RANK']), 'w')); "
             "sys.exit(int(os.environ['RANK']) == 2)" % str(tmp_path))
    rc = bench.spawn_ranks(4, [sys.executable, "-c", probe])
    assert rc == 1
    envs = [json.load(open(tmp_path / ("r%d" % r))) for r in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"] == [e["LOCAL_RANK"] for e in envs]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"} and {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert bench.spawn_ranks(2, [sys.executable, "-c", "pass"]) == 0
