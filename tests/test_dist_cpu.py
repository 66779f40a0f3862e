"""N>1 path on CPU: row strips + one all-gather (gloo, world_size 2 and 3), checked against the
single-image render.  Each rank's strip renderer here is the oracle (no GPU in this container);
the partitioning and the collective are the code bench.py runs over RCCL."""
import os
import socket

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
    if rank == 0:
        q.put(bool(np.array_equal(out, img)) and ok_pipe)
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
