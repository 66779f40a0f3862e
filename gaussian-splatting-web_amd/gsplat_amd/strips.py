"""Row-strip frame partitioning across ranks + the one framebuffer all-gather.

Rank g of G renders tile rows [g*ceil(TR/G), min((g+1)*ceil(TR/G), TR)) (TR = ceil(H/16)) into a
buffer of rows_padded = ceil(TR/G)*16 rows; one all_gather_into_tensor of those equal-size buffers
yields the image followed by padding rows.  Under backend "nccl" this is RCCL over xGMI.
The reference renders on one adapter (src/renderer.ts:301-330); this exchange is new.
"""
TILE = 16


def strip_geometry(H, index, count):
    """(first image row, rows_padded, first tile row, end tile row) of strip `index` of `count`."""
    tr = (H + TILE - 1) // TILE
    per = (tr + count - 1) // count
    t0 = min(index * per, tr)
    t1 = min((index + 1) * per, tr)
    return t0 * TILE, per * TILE, t0, t1


def gather_strips(strip, full=None, group=None):
    """All-gather equal-size strip buffers (torch tensors [rows_padded, W, C]) into `full`
    ([world*rows_padded, W, C]); returns `full`.  One collective per frame."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if full is None:
        full = torch.empty((world * strip.shape[0],) + tuple(strip.shape[1:]), dtype=strip.dtype,
                           device=strip.device)
    dist.all_gather_into_tensor(full, strip.contiguous(), group=group)
    return full


class StripPipeline:
    """Double-buffered strips: frame t's all-gather runs on a side stream while frame t+1 renders
    (SURVEY §8e).  Per frame: `strip = pipe.next_strip()`, render into it on the current stream,
    then `full = pipe.submit()` (the gathered image is ready once `finish()` or a later
    `next_strip()` for the same buffer has ordered the streams).  On CPU tensors (gloo) the
    gather is synchronous."""

    def __init__(self, rows_padded, W, channels=4, dtype=None, device=None, depth=2, group=None):
        import torch
        import torch.distributed as dist
        self.dist, self.group = dist, group
        world = dist.get_world_size(group)
        dtype = dtype or torch.float16
        device = torch.device(device or "cuda")
        self.strips = [torch.zeros((rows_padded, W, channels), dtype=dtype, device=device) for _ in range(depth)]
        # one rank: the strip is the whole image, nothing to gather
        self.single = world == 1
        self.fulls = self.strips if self.single else \
            [torch.zeros((world * rows_padded, W, channels), dtype=dtype, device=device) for _ in range(depth)]
        self.cuda = device.type == "cuda"
        if self.cuda:
            self.side = torch.cuda.Stream(device=device)
            self.rendered = [torch.cuda.Event() for _ in range(depth)]
            self.gathered = [torch.cuda.Event() for _ in range(depth)]
        self.k = 0

    def next_strip(self):
        """The buffer to render the next frame into (after its previous gather has finished)."""
        import torch
        b = self.k % len(self.strips)
        if self.cuda and not self.single and self.k >= len(self.strips):
            torch.cuda.current_stream().wait_event(self.gathered[b])
        return self.strips[b]

    def submit(self):
        """All-gather the strip just rendered into the current frame's full buffer; returns it."""
        import torch
        b = self.k % len(self.strips)
        if self.single:
            pass
        elif self.cuda:
            self.rendered[b].record(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                self.side.wait_event(self.rendered[b])
                self.dist.all_gather_into_tensor(self.fulls[b], self.strips[b], group=self.group)
                self.gathered[b].record(self.side)
        else:
            self.dist.all_gather_into_tensor(self.fulls[b], self.strips[b], group=self.group)
        self.k += 1
        return self.fulls[b]

    def finish(self):
        """Order every pending gather before the current stream's later work."""
        import torch
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.side)


def even_bounds(H, count):
    """Tile-row boundaries (count + 1) of the even split (floor(g * TR / count))."""
    tr = (H + TILE - 1) // TILE
    return [g * tr // count for g in range(count + 1)]


def balanced_bounds(bounds, local_cost, group=None, device=None):
    """K-balanced strips across ranks (SURVEY §8e "later"): every rank contributes its strip's
    cost (e.g. binned entries, gs_stats k_entries, plus a per-tile term), one small all-gather
    gives every rank the same vector, and gs_balance_strips (deterministic host arithmetic) turns
    it into the same new boundaries on every rank.  Returns the new boundaries (a list)."""
    import torch
    import torch.distributed as dist
    import gsplat_amd as gs
    world = dist.get_world_size(group)
    mine = torch.tensor([float(local_cost)], dtype=torch.float64, device=device)
    allc = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allc, mine, group=group)
    cost = [float(c.item()) for c in allc]
    return [int(b) for b in gs.balance_strips(bounds, cost)]


def assemble_uneven(full, bounds, rows_cap, H):
    """The image from an all-gather of padded uneven strips: rank g's buffer (rows_cap rows) holds
    tile rows [bounds[g], bounds[g+1])."""
    import torch
    parts = []
    for g in range(len(bounds) - 1):
        rows = max(0, min(bounds[g + 1] * TILE, H) - bounds[g] * TILE)
        parts.append(full[g * rows_cap:g * rows_cap + rows])
    return torch.cat(parts, 0)


def assemble(full, H):
    """Crop the gathered buffer to the H image rows."""
    return full[:H]


def padded_rows_total(H, count):
    return strip_geometry(H, 0, count)[1] * count


__all__ = ["strip_geometry", "gather_strips", "StripPipeline", "assemble", "padded_rows_total", "even_bounds",
           "balanced_bounds", "assemble_uneven"]
