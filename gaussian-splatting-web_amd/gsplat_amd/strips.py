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


def assemble(full, H):
    """Crop the gathered buffer to the H image rows."""
    return full[:H]


def padded_rows_total(H, count):
    return strip_geometry(H, 0, count)[1] * count


__all__ = ["strip_geometry", "gather_strips", "assemble", "padded_rows_total"]
