"""Multi-GPU sharding and the tuple gather (one process per GPU, torch.distributed).

Packets are independent — every `fast::parse_*` is a pure function of one packet's bytes
(src/parser/fast.rs) — so a batch shards by contiguous packet blocks with no exchange inside the
parse.  The only collective is the gather of the per-packet output columns to the root rank
(RCCL over xGMI with the "nccl" backend on GPUs; "gloo" works for CPU tensors in tests).
"""
import numpy as np

from . import schema


def shard_range(n, world, rank):
    """[lo, hi) of rank's contiguous block of n packets (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_fixed(slab, n, stride, world, rank, lens=None):
    """Fixed-stride shard: (slab view, n_local, lens view).  `slab` is a flat uint8 array or
    tensor; the view starts at a packet boundary."""
    lo, hi = shard_range(n, world, rank)
    view = slab[lo * stride:hi * stride]
    return view, hi - lo, (lens[lo:hi] if lens is not None else None), lo


def shard_indexed(offsets, lens, world, rank):
    """Indexed (pcap) shard by record index: (offsets, lens, first record index).  Offsets keep
    pointing into the full slab, so every rank may hold the whole file or its byte range."""
    lo, hi = shard_range(len(offsets), world, rank)
    return offsets[lo:hi], lens[lo:hi], lo


def pack_columns(res, columns):
    """Concatenate the columns of one shard into one flat uint8 tensor/array (the gather unit).
    Returns (flat, layout) with layout = [(name, shape, nbytes)]."""
    import torch
    parts, layout = [], []
    for c in columns:
        t = res[c]
        if isinstance(t, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(t))
        flat = t.contiguous().view(torch.uint8).reshape(-1)
        parts.append(flat)
        layout.append((c, tuple(t.shape), flat.numel()))
    return torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8), layout


def unpack_columns(flat, layout):
    import torch
    out, o = {}, 0
    for c, shp, nb in layout:
        dt = schema.column_dtype(c)
        out[c] = flat[o:o + nb].cpu().numpy().view(dt).reshape(shp)
        o += nb
    return out


def gather_columns(res, columns, n_local, dst=0, group=None):
    """Gather every rank's columns to `dst` and reassemble them in global packet order.
    Slot-major columns ([MAX_HDRS][n]) are concatenated along the packet axis.  Returns the
    merged {column: numpy} on dst, None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    flat, layout = pack_columns(res, columns)
    dev = flat.device
    sizes = torch.tensor([flat.numel(), n_local], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    maxb = int(max(s[0].item() for s in all_sizes))
    buf = torch.zeros(maxb, dtype=torch.uint8, device=dev)
    buf[:flat.numel()] = flat
    glist = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, glist, dst=dst, group=group)
    if rank != dst:
        return None
    merged = {}
    for r in range(world):
        nb, nl = int(all_sizes[r][0].item()), int(all_sizes[r][1].item())
        lay = []
        for c, shp, _ in layout:
            shp_r = schema.column_shape(c, nl)
            lay.append((c, shp_r, int(np.prod(shp_r)) * schema.column_dtype(c).itemsize))
        part = unpack_columns(glist[r][:nb], lay)
        for c in columns:
            merged.setdefault(c, []).append(part[c])
    for c in columns:
        axis = 1 if schema.column_shape(c, 1)[0] == schema.MAX_HDRS and c in ("hdr_type", "hdr_off") else 0
        merged[c] = np.concatenate(merged[c], axis=axis)
    return merged
