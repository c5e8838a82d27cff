"""Splitting one RX batch across GPUs.

Frames are independent: there is no cross-packet state on this path, so a
batch splits into contiguous index slices, one per rank (one process per
GPU). Slice boundaries follow the cumulative frame bytes, so each rank gets
about 1/N of the bytes, which matters for IMIX and mixed traces where frame
sizes vary 25x. Each rank copies its own slice host->device (the batch lives
in host memory, as in IX) and runs ``ixg_rx_batch_*`` on it; nothing crosses
xGMI on the data path. Records come back in input order through
``gather_records``: an all-gather of fixed-size 16-byte records.

When the batch instead starts in one GPU's HBM (SURVEY.md 8(e) option 1),
``scatter_slices`` / ``gather_slices`` move equal-sized slices out and the
records back over xGMI with one RCCL scatter and one gather.
"""
from __future__ import annotations

import numpy as np

from .traces import TAIL_PAD, Trace


def shard_bounds(lens: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [start, end) frame slices, one per rank, balanced by
    cumulative frame bytes (each frame counted at its 4-aligned size)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = int(lens.shape[0])
    w = (lens.astype(np.int64) + 3) & ~3
    cum = np.cumsum(w)
    total = int(cum[-1]) if n else 0
    cuts = [0]
    for r in range(1, world):
        # first frame whose cumulative end passes r/world of the bytes
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")) + (1 if n else 0))
    cuts.append(n)
    cuts = np.minimum(np.maximum.accumulate(np.array(cuts)), n).tolist()
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_trace(tr: Trace, start: int, end: int) -> Trace:
    """Frames [start, end) of `tr` as a self-contained trace: its own blob
    (with the tail pad the device API requires) and rebased offsets."""
    if end <= start:
        return Trace(np.zeros(TAIL_PAD, np.uint8), None, np.zeros(0, np.uint16), 4)
    lens = tr.len[start:end].copy()
    if tr.off is None:
        S = tr.stride
        blob = np.zeros((end - start) * S + TAIL_PAD, np.uint8)
        blob[:(end - start) * S] = tr.blob[start * S:end * S]
        return Trace(blob, None, lens, S)
    offs = tr.off[start:end].astype(np.uint64)
    lo = int(offs.min())
    hi = int((offs + ((lens.astype(np.uint64) + 3) & ~np.uint64(3))).max())
    blob = np.zeros(hi - lo + TAIL_PAD, np.uint8)
    blob[:hi - lo] = tr.blob[lo:hi]
    return Trace(blob, offs - np.uint64(lo), lens, 0)


def gather_records(rec: np.ndarray, bounds: list[tuple[int, int]], dist, device="cpu"):
    """All ranks' records in input order (every rank gets the full array).
    `rec`: this rank's [m, 16] uint8 records (m = its slice length)."""
    import torch
    world = len(bounds)
    m = max(e - s for s, e in bounds)
    buf = torch.zeros((m, 16), dtype=torch.uint8, device=device)
    mine = torch.from_numpy(np.ascontiguousarray(rec).reshape(-1, 16))
    buf[:mine.shape[0]] = mine.to(device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return np.concatenate([parts[r][:e - s].cpu().numpy() for r, (s, e) in enumerate(bounds)], axis=0)


def scatter_slices(full, out, dist, src: int = 0) -> None:
    """Option 1 of SURVEY.md 8(e): the batch sits on rank `src`'s GPU and its
    slices travel to the other GPUs over xGMI (one RCCL scatter; torch's
    backend "nccl" is RCCL on ROCm). `full`: the src rank's flat tensor of
    world * m elements (None on the other ranks); `out`: every rank's
    m-element slice. Slices are equal-sized: pad the batch to world * m."""
    world = dist.get_world_size()
    if dist.get_rank() == src:
        if full.numel() != world * out.numel():
            raise ValueError("full must hold world * out.numel() elements")
        dist.scatter(out, scatter_list=list(full.view(world, -1).unbind(0)), src=src)
    else:
        dist.scatter(out, src=src)


def gather_slices(part, dist, dst: int = 0):
    """The reverse: every rank's equal-sized `part` (e.g. its [m, 16]
    records) into one [world * m, ...] tensor on rank `dst` (None elsewhere),
    in rank order, over one RCCL gather."""
    import torch
    world = dist.get_world_size()
    if dist.get_rank() == dst:
        full = torch.empty((world,) + tuple(part.shape), dtype=part.dtype, device=part.device)
        dist.gather(part, gather_list=list(full.unbind(0)), dst=dst)
        return full.view((world * part.shape[0],) + tuple(part.shape[1:]))
    dist.gather(part, dst=dst)
    return None


def max_over_ranks(x: float, dist, device="cpu") -> float:
    """The slowest rank's value (bench.py's timing rule)."""
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
