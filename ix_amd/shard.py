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
``scatter_frames`` / ``gather_frame_records`` move each rank's
``shard_bounds`` slice out and its records back over xGMI as grouped RCCL
send/recv (one pair per peer; slices may differ in size), and
``scatter_slices`` / ``gather_slices`` do the same for equal-sized slices
with one RCCL scatter and one gather. bench.py's C4 line is the first.
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


def _p2p(ops, dist) -> None:
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


# the largest single send/recv: a slice of C4's 64M-frame batch is 12.7 GB
# at N = 8; transfers go out as <= 1 GiB pieces in the same group (message
# counts stay far from 2^31 in every library on the path)
P2P_MAX_BYTES = 1 << 30


def _pieces(t, max_bytes: int | None = None):
    """`t` split along dim 0 into views of at most max_bytes (default
    P2P_MAX_BYTES; sender and receiver split same-shaped tensors
    identically)."""
    if max_bytes is None:
        max_bytes = P2P_MAX_BYTES
    row = t.element_size() * (int(np.prod(t.shape[1:])) if t.dim() > 1 else 1)
    step = max(1, max_bytes // row)
    return [t[k:k + step] for k in range(0, t.shape[0], step)]


def _host_staged(dist, t) -> bool:
    """gloo moves host tensors only: device tensors are staged through host
    memory (the CPU rehearsal of the split; RCCL sends HBM to HBM)."""
    return t is not None and t.is_cuda and dist.get_backend() != "nccl"


def scatter_frames(blob, lens, stride: int, bounds, dist, device, src: int = 0):
    """C4's split (SURVEY.md 8(e) option 1) for a fixed-stride batch: rank
    `src` holds the whole batch (`blob`: n * stride frame bytes + TAIL_PAD,
    `lens`: n int16 lengths; None on the other ranks) and every other rank r
    receives frames [s_r, e_r) of `bounds` (shard_bounds: unequal slices are
    fine). Grouped send/recv per peer, in pieces of at most P2P_MAX_BYTES
    (RCCL batches them into one group, so the slices leave GPU `src` over
    their own xGMI links at once).

    Returns this rank's (blob, lens) on `device`, ready for ixg_rx_batch_dev:
    on `src` they are views into the batch (the frames after the slice, or
    the batch's own tail pad, cover the TAIL_PAD the device API reads past
    the last frame); elsewhere fresh buffers with a zeroed tail pad. All
    ranks must call it; bracket it with a barrier when timing it."""
    import torch
    rank = dist.get_rank()
    s, e = bounds[rank]
    m = e - s
    P = dist.P2POp
    if rank == src:
        if blob.numel() < len(lens) * stride + TAIL_PAD or bounds[-1][1] != len(lens):
            raise ValueError("blob/lens do not hold the whole batch the bounds describe")
        ops = []
        for r, (a, b) in enumerate(bounds):
            if r == src or b <= a:
                continue
            fb, lb = blob[a * stride:b * stride], lens[a:b]
            if _host_staged(dist, fb):
                fb, lb = fb.cpu(), lb.cpu()
            ops += [P(dist.isend, x, r) for x in _pieces(fb)] + [P(dist.isend, lb, r)]
        _p2p(ops, dist)
        return blob[s * stride:], lens[s:e]
    out_blob = torch.zeros(m * stride + TAIL_PAD, dtype=torch.uint8, device=device)
    out_lens = torch.empty(m, dtype=torch.int16, device=device)
    if m:
        rb, rl = out_blob[:m * stride], out_lens
        staged = _host_staged(dist, rb)
        if staged:
            rb, rl = torch.empty(m * stride, dtype=torch.uint8), torch.empty(m, dtype=torch.int16)
        _p2p([P(dist.irecv, x, src) for x in _pieces(rb)] + [P(dist.irecv, rl, src)], dist)
        if staged:
            out_blob[:m * stride].copy_(rb)
            out_lens.copy_(rl)
    return out_blob, out_lens


def gather_frame_records(rec, bounds, dist, out=None, dst: int = 0):
    """The reverse of scatter_frames: every rank's [e_r - s_r, 16] records
    land in rows [s_r, e_r) of `out` ([n, 16] uint8 on rank `dst`; None
    elsewhere), one grouped send/recv per peer. On `dst`, `rec` may already
    be the view out[s:e] (the kernels wrote there): then nothing is copied.
    Returns `out` on dst, None elsewhere."""
    import torch
    rank = dist.get_rank()
    P = dist.P2POp
    if rank != dst:
        if rec.shape[0]:
            t = rec.cpu() if _host_staged(dist, rec) else rec
            _p2p([P(dist.isend, x, dst) for x in _pieces(t)], dist)
        return None
    s, e = bounds[rank]
    if e > s and rec.data_ptr() != out[s:e].data_ptr():
        out[s:e].copy_(rec)
    ops, staged = [], []
    for r, (a, b) in enumerate(bounds):
        if r == dst or b <= a:
            continue
        t = out[a:b]
        if _host_staged(dist, t):
            t = torch.empty((b - a, 16), dtype=torch.uint8)
            staged.append((a, b, t))
        ops += [P(dist.irecv, x, r) for x in _pieces(t)]
    _p2p(ops, dist)
    for a, b, t in staged:
        out[a:b].copy_(t)
    return out


def max_over_ranks(x: float, dist, device="cpu") -> float:
    """The slowest rank's value (bench.py's timing rule)."""
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
