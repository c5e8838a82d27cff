"""The RCCL branches of the C4 split (ix_amd/shard.py: scatter_frames,
gather_frame_records, max_over_ranks) on the CPU, with a stand-in for
torch.distributed whose backend reports "nccl" (VERDICT r3
"the nccl branches have never run"). The driver's 8-GPU run takes these
branches; the gloo tests (tests/test_multi.py) take the host-staged ones.

The stand-in records every point-to-point op and carries the bytes between
the simulated ranks in process, so the test checks both the call pattern
the RCCL path makes (one batch_isend_irecv group per rank per phase, one
piece list per peer, pieces of at most P2P_MAX_BYTES, no host staging: every
tensor handed to the library is a view of the caller's buffer) and the data
that arrives (each rank's slice; every record back in its rows on rank 0).
"""
import numpy as np
import pytest
import torch

from ix_amd import shard

TAIL_PAD = shard.TAIL_PAD


class _Op:
    def __init__(self, fn, tensor, peer):
        self.fn, self.tensor, self.peer = fn, tensor, peer


class _World:
    """In-process ranks: sends are queued per (src, dst) pair and matched, in
    order, by the receiver's recvs."""

    def __init__(self, n):
        self.n = n
        self.mail = {}
        self.groups = {r: [] for r in range(n)}
        self.reduced = []

    def dist(self, rank):
        return _Dist(self, rank)


class _Dist:
    P2POp = _Op

    class ReduceOp:
        MAX = "max"

    def __init__(self, world, rank):
        self.w, self.r = world, rank

    def get_backend(self):
        return "nccl"

    def get_rank(self):
        return self.r

    def get_world_size(self):
        return self.w.n

    def isend(self, t, peer):  # only ever wrapped in P2POp
        raise AssertionError("isend outside a group")

    def irecv(self, t, peer):
        raise AssertionError("irecv outside a group")

    def batch_isend_irecv(self, ops):
        self.w.groups[self.r].append(list(ops))
        for op in ops:
            key = (self.r, op.peer) if op.fn == self.isend else (op.peer, self.r)
            q = self.w.mail.setdefault(key, [])
            if op.fn == self.isend:
                q.append(op.tensor.clone())
            else:
                assert q, f"rank {self.r}: a recv from {op.peer} with nothing sent"
                src = q.pop(0)
                assert src.shape == op.tensor.shape and src.dtype == op.tensor.dtype
                op.tensor.copy_(src)

        class _W:
            def wait(self):
                pass
        return [_W() for _ in ops]

    def all_reduce(self, t, op=None):
        assert op == self.ReduceOp.MAX
        self.w.reduced.append(float(t.item()))


def _views_of(t, base):
    """t's storage is base's (a view, not a staged copy)."""
    return t.untyped_storage().data_ptr() == base.untyped_storage().data_ptr()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_scatter_gather_nccl_pattern(world, monkeypatch):
    monkeypatch.setattr(shard, "P2P_MAX_BYTES", 4096)  # many pieces per peer
    S, n = 96, 1000 + world
    rng = np.random.default_rng(world)
    lens_np = rng.integers(60, S + 1, n).astype(np.int16)
    blob = torch.from_numpy(rng.integers(0, 256, n * S + TAIL_PAD, dtype=np.uint8))
    lens = torch.from_numpy(lens_np)
    bounds = shard.shard_bounds(lens_np, world)
    w = _World(world)
    got = {}
    # rank 0 posts its sends first, then every receiver its recvs
    for r in range(world):
        d = w.dist(r)
        got[r] = shard.scatter_frames(blob if r == 0 else None, lens if r == 0 else None, S, bounds, d, "cpu")
    for r in range(world):
        groups = w.groups[r]
        assert len(groups) == (1 if r == 0 or bounds[r][1] > bounds[r][0] else 0), f"rank {r}: {len(groups)} groups"
        a, b = bounds[r]
        fb, lb = got[r]
        assert torch.equal(fb[:(b - a) * S], blob[a * S:b * S]) and torch.equal(lb, lens[a:b])
        if r == 0:
            assert _views_of(fb, blob) and _views_of(lb, lens)
            ops = groups[0]
            peers = [op.peer for op in ops]
            assert sorted(set(peers)) == list(range(1, world))
            for p in range(1, world):
                mine = [op for op in ops if op.peer == p]
                pa, pb = bounds[p]
                want = -(-((pb - pa) * S) // 4096) + 1  # frame pieces + the lengths
                assert len(mine) == want, f"peer {p}: {len(mine)} ops, want {want}"
                assert all(op.fn == w.dist(0).isend or op.fn.__name__ == "isend" for op in mine)
                assert all(_views_of(op.tensor, blob) or _views_of(op.tensor, lens) for op in mine)
                assert all(op.tensor.numel() * op.tensor.element_size() <= 4096 for op in mine)
        else:
            assert fb.numel() == (b - a) * S + TAIL_PAD and bool((fb[(b - a) * S:] == 0).all())
            for op in groups[0]:
                assert op.peer == 0 and (_views_of(op.tensor, fb) or _views_of(op.tensor, lb))
    # records back: every rank's slice of a [n, 16] record array into rank 0's
    rec_full = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8))
    out = torch.zeros((n, 16), dtype=torch.uint8)
    w2 = _World(world)
    for r in list(range(1, world)) + [0]:  # senders first, then rank 0 receives
        a, b = bounds[r]
        rec = out[a:b] if r == 0 else rec_full[a:b].clone()
        if r == 0:
            out[a:b] = rec_full[a:b]
        res = shard.gather_frame_records(rec, bounds, w2.dist(r), out if r == 0 else None)
        assert (res is out) if r == 0 else res is None
        if r != 0:
            assert all(_views_of(op.tensor, rec) for g in w2.groups[r] for op in g)
    assert torch.equal(out, rec_full)
    for op in w2.groups[0][0]:
        assert _views_of(op.tensor, out)
    assert len(w2.groups[0]) == 1


def test_max_over_ranks_nccl_device():
    w = _World(2)
    assert shard.max_over_ranks(1.5, w.dist(1), device="cpu") == 1.5
    assert w.reduced == [1.5]
