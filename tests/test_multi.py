"""N>1 path: byte-balanced sharding, per-rank processing, record gather and
the max-over-ranks timing rule, with world_size 2 over gloo.
Each rank is a separate process (tests/multi_worker.py), as under torchrun."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from ix_amd import shard, traces

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, kind, n, engine, timeout=300, **extra):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IXT_KIND=kind, IXT_N=str(n), IXT_ENGINE=engine, **extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "multi_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0, out[-2000:]


@pytest.mark.parametrize("kind,n", [("imix", 3001), ("tcp64", 4096), ("mixed", 2000)])
def test_two_ranks_gloo(kind, n):
    _run(2, kind, n, "oracle")


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [("imix", 20001), ("mixed", 20000)])
def test_two_ranks_gloo_hip(kind, n):
    """Both ranks drive the HIP engine on the box's one GPU."""
    _run(2, kind, n, "hip")


@pytest.mark.parametrize("world,n", [(2, 512 * 6), (3, 512 * 4)])
def test_strong_split_gloo(world, n):
    """bench.py's C4 line (one batch on rank 0, split by shard_bounds,
    scattered, processed, records gathered) end to end over gloo; world 3
    gives unequal slices; transfers in 100 000-byte pieces (many per slice,
    the last one partial)."""
    _run(world, "strong", n, "oracle", IXT_P2P_MAX="100000")


@pytest.mark.gpu
def test_strong_split_gloo_hip():
    """The same leg with the HIP engine on the box's one GPU (two ranks
    sharing the card, device tensors staged through host memory by gloo)."""
    _run(2, "strong", 512 * 64, "hip")


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_bounds_balanced(world):
    tr = traces.make_trace("imix", 5000, seed=3)
    b = shard.shard_bounds(tr.len, world)
    assert b[0][0] == 0 and b[-1][1] == tr.n
    assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
    w = (tr.len.astype(np.int64) + 3) & ~3
    sizes = [int(w[s:e].sum()) for s, e in b]
    assert max(sizes) - min(sizes) <= 2 * 1516


def test_shard_bounds_small():
    assert shard.shard_bounds(np.zeros(0, np.uint16), 4) == [(0, 0)] * 4
    b = shard.shard_bounds(np.array([60], np.uint16), 2)
    assert sorted(e - s for s, e in b) == [0, 1]


def test_shard_trace_frames_identical():
    for kind in ("imix", "tcp64"):
        tr = traces.make_trace(kind, 777, seed=9)
        for s, e in shard.shard_bounds(tr.len, 3):
            part = shard.shard_trace(tr, s, e)
            assert part.n == e - s
            for i in (0, part.n // 2, part.n - 1):
                assert part.frame(i) == tr.frame(s + i)
            assert part.blob.shape[0] >= int(part.offsets()[-1]) + int(part.len[-1]) + traces.TAIL_PAD


def test_p2p_pieces_cover_in_order():
    """Transfers split into <= P2P_MAX_BYTES views that tile the tensor in
    order, the same way on both ends."""
    import torch
    t = torch.arange(10 * 16, dtype=torch.uint8).view(10, 16)
    ps = shard._pieces(t, 48)
    assert [p.shape[0] for p in ps] == [3, 3, 3, 1]
    assert torch.equal(torch.cat(ps), t)
    b = torch.arange(100, dtype=torch.uint8)
    assert [p.numel() for p in shard._pieces(b, 30)] == [30, 30, 30, 10]
    assert len(shard._pieces(torch.empty(0, dtype=torch.uint8), 30)) == 0


@pytest.mark.gpu
def test_bench_two_ranks_parity_vs_oracle():
    """bench.py at N = 2 (two gloo ranks sharing the box's card, as the
    driver's N > 1 runs but without RCCL): rank 0 prints one JSON line whose
    every device line was checked against the oracle (parity_vs_oracle),
    including the records gathered back from rank 1 (c4_strong)."""
    import json
    port = _free_port()
    env = dict(os.environ, IXG_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(os.path.dirname(HERE), "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--frames", str(1 << 16), "--secondary", "", "--extra", "c5r",
           "--strong-n", str(1 << 16), "--no-copy", "--no-tx", "--no-demux", "--cpu-seconds", "0.5"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2
    par = d["parity_vs_oracle"]
    assert par["c2"] == "ok" and par["c2b"] == "ok" and par["c5r"] == "ok" and par["c4_strong"] == "ok", par
    assert d["c4_strong"]["slice_frames"][0] + d["c4_strong"]["slice_frames"][1] >= 1 << 16
