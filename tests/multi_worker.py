"""One rank of tests/test_multi.py (launched as a subprocess per rank).

env: RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT, IXT_KIND, IXT_N,
IXT_ENGINE ("oracle": CPU stand-in for the per-rank device call, tests only;
"hip": the product engine on cuda:0).
Every rank checks the gathered records against the oracle over the whole
batch and exits 0 on success.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ix_amd import shard, traces  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    kind, n, eng = os.environ["IXT_KIND"], int(os.environ["IXT_N"]), os.environ["IXT_ENGINE"]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if kind == "strong":
        # small transfer pieces: every slice goes out as many sends
        shard.P2P_MAX_BYTES = int(os.environ.get("IXT_P2P_MAX", shard.P2P_MAX_BYTES))
        ok = strong(rank, world, n, eng)
        dist.barrier()
        dist.destroy_process_group()
        print(f"rank {rank}: strong split ok={ok}", flush=True)
        sys.exit(0 if ok else 1)
    flags = 2 if kind == "mixed" else 0
    tr = traces.make_trace(kind, n, seed=77, bad_ip=0.02, bad_l4=0.02)
    bounds = shard.shard_bounds(tr.len, world)
    s, e = bounds[rank]
    part = shard.shard_trace(tr, s, e)
    if eng == "hip":
        from ix_amd import ixgrx
        rec = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, flags), device=0).batch_trace(part)
        rec = rec.view(np.uint8).reshape(-1, 16)
    else:
        rec, _ = oracle.rx_trace(part, traces.RSS_KEY, flags=flags)
    allrec = shard.gather_records(rec, bounds, dist)
    exp, _ = oracle.rx_trace(tr, traces.RSS_KEY, flags=flags)
    ok = allrec.shape == exp.shape and bool((allrec == exp).all())
    # option 1: the batch on rank 0, slices scattered, records gathered back
    import torch
    m = 4096
    full = torch.arange(world * m, dtype=torch.int32) if rank == 0 else None
    mine = torch.empty(m, dtype=torch.int32)
    shard.scatter_slices(full, mine, dist)
    ok = ok and bool((mine == torch.arange(rank * m, (rank + 1) * m, dtype=torch.int32)).all())
    back = shard.gather_slices((mine * 2).view(-1, 4), dist)
    if rank == 0:
        ok = ok and bool((back.view(-1) == torch.arange(world * m, dtype=torch.int32) * 2).all())
    else:
        ok = ok and back is None
    slowest = shard.max_over_ranks(float(rank + 1), dist)
    ok = ok and slowest == float(world)
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: slice [{s},{e}) ok={ok}", flush=True)
    sys.exit(0 if ok else 1)


def strong(rank, world, n, eng):
    """bench.py's C4 strong-split leg end to end (bench.strong_leg): the
    batch on rank 0, shard_bounds slices sent with grouped send/recv, each
    rank processing its slice, the records gathered into rank 0's batch
    record array; rank 0 checks the whole array against the oracle."""
    import torch
    import bench
    from ix_amd import traces
    pool = 512
    if eng == "hip":
        from ix_amd import ixgrx
        dev = torch.device("cuda", 0)
        e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, 0), device=0)

        def run(blob, lens, S, m, out, stream):
            e.batch_dev(blob.data_ptr(), None, lens.data_ptr(), S, m, out.data_ptr(), None, stream)
    else:
        dev = torch.device("cpu")

        def run(blob, lens, S, m, out, stream):
            # CPU stand-in for the device call (tests only): the oracle over
            # exactly the slice buffers the scatter produced
            tr = traces.Trace(blob.numpy(), None, lens.numpy().view(np.uint16)[:m].copy(), S)
            rec, _ = oracle.rx_trace(tr, traces.RSS_KEY)
            out.copy_(torch.from_numpy(rec))
    res, chk = bench.strong_leg(dev, run, dist, world, rank, n_total=n, pool=pool, reps=2)
    ok = res["frames"] == n and res["kernel_ms"] >= 0
    if rank == 0:
        _, name, ptr, flags, first, tiled = chk
        exp, _ = oracle.rx_trace(ptr, traces.RSS_KEY, flags=flags)
        ok = ok and name == "c4_strong" and tiled and np.array_equal(first, exp) and res["parity"] != "MISMATCH"
        print(res, flush=True)
    return ok


if __name__ == "__main__":
    main()
