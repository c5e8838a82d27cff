"""Same-process A/B of the synchronous mbuf path (bench.py's mbuf_path: 2M C2
frames in IX mbufs -> ixg_rx_batch_mbufs, one host thread) over library
builds: ab_mbuf.py LIB1+LIB2+... [ROUNDS]."""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)


def main():
    import bench
    from ix_amd import ixgrx, traces
    libs = sys.argv[1].replace("+", ",").split(",")
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    engs = {lib: ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY), lib_path=os.path.join(ROOT, lib)) for lib in libs}
    res = {os.path.basename(lib): [] for lib in libs}
    for _ in range(rounds):
        for lib, e in engs.items():
            line, _ = bench.mbuf_path(e, 1 << 21, seed=0x1BF000)
            res[os.path.basename(lib)].append(line["mpps"])
    print(json.dumps({k: {"max_mpps": max(v), "mpps": v} for k, v in res.items()}))


if __name__ == "__main__":
    main()
