#!/usr/bin/env python3
"""Asynchronous host path (DIRECT, staged, default config): 1/4/8/16 threads,
2 s per point, with whichever ix_amd/libixgrx.so is in place (GPU box)."""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import bench
    from ix_amd import traces
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    pool = traces.make_trace("tcp64", 1 << 16, seed=0x1BF000)
    f = os.path.join(tempfile.mkdtemp(), "frames.bin")
    bench.write_frames_file(pool, f)
    for rep in range(2):
        for t in (1, 4, 8, 16):
            r = bench._loop_run(f, "loop", 120, threads=t, seconds=2.0, batch=64, arena=1 << 17)
            print(json.dumps({"lib": tag, "rep": rep, "threads": t, "mpps": r.get("mpps"),
                              "lat_p50": r.get("latency_us", {}).get("p50"), "err": r.get("error")}), flush=True)


if __name__ == "__main__":
    main()
