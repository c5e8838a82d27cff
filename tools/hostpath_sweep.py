#!/usr/bin/env python3
"""Sweep the asynchronous host path's knobs with examples/ix_async_loop
(threads x batch_frames x depth x direct), 2 s per point; one JSON line per
point (GPU box)."""
import itertools
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import bench
    from ix_amd import traces
    pts = sys.argv[1] if len(sys.argv) > 1 else "default"
    pool = traces.make_trace("tcp64", 1 << 16, seed=0x1BF000)
    f = os.path.join(tempfile.mkdtemp(), "frames.bin")
    bench.write_frames_file(pool, f)
    grid = [(t, bf, dp, di) for t, bf, dp, di in itertools.product((1, 4, 8, 16), (4096, 16384), (2, 8), (0, 1))]
    for t, bf, dp, di in grid:
        r = bench._loop_run(f, "loop", 120, threads=t, seconds=2.0, batch=64, arena=1 << 16, cfg_frames=bf,
                            cfg_bytes=bf * 64, cfg_depth=dp, direct=di)
        print(json.dumps({"threads": t, "batch_frames": bf, "depth": dp, "direct": di,
                          "mpps": r.get("mpps"), "lat_p50": r.get("latency_us", {}).get("p50"),
                          "lat_p99": r.get("latency_us", {}).get("p99"), "err": r.get("error")}), flush=True)


if __name__ == "__main__":
    main()
