#!/usr/bin/env python3
"""Asynchronous host path (DIRECT, staged): depth 2 vs 3 (the default) and
16K vs 64K-frame batches at 1/4/8/16 threads, 2 s per point (GPU box)."""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import bench
    from ix_amd import traces
    pool = traces.make_trace("tcp64", 1 << 16, seed=0x1BF000)
    f = os.path.join(tempfile.mkdtemp(), "frames.bin")
    bench.write_frames_file(pool, f)
    for t in (1, 4, 8, 16):
        for depth in (2, 3, 4):
            for bf in (16384, 65536):
                r = bench._loop_run(f, "loop", 120, threads=t, seconds=2.0, batch=64, arena=1 << 17,
                                    cfg_frames=bf, cfg_bytes=bf * 128, cfg_depth=depth)
                print(json.dumps({"threads": t, "depth": depth, "batch_frames": bf, "mpps": r.get("mpps"),
                                  "lat_p50": r.get("latency_us", {}).get("p50"),
                                  "lat_p99": r.get("latency_us", {}).get("p99"), "err": r.get("error")}), flush=True)


if __name__ == "__main__":
    main()
