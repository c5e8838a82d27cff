"""Host-path probe (VERDICT r3 Next #5): the IX loop example's per-thread
breakdown at 1/4/16 threads, staged and zero copy, over C2's 60-B frames and
over 1514-B frames, plus a batch-size sweep of the staged loop. One JSON
object per run on stdout; the summary at the end.

usage: python3 tools/dbg/host_probe.py [seconds]
"""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import bench  # noqa: E402
from ix_amd import traces  # noqa: E402

sec = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
tmp = tempfile.mkdtemp(prefix="ixg_probe_")
files = {}
for kind in ("tcp64", "imix", "tcp1514"):
    p = os.path.join(tmp, kind + ".bin")
    bench.write_frames_file(traces.make_trace(kind, 1 << 14 if kind != "tcp64" else 1 << 16, seed=7), p)
    files[kind] = p

out = []


def run(kind, **kw):
    kw.setdefault("seconds", sec)
    kw.setdefault("batch", 64)
    kw.setdefault("arena", 1 << 17 if kind == "tcp64" else 1 << 15)
    r = bench._loop_run(files[kind], "loop", 300, **kw)
    r = {"trace": kind, "args": kw, **r}
    print(json.dumps(r), flush=True)
    out.append(r)


quick = len(sys.argv) > 2 and sys.argv[2] == "quick"
if len(sys.argv) > 2 and sys.argv[2] == "zc":  # staged vs registered, per frame size
    for kind in ("tcp64", "imix", "tcp1514"):
        for t in (1, 16):
            for reg in (0, 1):
                run(kind, threads=t, register=reg)
    sys.exit(0)
for kind in (("tcp64",) if quick else ("tcp64", "tcp1514")):
    for reg in ((0,) if quick else (0, 1)):
        for t in (1, 4, 16):
            run(kind, threads=t, register=reg)
# the staged loop at 16 threads with bigger device batches and deeper queues
for extra in (dict(cfg_wait_us=200),) if quick else (dict(cfg_depth=4), dict(cfg_wait_us=200), dict(cfg_frames=65536, cfg_bytes=16 << 20, cfg_depth=4),
              dict(direct=0)):
    run("tcp64", threads=16, **extra)
