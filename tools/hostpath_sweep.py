#!/usr/bin/env python3
"""Sweep the asynchronous host path with examples/ix_async_loop on the GPU
box: one JSON line per point, with the run's cgroup CPU throttling
(cpu.stat nr_throttled / throttled_usec deltas: the box's quota is 16 CPUs).

  tools/hostpath_sweep.py SET [SECONDS]
  SET: grid     threads x batch_frames x depth x direct (C2 frames)
       threads  1/4/8/16 threads at the defaults (C2 frames)
       idle     16 threads, idle=wait vs idle=spin (C2 frames)
       big      1514-B frames at 16 threads, staged vs zero copy, batch_bytes
                4 MiB / 1 MiB / 512 KiB / 256 KiB
       bigbytes 1514-B frames at 16 threads, staged and zero copy, batch_bytes
                512 / 640 / 768 / 1024 KiB, three rounds
       pages    1514-B frames at 16 threads, staged and zero copy, mbuf arenas
                on 2 MB pages (the default, as IX's mempools) vs 4 KB pages
       hwq      16 threads, GPU_MAX_HW_QUEUES 4 / 8 / 16 (the process's hardware
                queues): C2 frames, and 1514-B frames staged / zero copy at
                1 MiB and 512 KiB batch_bytes
       depth    16 threads, idle=wait: depth 2/3/4 x max_wait_us 50/100
       abbig:L1,L2,..  as ab, over 1514-B frames: staged and zero copy at
                batch_bytes 1 MiB and 512 KiB
       tailab:L1,L2,..  the 16-thread tail: C2 frames staged and 1514-B frames
                zero copy, library builds interleaved over 3 rounds, with the
                worst batch's latency split and the cgroup throttling
       pin      the 16-thread tail with the threads pinned one per CPU at
                strides 0 (unpinned) / 8 / 2, C2 staged and 1514-B zero copy
       ab:L1,L2,..  (or L1+L2+..) 16 threads, idle=wait, library builds interleaved over 4
                rounds (each Li a directory holding a libixgrx.so, or
                "default"): same-box A/B of host-path library variants
"""
import itertools
import re
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f)}
    except OSError:
        return {}


def point(path, label, env=None, **kw):
    import bench
    s0 = cpu_stat()
    r = bench._loop_run(path, "loop", 120, env=env, batch=64, **kw)
    s1 = cpu_stat()
    b = r.get("breakdown", {})
    out = {**label, "mpps": r.get("mpps"), "lat": r.get("latency_us"), "max_launch_us": b.get("max_launch_us"),
           "max_loop_gap_us": b.get("max_loop_gap_us"), "frames_per_batch": b.get("frames_per_batch"),
           "refused_share": b.get("refused_share"), "staged_bytes_per_frame": r.get("staged_bytes_per_frame"),
           "arena_pages": r.get("cfg", {}).get("arena_pages"),
           "throttled": s1.get("nr_throttled", 0) - s0.get("nr_throttled", 0),
           "throttled_ms": (s1.get("throttled_usec", 0) - s0.get("throttled_usec", 0)) / 1e3,
           "worst_batch_us": r.get("worst_batch_us"), "err": r.get("error")}
    print(json.dumps(out), flush=True)


def main():
    import bench
    from ix_amd import traces
    which = sys.argv[1] if len(sys.argv) > 1 else "threads"
    sec = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    tmp = tempfile.mkdtemp()
    f = os.path.join(tmp, "frames.bin")
    bench.write_frames_file(traces.make_trace("tcp64", 1 << 16, seed=0x1BF000), f)
    if which == "grid":
        for t, bf, dp, di in itertools.product((1, 4, 8, 16), (4096, 16384), (2, 8), (0, 1)):
            point(f, dict(threads=t, batch_frames=bf, depth=dp, direct=di), threads=t, seconds=sec,
                  arena=1 << 16, cfg_frames=bf, cfg_bytes=bf * 64, cfg_depth=dp, direct=di)
    elif which == "threads":
        for t in (1, 4, 8, 16):
            point(f, dict(threads=t), threads=t, seconds=sec, arena=1 << 17)
    elif which == "idle":
        for idle in ("wait", "spin", "wait"):
            point(f, dict(threads=16, idle=idle), threads=16, seconds=sec, arena=1 << 17, idle=idle)
    elif which == "depth":
        for dp, wu in itertools.product((2, 3, 4), (50, 100)):
            point(f, dict(threads=16, depth=dp, max_wait_us=wu), threads=16, seconds=sec, arena=1 << 17,
                  cfg_depth=dp, cfg_wait_us=wu)
    elif which == "big":
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for bb in (4 << 20, 1 << 20, 512 << 10, 256 << 10):
            for reg in (0, 1):
                point(fb, dict(threads=16, batch_bytes=bb, zero_copy=reg), threads=16, seconds=sec,
                      arena=1 << 15, register=reg, cfg_bytes=bb)
    elif which == "bigbytes":
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for rep in range(3):
            for bb in (512 << 10, 640 << 10, 768 << 10, 1 << 20):
                for reg in (0, 1):
                    point(fb, dict(rep=rep, batch_bytes=bb, zero_copy=reg), threads=16, seconds=sec,
                          arena=1 << 15, register=reg, cfg_bytes=bb)
    elif which == "pages":
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for rep in range(3):
            for pages in ("huge", "4k"):
                for reg in (0, 1):
                    point(fb, dict(rep=rep, pages=pages, zero_copy=reg), threads=16, seconds=sec,
                          arena=1 << 15, register=reg, pages=pages)
    elif which == "hwq":
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for rep, q in itertools.product(range(2), (4, 8, 16)):
            env = {"GPU_MAX_HW_QUEUES": str(q)}
            point(f, dict(hwq=q, frames=60), env=env, threads=16, seconds=sec, arena=1 << 17)
            for bb, reg in ((1 << 20, 0), (1 << 20, 1), (512 << 10, 0), (512 << 10, 1)):
                point(fb, dict(hwq=q, frames=1514, batch_bytes=bb, zero_copy=reg), env=env, threads=16,
                      seconds=sec, arena=1 << 15, register=reg, cfg_bytes=bb)
    elif which.startswith("abbig:"):
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for rep in range(2):
            for bb, reg in ((1 << 20, 0), (1 << 20, 1), (512 << 10, 0), (512 << 10, 1)):
                for lib in re.split("[,+]", which[6:]):
                    env = None if lib == "default" else {"LD_LIBRARY_PATH": lib}
                    point(fb, dict(lib=lib, rep=rep, batch_bytes=bb, zero_copy=reg), env=env, threads=16,
                          seconds=sec, arena=1 << 15, register=reg, cfg_bytes=bb)
    elif which == "pin" or which.startswith("pin:"):
        PINS = which[4:].split(",") if which.startswith("pin:") else ("0", "8", "2")
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for rep in range(3):
            for pin in PINS:
                # "sK": pinset=K (a block of K CPUs and their SMT siblings per thread)
                kw = dict(pinset=int(pin[1:])) if str(pin).startswith("s") else dict(pin=int(pin))
                point(f, dict(pin=pin, rep=rep, frames=60), threads=16, seconds=sec, arena=1 << 17, **kw)
                point(fb, dict(pin=pin, rep=rep, frames=1514, zero_copy=1), threads=16, seconds=sec,
                      arena=1 << 15, register=1, **kw)
    elif which.startswith("tailab:"):
        fb = os.path.join(tmp, "frames1514.bin")
        bench.write_frames_file(traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001), fb)
        for rep in range(3):
            for lib in re.split("[,+]", which[7:]):
                env = None if lib == "default" else {"LD_LIBRARY_PATH": lib}
                point(f, dict(lib=lib, rep=rep, frames=60), env=env, threads=16, seconds=sec, arena=1 << 17)
                point(fb, dict(lib=lib, rep=rep, frames=1514, zero_copy=1), env=env, threads=16, seconds=sec,
                      arena=1 << 15, register=1)
    elif which.startswith("ab:"):
        import subprocess
        libs = re.split("[,+]", which[3:])
        for rep in range(4):
            for lib in libs:
                env = dict(os.environ)
                if lib != "default":
                    env["LD_LIBRARY_PATH"] = lib
                s0 = cpu_stat()
                r = subprocess.run([bench.LOOP_EXE, f, "loop", "threads=16", f"seconds={sec}", "batch=64",
                                    f"arena={1 << 17}"], capture_output=True, text=True, timeout=120, env=env)
                s1 = cpu_stat()
                d = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {}
                print(json.dumps({"lib": lib, "rep": rep, "mpps": d.get("mpps"), "lat": d.get("latency_us"),
                                  "max_launch_us": d.get("breakdown", {}).get("max_launch_us"),
                                  "throttled": s1.get("nr_throttled", 0) - s0.get("nr_throttled", 0),
                                  "rc": r.returncode}), flush=True)
    else:
        raise SystemExit(f"unknown set {which}")


if __name__ == "__main__":
    main()
