"""examples/ix_rx_shim.c (INTEGRATION.md's call-site sketch) and
examples/ix_echo_pipeline.c (TX -> RX + demux -> usys descriptors through the
C ABI) build against include/ixgrx.h + libixgrx.so and run: on CPU they must
fail cleanly at ixg_rx_init (no device, exit 2); on the GPU all 64 frames
reach the TCP callee, and every echo reply round-trips to its own PCB and
descriptor."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    exe = str(tmp_path / "ix_rx_shim")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "ix_rx_shim.c"), "-L" + os.path.join(ROOT, "ix_amd"),
                    "-lixgrx", "-Wl,-rpath," + os.path.join(ROOT, "ix_amd"), "-o", exe], check=True)
    return exe


def test_example_builds_and_fails_cleanly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    r = subprocess.run([_build(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "ixg_rx_init" in r.stderr


@pytest.mark.gpu
def test_example_runs_on_gpu(tmp_path):
    r = subprocess.run([_build(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tcp=64" in r.stdout


def _build_pipeline(tmp_path):
    exe = str(tmp_path / "ix_echo_pipeline")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include",
                    os.path.join(ROOT, "examples", "ix_echo_pipeline.c"), "-L" + os.path.join(ROOT, "ix_amd"),
                    "-lixgrx", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + os.path.join(ROOT, "ix_amd"),
                    "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
    return exe


def test_pipeline_example_builds_and_fails_cleanly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    r = subprocess.run([_build_pipeline(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "ixg_rx_init" in r.stderr


@pytest.mark.gpu
def test_pipeline_example_runs_on_gpu(tmp_path):
    r = subprocess.run([_build_pipeline(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "usys_tcp_recv=4096/4096" in r.stdout and "tcp_head=4096" in r.stdout


def _build_loop(tmp_path):
    exe = str(tmp_path / "ix_async_loop")
    subprocess.run(["gcc", "-std=gnu11", "-O2", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "ix_async_loop.c"), "-L" + os.path.join(ROOT, "ix_amd"),
                    "-lixgrx", "-lpthread", "-Wl,-rpath," + os.path.join(ROOT, "ix_amd"), "-o", exe], check=True)
    return exe


def _frames_file(tmp_path, kind="imix", n=5000):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from ix_amd import traces
    tr = traces.make_trace(kind, n, seed=0x1A77, bad_ip=0.02, bad_l4=0.02)
    p = str(tmp_path / "frames.bin")
    bench.write_frames_file(tr, p)
    return tr, p


def test_async_loop_builds_and_fails_cleanly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    _, f = _frames_file(tmp_path, n=100)
    r = subprocess.run([_build_loop(tmp_path), f, "loop", "seconds=0.1"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "no such HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["direct=0"], ["register=1"], ["cfg_wait_us=0", "cfg_depth=2"]])
def test_async_loop_runs_on_gpu(tmp_path, extra):
    """IX's run loop over the asynchronous path, 4 CPUs (threads), <= 64
    frames per iteration: thread 0's records (submission order) are the
    oracle's, and every frame submitted comes back."""
    import json
    import numpy as np
    from oracle import oracle
    from ix_amd import traces
    tr, f = _frames_file(tmp_path)
    dump = str(tmp_path / "dump.bin")
    r = subprocess.run([_build_loop(tmp_path), f, "loop", "threads=4", "seconds=0.5", "arena=8192",
                        "dump=" + dump] + extra, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["frames"] > 0 and res["latency_us"]["n"] > 0
    v = res["verdicts"]
    assert sum(v.values()) == res["frames"]
    recs = np.fromfile(dump, dtype=np.uint8).reshape(-1, 16)
    er, _ = oracle.rx_trace(tr, traces.RSS_KEY, threads=8)
    assert recs.shape == er.shape and np.array_equal(recs, er)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n", [("sync", 64), ("sync", 1024), ("async1", 64)])
def test_async_loop_latency_modes(tmp_path, mode, n):
    import json
    _, f = _frames_file(tmp_path, "tcp64", 2048)
    r = subprocess.run([_build_loop(tmp_path), f, mode, f"n={n}", "seconds=0.2"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["calls"] > 0 and res["latency_us"]["p50"] > 0
