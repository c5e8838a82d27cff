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
    assert "usys_tcp_recv=4096/4096" in r.stdout
