"""Host sanitizers: the C host library (ix_amd/csrc/ixgrx_host.c)
and the oracle (oracle/ixgrx_oracle.c) built with -fsanitize=address,undefined,
and the CPU test tier re-run against those builds in a child process with the
sanitizer runtimes preloaded. The host paths' staging and ring logic runs
sanitized over the CPU stand-in for HIP (tests/fakehip). The two C examples
are built against the sanitized host library and run too (on a machine without a GPU they stop at
ixg_rx_init's -ENODEV, after exercising argument checking and context setup).

Any ASan report or UBSan error aborts the child (-fno-sanitize-recover), so
the child's exit status is the verdict. CPU only.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_LIB = os.path.join(ROOT, "build", "san", "libixgrx.so")
SAN_ORACLE = os.path.join(ROOT, "oracle", "_san", "liboracle.so")
SAN_FAKE = os.path.join(ROOT, "build", "fakehip", "libixgrx_fake_san.so")


def _runtime(name):
    p = subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


ASAN, UBSAN = _runtime("libasan.so"), _runtime("libubsan.so")
pytestmark = pytest.mark.skipif(not (ASAN and UBSAN), reason="gcc sanitizer runtimes not installed")


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "ix_amd", "csrc"), "san"], check=True,
                   capture_output=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "fakehip")], check=True, capture_output=True)
    assert os.path.exists(SAN_LIB) and os.path.exists(SAN_ORACLE) and os.path.exists(SAN_FAKE)


def _env():
    env = dict(os.environ)
    env["LD_PRELOAD"] = ASAN + ":" + UBSAN
    env["ASAN_OPTIONS"] = "detect_leaks=0:verify_asan_link_order=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["IXG_SAN_LIB"] = SAN_LIB        # tests/conftest.py swaps these builds in
    env["IXG_SAN_ORACLE"] = SAN_ORACLE
    env["IXG_FAKE_LIB"] = SAN_FAKE       # tests/test_hostpath_cpu.py: the host paths over fakehip
    return env


def test_examples_under_sanitizers(san_build):
    for ex in ("ix_rx_shim", "ix_echo_pipeline"):
        p = subprocess.run([os.path.join(ROOT, "build", "san", ex)], capture_output=True, text=True, timeout=300,
                           env=_env())
        # 2 = no HIP device (CPU container); 0 = ran on a GPU
        assert p.returncode in (0, 2), f"{ex}: rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}"
        assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]


def test_cpu_tier_under_sanitizers(san_build):
    """The CPU tests that drive C code (oracle vs the reference goldens, the
    ABI's host-side entry points, TX/demux/event oracles), with both C
    libraries replaced by their sanitized builds."""
    tests = ["test_oracle_golden.py", "test_abi.py", "test_tx.py", "test_demux.py", "test_events.py",
             "test_traces.py", "test_hostpath_cpu.py"]
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"] + \
        [os.path.join(ROOT, "tests", t) for t in tests]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=_env(), cwd=ROOT)
    tail = p.stdout[-3000:] + p.stderr[-5000:]
    assert p.returncode == 0, tail
    assert "sanitized builds in use" in p.stdout, tail
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, tail
