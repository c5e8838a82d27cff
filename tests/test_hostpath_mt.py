"""Many IX CPUs at once on the C host library, on the CPU (no GPU): the
driver tests/fakehip/mt_async.c runs 16 threads, one context each, through
ixg_rx_submit_mbufs / ixg_rx_poll (and, on some threads, ixg_rx_set_fdir
with batches in flight and the synchronous ixg_rx_batch_mbufs) over the fake
HIP runtime, so the launch path (launch_open -> ixg_stage_launch ->
ixg_launch_ds -> ixgrx_launch) runs on every thread at once; every record
is checked against the oracle's, in submission order. Built plain, under
ThreadSanitizer and under ASan/UBSan (the 16-thread
SIGSEGV of the launch path). The zero-copy and failing-launch variant is the
ADVICE r04 case: a launch that fails and is retried must lay the in-place
frames' offsets out again from the gathered ones."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "fakehip")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "fakehip")], check=True)
    return OUT


@pytest.mark.parametrize("variant", ["mt_async", "mt_async_tsan", "mt_async_san"])
@pytest.mark.parametrize("mode", [[], ["zc=1", "fail=1"]], ids=["staged", "zero_copy_failing_launches"])
def test_sixteen_contexts(built, variant, mode):
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 exitcode=66"
    env["ASAN_OPTIONS"] = "detect_leaks=1 abort_on_error=1"
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(built, variant), "16", "2000", "2"] + mode, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("ok threads=16 records=64000"), r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
