"""Shared test setup: `gpu` marker, golden fixtures, repo on sys.path."""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    _use_sanitized_builds()


def _use_sanitized_builds():
    """tests/test_sanitize.py re-runs the CPU tier with the ASan/UBSan builds
    of the host library and the oracle: it names them in IXG_SAN_LIB /
    IXG_SAN_ORACLE, and they are installed here under the default paths'
    cache keys (test harness only; the product binding has no such switch)."""
    lib, orc = os.environ.get("IXG_SAN_LIB"), os.environ.get("IXG_SAN_ORACLE")
    if not (lib and orc):
        return
    from ix_amd import ixgrx
    from oracle import oracle
    ixgrx._libs[os.path.abspath(ixgrx.LIB_PATH)] = ixgrx.load_library(lib)
    oracle.LIB = orc
    oracle._lib = None
    print("sanitized builds in use:", lib, orc)


def golden_names(prefix: str = ""):
    """RX fixtures by default; demux fixtures are the ones named demux_*, the
    TX fixture is tx.npz (tests/test_tx.py), the event fixture ev.npz
    (tests/test_events.py)."""
    names = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))
    if prefix:
        return [n for n in names if n.startswith(prefix)]
    return [n for n in names if not n.startswith("demux") and n not in ("tx", "ev")]


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.fixture(params=golden_names())
def golden(request):
    g = load_golden(request.param)
    g["name"] = request.param
    return g


@pytest.fixture(params=golden_names("demux"))
def golden_demux(request):
    g = load_golden(request.param)
    g["name"] = request.param
    return g
