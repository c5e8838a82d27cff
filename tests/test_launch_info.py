"""ixg_rx_launch_info: the split the device chose for the context's last
launch, for the batch shapes of BASELINE.json's configs."""
import numpy as np
import pytest

from ix_amd import ixgrx, traces

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,layout,mode,big,sampled", [
    ("tcp64", "stride", "fast", False, False),      # C2: the coalesced kernel, no sampler
    ("imix", "packed", "long", False, True),        # C3
    ("mixed", "packed", "short", False, True),      # C5
    ("tcp1514", "packed", "long", True, True),      # C4's frames in the offset layout
])
def test_launch_info(kind, layout, mode, big, sampled):
    tr = traces.make_trace(kind, 64 * 300, seed=41)
    if layout == "packed" and tr.off is None:
        tr = traces.Trace(tr.blob, tr.offsets().copy(), tr.len, 0)
    e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, flags=ixgrx.IXG_F_IPV6 if kind == "mixed" else 0))
    try:
        e.batch_trace(tr)
        info = e.launch_info()
    finally:
        e.close()
    assert info == {"mode": mode, "big": big, "sampled": sampled}, info
