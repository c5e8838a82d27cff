"""Synthetic traces are what they claim: valid frames of the named shapes."""
import numpy as np
import pytest

from ix_amd import traces
from oracle import oracle


@pytest.mark.parametrize("kind", ["tcp64", "tcp64opt", "imix", "tcp1514", "mixed"])
def test_trace_valid(kind):
    tr = traces.make_trace(kind, 600, seed=0x1B0000 + 7)
    flags = 2 if kind == "mixed" else 0
    rec, cs = oracle.rx_trace(tr, traces.RSS_KEY, flags=flags, hash_mode=oracle.HASH_TABLE)
    v = rec[:, 2]
    ok = {1, 2, 5, 6}
    assert set(np.unique(v).tolist()) <= ok, np.unique(v)
    assert ((rec[:, 3] & 0x0C) == 0x0C).all()  # L4 checksum checked and ok
    if kind == "tcp64":
        assert (tr.len == 60).all() and (rec[:, 2] == 1).all()
    if kind == "tcp1514":
        assert (tr.len == 1514).all()
    if kind == "tcp64opt":  # C2's slots, one IPv4 option word: never fixed-shape
        assert (tr.len == 60).all() and tr.stride == 60 and (rec[:, 2] == 1).all()
        assert (tr.blob[14::60][:tr.n] == 0x46).all()


def test_trace_bad_fraction():
    tr = traces.make_trace("tcp64", 4000, seed=3, bad_ip=0.05, bad_l4=0.05)
    rec, _ = oracle.rx_trace(tr, traces.RSS_KEY, hash_mode=oracle.HASH_TABLE)
    v = rec[:, 2]
    assert 0.02 < (v == 0x8E).mean() < 0.09 and 0.02 < (v == 0x8F).mean() < 0.09


def test_pool_tiling_repeats_records():
    tr = traces.make_trace("tcp64", 1000, seed=5, pool=100)
    rec, _ = oracle.rx_trace(tr, traces.RSS_KEY, hash_mode=oracle.HASH_TABLE)
    assert (rec[100:200] == rec[:100]).all()
