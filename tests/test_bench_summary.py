"""bench.summary (VERDICT r3 Next #3): every line of a bench run in one
compact object, last in the JSON line, small enough for the tail the
driver's record keeps. Built here from a synthetic result dict with every
line bench.py can emit (no GPU)."""
import json

import bench


def _line(frac=0.5, ms=0.3, mpps=1000.0):
    return {"roofline_frac": frac, "kernel_ms_avg": ms, "mpps": mpps, "parity": "ok"}


def _loop(mpps, mx=100.0):
    return {"mpps": mpps, "latency_us": {"p50": 50.0, "p99": 90.0, "max": mx}}


def _res():
    return {
        "value": 77191.3, "parity": "ok",
        "roofline": {"frac": 0.691, "kernel_ms_avg": 0.2185},
        "bad_csum": _line(), "secondary": _line(0.7, 2.3, 3650.0),
        "lines": {"c3": _line(0.55, 1.45), "c5": _line(0.56, 0.43), "c5r": _line(0.38, 0.41)},
        "c4_strong": {"roofline_frac_per_gpu": 0.75, "kernel_ms": 17.0, "mpps_device_resident": 3936.0,
                      "parity": "ok"},
        "demux": {"fused": _line(), "separate": _line(), "parity": "ok",
                  "mixed": {"fused": _line(), "parity": "ok", "kinds": {"ACTIVE": 3, "TIMEWAIT": 1, "LISTEN": 1}},
                  "mixed_nolisten": {"fused": _line(), "parity": "ok", "kinds": {"ACTIVE": 3, "RESET": 1}}},
        "events": {"roofline_frac": 0.58, "kernel_ms_avg": 0.3, "mevents_per_s": 39000.0, "parity": "ok"},
        "tcpx": _line(), "tx": {"tcp64": _line(), "tcp1514": _line()},
        "host_path": {"parity": "ok", "loop": {"threads1": _loop(100.0), "threads4": _loop(400.0),
                                               "threads16": _loop(700.0, 12000.0),
                                               "tcp1514_threads16": _loop(28.0),
                                               "tcp1514_threads16_zero_copy": _loop(33.0)}},
        "cpu_baseline": {"value": 1068.4},
    }


def test_summary_every_line_and_compact():
    s = bench.summary(_res())
    for k in ("c2", "c2b", "c4", "c3", "c5", "c5r", "c4_strong", "demux_fused", "demux_sep", "demux_mixed",
              "demux_mixed_nolisten", "events", "tcpx", "tx_tcp64", "tx_tcp1514", "host_path", "cpu_baseline_mpps"):
        assert k in s, k
    for k in ("c2", "c3", "c5r", "demux_fused", "events"):
        assert set(s[k]) >= {"frac", "kernel_ms", "mpps", "parity"}
    assert s["c2"]["frac"] == 0.691 and s["c2"]["kernel_ms"] == 0.2185
    assert s["demux_mixed"]["kinds"] == {"ACTIVE": 3, "TIMEWAIT": 1, "LISTEN": 1}
    hp = s["host_path"]
    assert hp["t1"] == 100.0 and hp["t16"] == 700.0 and hp["tcp1514_t16_zero_copy"] == 33.0
    assert hp["t16_max_latency_us"] == 12000.0 and hp["parity"] == "ok"
    assert len(json.dumps(s)) < 2000


def test_summary_minimal_run():
    """A run with only the primary line (--secondary '' --extra '' --no-demux ...)."""
    r = {"value": 1.0, "parity": "ok", "roofline": {"frac": 0.5, "kernel_ms_avg": 0.2}}
    assert list(bench.summary(r)) == ["c2"]
