"""Build check: no product kernel spills registers to scratch.

Register spills are silent performance regressions (a refactor of the PCB
walk once cost the general kernels 33 spilled VGPRs with every parity test
still green). This compiles each HIP source for gfx950 with hipcc's
resource-usage remarks and asserts zero scratch for every kernel the C ABI
launches. CPU only (hipcc cross-compiles); ~1 minute.
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "ix_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = ["ixgrx_kernels.hip", "ixgrx_tx.hip", "ixgrx_demux.hip", "ixgrx_ev.hip"]
# A/B-only variants (IXGRX_GEN_VARIANT / IXGRX_SHORT_VARIANT, never launched
# by default) built with occupancy targets that trade registers for waves
AB_ONLY = re.compile(r"ixg_rx_(general_w[34]|short_w4)_[so]$")


def _resources(src):
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", os.path.join(CSRC, src),
                          "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, check=True, cwd=CSRC).stderr
    res, name = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            res[name] = {}
            continue
        m = re.search(r"remark:\s+(ScratchSize \[bytes/lane\]|VGPRs Spill|VGPRs): (\d+)", line)
        if m and name:
            res[name][m.group(1)] = int(m.group(2))
    return res


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src", SOURCES)
def test_no_scratch(src):
    res = _resources(src)
    assert res, f"no kernels found in {src}"
    bad = {k: v for k, v in res.items()
           if not AB_ONLY.search(k) and (v.get("ScratchSize [bytes/lane]", 0) or v.get("VGPRs Spill", 0))}
    assert not bad, f"kernels with scratch / spills in {src}: {bad}"
