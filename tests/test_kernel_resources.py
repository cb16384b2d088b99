"""Compile-time resource check of every hand-written gfx950 kernel (CPU only: hipcc
cross-compiles). A kernel that spills to scratch or outgrows the 160 KiB of LDS per
CU is a performance bug that no numerics test catches - e.g. a by-value kernel
argument whose address escapes gets copied to per-lane scratch (1456 B/lane, seen
once in window_stats.hip and fixed)."""

import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
LDS_BYTES_PER_CU = 160 * 1024


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["window_stats.hip", "long_window.hip", "node_window.hip", "publish.hip", "calib.hip"])
def test_kernels_have_no_scratch_and_fit_lds(src, tmp_path):
    res = subprocess.run(
        [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/csrc", "--cuda-device-only", "-c",
         os.path.join(ROOT, "csrc", src), "-o", str(tmp_path / "k.o"), "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True, timeout=600,
    )
    assert res.returncode == 0, res.stderr[-3000:]
    kernels = {}
    name = None
    for line in res.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            kernels[name] = {}
            continue
        m = re.search(r"(ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]|VGPRs): (\d+)", line)
        if m and name is not None:
            kernels[name][m.group(1)] = int(m.group(2))
    assert kernels, res.stderr[-2000:]
    for k, r in kernels.items():
        assert r.get("ScratchSize [bytes/lane]", 0) == 0, (k, r)
        assert r.get("LDS Size [bytes/block]", 0) <= LDS_BYTES_PER_CU, (k, r)
