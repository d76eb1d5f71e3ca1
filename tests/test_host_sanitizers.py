"""Host-side sanitizer run: the geometry helpers shared by the host
launchers and the HIP kernels, compiled with AddressSanitizer + UBSan and executed on the
CPU.  (GPU-side ASan / XNACK are unavailable on the MI355X pool; kernels are checked
numerically against PyTorch instead, and DMLAB_SYNC_DEBUG=1 localises device faults.)"""
import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_geom_fastdiv_asan_ubsan(tmp_path):
    exe = tmp_path / "geom_check"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", str(HERE / "native" / "geom_check.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout
