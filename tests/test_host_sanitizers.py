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


ROOT = HERE.parent


def _libs():
    out = []
    for n in ("libasan.so", "libubsan.so"):
        p = subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
        if not p or not Path(p).exists():
            return None
        out.append(p)
    return out


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None,
                    reason="no host C++ compiler")
@pytest.mark.timeout(900)
def test_reducer_asan_ubsan_two_rank_ddp():
    """The C++ DDP bucket reducer (csrc/reducer.cpp) and its pybind argument checks, built
    for the CPU with AddressSanitizer + UBSan, driving a 2-rank gloo DDP run (fp32 and bf16
    communication, no_sync accumulation, out-of-range ids rejected)."""
    import os
    import sysconfig

    import torch
    from torch.utils import cpp_extension as ce

    libs = _libs()
    if libs is None:
        pytest.skip("libasan / libubsan not found")
    out = ROOT / "build" / "asan"
    out.mkdir(parents=True, exist_ok=True)
    so = out / ("reducer_asan" + sysconfig.get_config_var("EXT_SUFFIX"))
    src = ROOT / "csrc" / "reducer.cpp"
    mod = out / "mod.cpp"
    mod.write_text('#include <torch/extension.h>\nvoid register_reducer(pybind11::module_& m);\n'
                   'PYBIND11_MODULE(reducer_asan, m) { register_reducer(m); }\n')
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        lp = ce.library_paths()
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared",
               "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
               f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
               "-DTORCH_EXTENSION_NAME=reducer_asan", "-DTORCH_API_INCLUDE_EXTENSION_H",
               *[f"-I{i}" for i in ce.include_paths()], f"-I{sysconfig.get_paths()['include']}",
               str(src), str(mod), "-o", str(so), *[f"-L{p}" for p in lp],
               *[f"-Wl,-rpath,{p}" for p in lp], "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ)
    env["LD_PRELOAD"] = ":".join(libs + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else []))
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run(["python", str(HERE / "native" / "reducer_asan_driver.py"), str(out)],
                       capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.stdout.strip().endswith("ok"), r.stdout
