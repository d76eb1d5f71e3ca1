"""In-tree build of the dmlab native extension (``dmlab/_C*.so``).

Every ``csrc/*.hip`` translation unit is compiled by ``hipcc --offload-arch=gfx950``
(CDNA4 only, no multi-arch fat binary, no hipify step); ``csrc/bindings.cpp`` is
compiled against the PyTorch-ROCm headers; the objects are linked into one shared
library that lives inside the package, so the file travels with the repository
snapshot to the GPU box and the driver can see which ``.so`` was loaded.

Usage::

    python -m dmlab._build            # incremental
    python -m dmlab._build --force    # full rebuild
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "dmlab"
ARCH = os.environ.get("DMLAB_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    try:
        inc = ce.include_paths(device_type="cuda")
        lib = ce.library_paths(device_type="cuda")
    except TypeError:  # older signature
        inc = ce.include_paths(True)
        lib = ce.library_paths(True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers():
    return sorted(CSRC.rglob("*.h"))


def _sources():
    hip = sorted(CSRC.rglob("*.hip"))
    cpp = sorted(CSRC.rglob("*.cpp"))
    return hip, cpp


def _needs(obj: Path, src: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return r.returncode, " ".join(map(str, cmd)), r.stdout


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    inc, lib, abi = _torch_paths()
    BUILD.mkdir(parents=True, exist_ok=True)
    hip, cpp = _sources()
    hdrs = _headers()
    common = [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", f"-I{CSRC}",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
    ]
    py_inc = sysconfig.get_paths()["include"]
    torch_flags = [f"-I{p}" for p in inc] + [
        f"-I{py_inc}", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-D__HIP_PLATFORM_AMD__=1",
    ]
    jobs_list = []
    objs = []
    for src in hip + cpp:
        rel = src.relative_to(CSRC)
        obj = BUILD / (str(rel).replace("/", "__") + ".o")
        objs.append(obj)
        if force or _needs(obj, src, hdrs):
            cmd = [HIPCC] + common + (torch_flags if src.suffix == ".cpp" else []) + [
                "-c", str(src), "-o", str(obj)]
            jobs_list.append(cmd)
    jobs = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for rc, cmd, out in ex.map(_run, jobs_list):
                if verbose or rc != 0:
                    print(cmd)
                    print(out)
                if rc != 0:
                    raise RuntimeError(f"hipcc failed:\n{cmd}\n{out}")
    out = ext_path()
    if force or jobs_list or not out.exists():
        # link to a temporary file and rename it into place: the in-tree .so is always a
        # complete library (a snapshot of the tree taken mid-build never sees a partial one)
        tmp = out.with_name(out.name + ".tmp")
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp)] + [
            str(o) for o in objs] + [f"-L{p}" for p in lib] + [
            f"-Wl,-rpath,{p}" for p in lib] + [
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
        rc, cmd, txt = _run(link)
        if verbose or rc != 0:
            print(cmd)
            print(txt)
        if rc != 0:
            raise RuntimeError(f"link failed:\n{cmd}\n{txt}")
        os.replace(tmp, out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(f"built {p}")


if __name__ == "__main__":
    sys.exit(main())
