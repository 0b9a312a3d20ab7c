"""In-tree build of the two native extension modules.

* ``_native``  host C++ (HDF5 writer/reader, contour geometry, image resize): g++ + pybind11, no GPU toolchain.
* ``_C``       HIP/CDNA4 kernels for gfx950 (``csrc/kernels/*.hip``, torch-free translation units compiled with
               ``hipcc --offload-arch=gfx950``) + one binding TU (``csrc/bindings.cpp``, torch/extension.h).

Objects are cached under ``build/`` keyed by a hash of (source, headers, flags); the ``.so`` files land inside the
package so they travel with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _hash(paths: List[str], flags: List[str]) -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:20]


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout[-6000:]}")


def _compile_all(jobs, max_workers: int) -> List[str]:
    with cf.ThreadPoolExecutor(max_workers=max_workers) as ex:
        return list(ex.map(lambda j: j(), jobs))


def _pybind_includes() -> List[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def native_path() -> str:
    return os.path.join(PKG, "_native" + EXT)


def hip_path() -> str:
    return os.path.join(PKG, "_C" + EXT)


def _native_inputs():
    srcs = sorted(glob.glob(os.path.join(CSRC, "native", "*.cpp")))
    flags = ["-O2", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-Wall", "-Wno-unused-variable"] + _pybind_includes()
    import pybind11
    portable = [f for f in flags if not f.startswith("-I")] + [pybind11.__version__, sys.version.split()[0]]
    return srcs, flags, _hash(srcs, portable)


def is_current(path: str, key: str) -> bool:
    """The built module exists and its stamp matches the hash of the sources/flags it must be built from."""
    stamp = path + ".stamp"
    if not (os.path.exists(path) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read() == key


def native_key() -> str:
    return _native_inputs()[2]


def build_native(force: bool = False, verbose: bool = True) -> str:
    srcs, flags, key = _native_inputs()
    out = native_path()
    stamp = out + ".stamp"
    if not force and is_current(out, key):
        return out
    os.makedirs(os.path.join(BUILD, "native"), exist_ok=True)
    cxx = os.environ.get("CXX", "g++")

    def job(src):
        def run():
            obj = os.path.join(BUILD, "native", os.path.basename(src) + ".o")
            _run([cxx, *flags, "-c", src, "-o", obj])
            return obj
        return run

    objs = _compile_all([job(s) for s in srcs], 4)
    tmp = out + ".tmp"
    _run([cxx, "-shared", "-o", tmp, *objs, "-lpthread"])
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    if verbose:
        print(f"[build] {os.path.relpath(out, ROOT)}")
    return out


def _torch_flags():
    import torch
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = [f"-I{tdir}/include", f"-I{tdir}/include/torch/csrc/api/include"]
    libs = [f"-L{tdir}/lib", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-Wl,-rpath,{tdir}/lib"]
    return inc, libs, abi


def _hip_inputs():
    kern = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")) + glob.glob(os.path.join(CSRC, "*.h")))
    binding = os.path.join(CSRC, "bindings.cpp")
    inc, libs, abi = _torch_flags()
    base = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", f"-I{CSRC}", f"-I{CSRC}/kernels",
            "-Wno-unused-result", "-Wno-unused-command-line-argument", "-ffp-contract=fast"]
    import torch
    # the key must not depend on where the tree or torch live (the snapshot runs from another path on the GPU
    # box): source bytes + path-free flags + torch version + arch
    portable = [f for f in base if not f.startswith("-I")] + [torch.__version__, ARCH, str(abi)]
    key = _hash(kern + headers + [binding], portable)
    return kern, headers, binding, inc, libs, abi, base, key


def hip_key() -> str:
    return _hip_inputs()[-1]


def build_hip(force: bool = False, verbose: bool = True, jobs: int = 0) -> str:
    kern, headers, binding, inc, libs, abi, base, key = _hip_inputs()
    out = hip_path()
    stamp = out + ".stamp"
    if not force and is_current(out, key):
        return out
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    os.makedirs(os.path.join(BUILD, "hip"), exist_ok=True)

    def job(src, extra):
        def run():
            k = _hash([src] + headers, base + extra)
            obj = os.path.join(BUILD, "hip", f"{os.path.basename(src)}.{k}.o")
            if not os.path.exists(obj):
                _run([HIPCC, *base, *extra, "-c", src, "-o", obj + ".tmp"])
                os.replace(obj + ".tmp", obj)
            return obj
        return run

    bflags = inc + _pybind_includes() + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
                                         "-DTORCH_API_INCLUDE_EXTENSION_H", "-x", "hip"]
    js = [job(s, []) for s in kern] + [job(binding, bflags)]
    objs = _compile_all(js, jobs or min(8, os.cpu_count() or 4))
    tmp = out + ".tmp"
    _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs, *libs])
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    if verbose:
        print(f"[build] {os.path.relpath(out, ROOT)} ({len(kern)} kernel TUs, {ARCH})")
    return out


if __name__ == "__main__":
    build_native(force="--force" in sys.argv)
    if "--native-only" not in sys.argv:
        build_hip(force="--force" in sys.argv)
