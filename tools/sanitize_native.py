"""Host-side sanitizer run of the C++ runtime: builds csrc/native/*.cpp with
-fsanitize=address,undefined into a scratch directory and exercises the HDF5 writer/reader, the contour tracer and
the resize kernel through that build in a child process (ASan runtime preloaded ahead of anything already listed in
LD_PRELOAD, leak checking off - CPython itself does not free everything at exit).

    python tools/sanitize_native.py [workdir]      -> exit status 0 when clean
"""
import glob
import os
import subprocess
import sys
import sysconfig
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import importlib.util, sys
import numpy as np
spec = importlib.util.spec_from_file_location("_native", sys.argv[1])
m = importlib.util.module_from_spec(spec)
spec.loader.exec_module(m)
h5 = m.h5lite
rng = np.random.default_rng(0)
tree = {"attrs": {"s": "text", "names": [b"a", b"bb", b"ccc"], "i": np.arange(5, dtype=np.int64)},
        "groups": {f"g{i}": {"attrs": {"k": f"v{i}"}, "groups": {},
                             "datasets": {f"d{j}:0": rng.standard_normal((3, j + 2)).astype(np.float32)
                                          for j in range(6)}} for i in range(40)},
        "datasets": {"top": np.arange(12, dtype=np.float32).reshape(3, 4)}}
p = sys.argv[2]
h5.write_file(p, tree)
back = h5.read_file(p)
assert sorted(back["groups"]) == sorted(tree["groups"])
for g, node in tree["groups"].items():
    for d, arr in node["datasets"].items():
        assert np.array_equal(np.asarray(back["groups"][g]["datasets"][d]["data"]), arr)
assert np.array_equal(np.asarray(back["datasets"]["top"]["data"]), tree["datasets"]["top"])
c = m.contour
for seed in range(20):
    img = (rng.random((40 + seed, 57)) > 0.6).astype(np.uint8) * 255
    cs, hier, _ = c.find_contours(img, 127, True)
    for pts in cs:
        c.contour_area(pts, False)
        c.arc_length(pts, True)
        c.approx_poly_dp(pts, 1.5, True)
src = rng.integers(0, 255, (31, 45, 3), dtype=np.uint8)
out = m.resize_bilinear(src, 64, 64) if hasattr(m, "resize_bilinear") else None
print("sanitized native selftest ok")
'''


def main(work=None) -> int:
    import pybind11
    work = work or tempfile.mkdtemp(prefix="cfl_asan_")
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    so = os.path.join(work, "_native" + ext)
    flags = ["-O1", "-g", "-fPIC", "-std=c++17", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=undefined", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "native", "*.cpp")))
    r = subprocess.run(["g++", *flags, "-shared", "-o", so, *srcs, "-lpthread"], capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr[-4000:])
        return 2
    asan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    ubsan = subprocess.run(["g++", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ)
    pre = [asan, ubsan] + [x for x in env.get("LD_PRELOAD", "").split(":") if x]   # keep whatever is listed
    env["LD_PRELOAD"] = ":".join(pre)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    child = os.path.join(work, "child.py")
    with open(child, "w") as f:
        f.write(CHILD)
    r = subprocess.run([sys.executable, child, so, os.path.join(work, "t.h5")], env=env, capture_output=True,
                       text=True, timeout=600)
    sys.stdout.write(r.stdout[-2000:])
    sys.stderr.write(r.stderr[-6000:])
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else None))
