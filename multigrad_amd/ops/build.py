"""In-tree build of the native extension ``multigrad_amd/_C.so`` for gfx950.

``.hip`` sources are compiled by ``hipcc --offload-arch=gfx950`` and ``.cpp`` host sources
by ``g++``; the shared object is linked with ``g++`` against PyTorch's bundled HIP
runtime, so the process maps exactly one ``libamdhip64`` (verified on MI355X).  No
hipify step and no JIT cache: the ``.so`` lives next to the package and travels with
the source tree.

Usage: ``python -m multigrad_amd.ops.build [--force] [-j N] [-v]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from typing import List

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
OBJ_DIR = os.environ.get("MULTIGRAD_OBJ_DIR", os.path.join(os.path.dirname(PKG_DIR), "build", "obj"))
TARGET = os.environ.get("MULTIGRAD_TARGET", os.path.join(PKG_DIR, "_C.so"))
ARCH = os.environ.get("MULTIGRAD_OFFLOAD_ARCH", os.environ.get("PYTORCH_ROCM_ARCH", "gfx950"))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_dirs():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def sources() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers() -> List[str]:
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hpp"))]


def _obj(src: str) -> str:
    return os.path.join(OBJ_DIR, os.path.basename(src) + ".o")


def _stale(out: str, deps: List[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def source_hash() -> str:
    """SHA-1 over every native source and header (name + content), the build stamp that
    ``_C.build_info()`` reports, so a run's records show which sources its binary came
    from."""
    import hashlib
    h = hashlib.sha1()
    for f in sorted(sources() + _headers()):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _stamp_path() -> str:
    return os.path.join(OBJ_DIR, "source_hash.txt")


def _compile_cmd(src: str) -> List[str]:
    inc, _, abi = _torch_dirs()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-Wno-unused-result",
              f"-I{CSRC}", f"-I{py_inc}"] + [f"-I{d}" for d in inc] + [f"-I{ROCM}/include"]
    if os.path.basename(src) == "bindings.cpp":
        common = common + [f'-DMG_BUILD_HASH="{source_hash()}"', f'-DMG_BUILD_ARCH="{ARCH}"']
    if src.endswith(".hip"):
        extra = os.environ.get("MULTIGRAD_HIPCC_FLAGS", "").split()
        return [os.path.join(ROCM, "bin", "hipcc"), "-c", src, "-o", _obj(src),
                f"--offload-arch={ARCH}", "-ffp-contract=fast"] + common + extra
    return ["g++", "-c", src, "-o", _obj(src)] + common


def build(force: bool = False, verbose: bool = False, jobs: int = 0) -> str:
    """Compile stale objects and (re)link ``_C.so``; returns the library path."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = sources()
    hdrs = _headers()
    todo = [s for s in srcs if force or _stale(_obj(s), [s] + hdrs)]
    # the stamp compiled into bindings.cpp must follow every source change
    digest = source_hash()
    old = open(_stamp_path()).read().strip() if os.path.exists(_stamp_path()) else ""
    bind = [s for s in srcs if os.path.basename(s) == "bindings.cpp"]
    if digest != old:
        todo = sorted(set(todo) | set(bind))
    jobs = jobs or min(len(todo) or 1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8)

    def run(src):
        cmd = _compile_cmd(src)
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {os.path.basename(src)}\n{r.stdout}\n{r.stderr}")
        return src

    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for s in ex.map(run, todo):
                if verbose:
                    print(f"compiled {os.path.basename(s)}", flush=True)
    objs = [_obj(s) for s in srcs]
    if force or todo or _stale(TARGET, objs):
        _, libdir, _ = _torch_dirs()
        tmp = TARGET + f".tmp{os.getpid()}"
        cmd = ["g++", "-shared", "-o", tmp] + objs + [
            f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", "-lamdhip64", f"-Wl,-rpath,{libdir}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, TARGET)
    with open(_stamp_path(), "w") as f:
        f.write(digest)
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose, jobs=a.jobs))


if __name__ == "__main__":
    main()
