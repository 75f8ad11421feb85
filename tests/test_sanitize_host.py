"""the native host runtime (csrc/runtime.cpp) under AddressSanitizer +
UndefinedBehaviorSanitizer, driven over edge-case schedules and compared with the regular
build.  (GPU ASan and xnack+ are unavailable on this pool; GPU kernels are covered by the
fp32-reference numerics tests.)"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib(name):
    try:
        p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    except OSError:
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(shutil.which("g++") is None or _lib("libasan.so") is None,
                    reason="needs g++ with libasan")
def test_host_runtime_under_asan_ubsan():
    so = os.path.join(ROOT, "build", "asan", "_C_host_asan.so")
    src = [os.path.join(ROOT, "multigrad_amd", "csrc", "runtime.cpp"),
           os.path.join(ROOT, "tools", "sanitize", "host_bindings.cpp")]
    if not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in src):
        r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "build.sh")],
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, LD_PRELOAD=f"{_lib('libasan.so')} {_lib('libubsan.so') or ''}".strip(),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize", "drive.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "cases clean" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
