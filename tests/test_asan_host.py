"""CPU: the host side of the C ABI under AddressSanitizer (SURVEY §5 sanitizers).

librecsys_amd is rebuilt with ``-Xarch_host -fsanitize=address`` (host code instrumented; the
device code objects are the same gfx950 kernels) into tools/_bin/ (objects cached under
recommendsystem_amd/_build with their own flag tag), and tests/asan_host_probe.py drives every
entry point's host logic -- argument validation, the size / plan queries, the GEMM planner and
the InteractingLayer dry-run dispatch -- in a subprocess with the ASan runtime preloaded.  A
sanitizer report (or any crash) fails the test.  No GPU is used (no kernel is launched: every
call either is a pure query or is rejected by argument validation)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_bin", "librecsys_asan.so")


def _asan_runtime():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        return None, None
    r = subprocess.run([hipcc, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                       text=True)
    path = r.stdout.strip()
    return hipcc, (path if os.path.isabs(path) and os.path.exists(path) else None)


def test_c_abi_host_code_under_asan():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("host-only probe: runs on the CPU container (it calls entry points with null "
                    "device pointers)")
    hipcc, rt = _asan_runtime()
    if rt is None:
        pytest.skip("hipcc / the ASan runtime not available")
    env = dict(os.environ, RS_LIB_OUT=OUT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "recommendsystem_amd", "build.py"),
                        "-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer"],
                       capture_output=True, text=True, env=env, timeout=1500)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    env.pop("RS_LIB_OUT", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_host_probe.py"), OUT,
                        os.path.join(ROOT, "include", "recsys_amd.h")],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "no sanitizer report" in r.stdout, (r.stdout[-2000:] +
                                                                     r.stderr[-6000:])
