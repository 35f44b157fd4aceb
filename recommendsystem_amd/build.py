"""Build the gfx950 C-ABI library ``librecsys_amd.so`` in-tree with hipcc.

Every ``csrc/*.hip`` file is compiled to an object for ``--offload-arch=gfx950`` (in parallel,
skipping objects newer than their sources and headers), then linked into one shared library next
to this file.  The library exports exactly the ``extern "C"`` entry points declared in
``include/recsys_amd.h``; no torch headers are involved.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "_build")
# RS_LIB_OUT: build a kernel variant (extra -D flags) to another path, loaded with RS_LIB_PATH
LIB_PATH = os.environ.get("RS_LIB_OUT") or os.path.join(PKG_DIR, "librecsys_amd.so")
ARCH = os.environ.get("RS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build recommendsystem_amd)")


COMMON_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-munsafe-fp-atomics",
    "-fvisibility=hidden",
    "-Wno-unused-result",
]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _tag(extra: list[str]) -> str:
    import hashlib
    return hashlib.sha1(" ".join(extra).encode()).hexdigest()[:8]


# per-unit flags (measured choices, see the unit's header comment)
PER_SOURCE_FLAGS = {"il_inst_a_fwd.hip": ["-fno-slp-vectorize"]}


def _compile(src: str, headers: list[str], extra: list[str]) -> str:
    extra = list(extra) + PER_SOURCE_FLAGS.get(os.path.basename(src), [])
    obj = os.path.join(BUILD_DIR, f"{os.path.basename(src)}.{_tag(extra)}.o")
    if _newer(obj, [src] + headers):
        cmd = [_hipcc(), *COMMON_FLAGS, *extra, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, extra: list[str] | None = None) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.hpp")))
    extra = list(extra or [])
    workers = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        objs = list(ex.map(lambda s: _compile(s, headers, extra), srcs))
    stamp = os.path.join(BUILD_DIR, "lib.flags")
    prev = open(stamp).read() if os.path.exists(stamp) else None
    if _newer(LIB_PATH, objs) or prev != _tag(extra):
        # a host-sanitizer build (-Xarch_host -fsanitize=...) links the shared sanitizer runtime
        san = [f for f in extra if f.startswith("-fsanitize=")]
        link = [*san, "-shared-libasan"] if san else []
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)  # (RS_LIB_OUT may name a fresh dir)
        cmd =[_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *link, *objs,
               "-L/opt/rocm/lib", "-lhipblaslt", "-Wl,-rpath,/opt/rocm/lib", "-o", LIB_PATH]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        with open(stamp, "w") as f:
            f.write(_tag(extra))
    if verbose:
        print(f"built {LIB_PATH}")
    return LIB_PATH


if __name__ == "__main__":
    build(verbose=True, extra=sys.argv[1:])
