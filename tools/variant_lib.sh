#!/bin/bash
# Link a kernel-variant library: ONE source recompiled with extra -D flags, every other object
# taken from the default in-tree build (recommendsystem_amd/_build, default flags per source).
#   bash tools/variant_lib.sh OUT.so SOURCE.hip -DFLAG=... [...]
set -e
cd "$(dirname "$0")/.."
out=$1; src=$2; shift 2
b=recommendsystem_amd/_build
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -fvisibility=hidden -Wno-unused-result "$@" -c recommendsystem_amd/csrc/$src -o $tmp/var.o
objs=$(python3 - "$src" <<'PY'
import glob, os, sys
sys.path.insert(0, ".")
from recommendsystem_amd import build as B
for f in sorted(glob.glob(os.path.join(B.CSRC, "*.hip"))):
    n = os.path.basename(f)
    if n != sys.argv[1]:
        print(os.path.join(B.BUILD_DIR, f"{n}.{B._tag(B.PER_SOURCE_FLAGS.get(n, []))}.o"))
PY
)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $tmp/var.o $objs -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib -o "$out"
rm -rf $tmp
echo "built $out"
