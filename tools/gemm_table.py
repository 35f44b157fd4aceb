"""Tabulate tools/gemm_shapes.py logs of a tile sweep: one row per shape, one column per setting."""
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
rows, cols = {}, []
for f in sorted(d.glob("*.log")):
    if f.name.startswith(("pytest", "diag", "wl_")):
        continue
    cols.append(f.stem)
    for line in f.read_text().splitlines():
        if line.startswith('{"kind"'):
            r = json.loads(line)
            key = (r["kind"], r["M"], r["K"], r["N"])
            rows.setdefault(key, {})[f.stem] = r["us"]
            rows[key]["blas"] = r["blas_us"]
            rows[key]["calls"] = r["calls"]
cols.append("blas")
print("%-28s" % "shape" + "".join("%16s" % c[-16:] for c in cols))
for key, v in rows.items():
    print("%-28s" % ("%s %dx%dx%d" % key) + "".join("%16s" % (v.get(c, "")) for c in cols))
