"""Per-kernel instruction-class counts of a hipcc --save-temps gfx950 .s file.

    python tools/isa_stats.py file.s [name-substring]
"""
import re
import sys

CLASSES = [("scratch", r"scratch_"), ("v_pk_fma", r"v_pk_fma_f32"), ("v_fma", r"v_fmac?_f32"),
           ("mfma", r"v_mfma"), ("ds_read", r"ds_read"), ("ds_write", r"ds_write"),
           ("s_barrier", r"s_barrier"), ("glds", r"global_load_lds"), ("vmcnt(0)", r"vmcnt\(0\)"),
           ("gload", r"global_load_dword"), ("atomic", r"global_atomic"), ("exp", r"v_exp_f32")]


def main(path, sub=""):
    s = open(path).read()
    meta = {m.group(1): (m.group(2), m.group(3), m.group(4)) for m in re.finditer(
        r"\.name:\s+(\S+).*?\.private_segment_fixed_size:\s+(\d+).*?\.sgpr_count:\s+(\d+).*?"
        r"\.vgpr_count:\s+(\d+)", s, re.S)}
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
    for k, (pos, name) in enumerate(starts):
        if sub not in name:
            continue
        end = s.find(".Lfunc_end", pos)
        body = s[pos:end]
        cnt = " ".join(f"{n}={len(re.findall(p, body))}" for n, p in CLASSES)
        priv, sg, vg = meta.get(name, ("?", "?", "?"))
        print(f"{name[:70]}\n   vgpr={vg} sgpr={sg} private={priv} {cnt}")


if __name__ == "__main__":
    main(*sys.argv[1:])
