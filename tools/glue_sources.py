"""Where do the torch (non-librecsys) kernels of a workload step come from?  One eager training
step under torch.profiler (with Python stacks); prints every aten op that launched GPU work with
its count and the innermost recommendsystem_amd / bench frame that called it.

    python tools/glue_sources.py staytime|din|multi_head [batch]
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def build(name, B, dev):
    from recommendsystem_amd import workloads as W
    from recommendsystem_amd.models import MultiHeadConfig, MultiHeadRanker
    from recommendsystem_amd.trainer import Trainer
    rng = np.random.default_rng(0)
    if name == "multi_head":
        m = MultiHeadRanker(MultiHeadConfig(), device=dev, seed=0)
        return Trainer(m, 1e-5, m.tables()), W.multi_head_batch(rng, B, m.cfg, dev)
    if name == "din":
        m = W.DINPool(device=dev, seed=0)
        return Trainer(m, 5e-5, [m.table]), W.din_batch(rng, B, 100, 1_000_000, dev)
    m = W.StaytimeRoughRank(device=dev, seed=0, rows=1_000_000)
    return (Trainer(m, 5e-4, [m.table], lr_groups=[(m.dssm, m.rr_cfg.lr_dense)]),
            W.staytime_batch(rng, B, m, dev))


def main(name="staytime", B=512):
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    dev = torch.device("cuda")
    trn, batch = build(name, int(B), dev)
    trn.step(*batch)
    torch.cuda.synchronize()
    cnt = collections.Counter()
    skip = ("aten::empty", "aten::view", "aten::_unsafe_view", "aten::as_strided", "aten::t",
            "aten::detach", "aten::alias", "aten::reshape", "aten::slice", "aten::select",
            "aten::expand", "aten::unsqueeze", "aten::squeeze", "aten::permute", "aten::transpose",
            "aten::split", "aten::split_with_sizes", "aten::unbind", "aten::new_empty",
            "aten::empty_like", "aten::lift_fresh", "aten::_to_copy", "aten::item",
            "aten::_local_scalar_dense", "aten::is_nonzero", "aten::set_", "aten::empty_strided")

    class Spy(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            nm = "aten::" + func.__name__.split(".")[0]
            if nm not in skip:
                frame = "autograd engine / torch internals"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    f = fr.filename
                    if "recommendsystem_amd" in f or "bench.py" in f:
                        frame = f"{f.split('recommendsystem_amd/')[-1]}:{fr.lineno} {fr.name}"
                        break
                cnt[(nm, frame)] += 1
            return func(*args, **(kwargs or {}))

    with Spy():
        trn.step(*batch)
        torch.cuda.synchronize()
    for (op, fr), n in sorted(cnt.items(), key=lambda x: -x[1]):
        print(f"{n:4d}  {op:28s} {fr}")


if __name__ == "__main__":
    main(*sys.argv[1:])
