"""Time rs_sparse_grad_accumulate + rs_sparse_adam alone at config-2 shape (B=4096, F=26, dim 16)
for several id distributions (Zipf(1.2) as in bench.py, uniform, all-one-row)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle
from recommendsystem_amd.embedding import SparseTable, SparseAdam


def main(B=4096, F=26, dim=16, vocab=100_000, reps=30):
    _lib.load()
    dev = torch.device("cuda")
    t = SparseTable(F * vocab, dim, SparseAdam(1e-3), device=dev, seed=0, max_touched=B * F)
    rng = np.random.default_rng(0)
    dout = torch.randn(B, F * dim, device=dev)
    out = {}
    for name, ids in (("zipf", np.minimum(rng.zipf(1.2, size=(B, F)) - 1, vocab - 1)),
                      ("uniform", rng.integers(0, vocab, size=(B, F))),
                      ("one_row", np.zeros((B, F), dtype=np.int64))):
        rows = torch.from_numpy((ids + np.arange(F)[None, :] * vocab).astype(np.int32).reshape(-1)).to(dev)
        s = stream_handle()
        acc = lambda: call("rs_sparse_grad_accumulate", s, ptr(rows), None, B, F, ptr(dout), F * dim,
                           dim, dim, 0, ptr(t.grad), ptr(t.flag), ptr(t.touched), ptr(t.n_touched),
                           t.touched_cap)
        step = lambda: t.step()
        for fn in (acc, step):
            fn()
        torch.cuda.synchronize()
        res = {}
        for k, fn in (("accum_us", acc), ("adam_us", step)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            tot = 0.0
            for _ in range(reps):
                if k == "accum_us":
                    e0.record(); acc(); e1.record(); torch.cuda.synchronize(); tot += e0.elapsed_time(e1)
                    step(); torch.cuda.synchronize()
                else:
                    acc(); torch.cuda.synchronize()
                    e0.record(); step(); e1.record(); torch.cuda.synchronize(); tot += e0.elapsed_time(e1)
            res[k] = round(tot / reps * 1e3, 2)
        res["unique_rows"] = int(len(np.unique(rows.cpu().numpy())))
        out[name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
