"""Time the sequence-history push at the config-4 DIN shape (B = 1024, T = 100, 1M x 16 table,
Zipf(1.2) ids, lengths uniform 0..T): the push as [B, T] "fields" (what SequenceEmbedding's
backward launches), flattened to [B*T, 1], and the deterministic sorted variant; each launch is
timed alone with the sparse optimizer run in between (flags and gradient rows reset as in a step)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd.embedding import SparseAdam, SparseTable


def main(B=1024, T=100, dim=16, vocab=1_000_000, reps=30):
    _lib.load()
    dev = torch.device("cuda")
    t = SparseTable(vocab, dim, SparseAdam(1e-3), device=dev, seed=0, max_touched=B * T)
    rng = np.random.default_rng(0)
    lens = rng.integers(0, T + 1, size=B)
    ids = np.minimum(rng.zipf(1.2, size=(B, T)) - 1, vocab - 1)
    ids[np.arange(T)[None, :] >= lens[:, None]] = -1
    rows = torch.from_numpy(ids.astype(np.int32).reshape(-1)).to(dev)
    dout = torch.randn(B, T, dim, device=dev)
    variants = {
        "fields_BxT": lambda: t.accumulate(rows, None, B, T, dout, T * dim, dim, 0),
        "flat_BTx1": lambda: t.accumulate(rows, None, B * T, 1, dout, dim, dim, 0),
    }

    def sorted_push():
        t.deterministic = True
        t.accumulate(rows, None, B * T, 1, dout, dim, dim, 0)
        t.deterministic = False
    t.sorted_workspace(B * T)
    variants["sorted"] = sorted_push
    out = {"valid_ids": int((ids >= 0).sum()), "unique_rows": int(len(np.unique(ids[ids >= 0])))}
    for name, fn in variants.items():
        fn(); t.step(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tot = 0.0
        for _ in range(reps):
            e0.record(); fn(); e1.record(); torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
            t.step(); torch.cuda.synchronize()
        out[name + "_us"] = round(tot / reps * 1e3, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
