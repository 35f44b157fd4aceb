"""Generate the committed golden fixtures (small .npz vectors) FROM THE CPU ORACLE.

The reference (TF/Keras + tensornet) cannot run here and ships no fixtures, so
these vectors pin the oracle and the HIP kernels against regressions; they are not reference
outputs (parity unpinned, see oracle/ctr_oracle.py).  Re-run with
    python tests/golden/make_golden.py
Every input is drawn from numpy.random.default_rng with the seed stored in the file.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ctr_oracle as npo  # noqa: E402


def glorot(rng, fan_in, fan_out, shape=None):
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape or (fan_in, fan_out))


def il_case(seed, B, F, E, U, H, L, res, drop=0.0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-0.5, 0.5, size=(B, F, E)).astype(np.float32)
    W = np.concatenate([glorot(rng, E, U) for _ in range(4)], axis=1).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, size=4 * U).astype(np.float32)
    g = rng.uniform(0.5, 1.5, size=U).astype(np.float32)
    be = rng.uniform(-0.2, 0.2, size=U).astype(np.float32)
    y = npo.interacting_layer(x.astype(np.float64), W.astype(np.float64), b.astype(np.float64),
                              g.astype(np.float64), be.astype(np.float64), L, H, res,
                              drop_rate=drop, seed=seed)
    return dict(seed=seed, x=x, W=W, bias=b, gamma=g, beta=be, y=y,
                shape=np.array([B, F, E, U, H, L, int(res)]), drop=np.float64(drop))


def autoint_case(seed, B=8, F=26, E=16, vocab=97):
    rng = np.random.default_rng(seed)
    table = rng.uniform(-0.05, 0.05, size=(F * vocab, E)).astype(np.float32)
    ids = rng.integers(0, 10 ** 6, size=(B, F), dtype=np.int64)
    labels = (rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)
    row_base = np.arange(F, dtype=np.int64) * vocab
    bucket = np.full(F, vocab, dtype=np.int64)
    x0, rows = npo.embedding_lookup(ids, None, B, F, row_base, bucket, table.astype(np.float64))
    U, H, L = 16, 2, 3
    W = np.concatenate([glorot(rng, E, U) for _ in range(4)], axis=1).astype(np.float32)
    il = dict(W=W, bias=np.zeros(4 * U, np.float32), gamma=np.ones(U, np.float32),
              beta=np.zeros(U, np.float32))
    W1, W2 = glorot(rng, F * E, 32).astype(np.float32), glorot(rng, 32, 16).astype(np.float32)
    W3 = glorot(rng, 16 + F * U, 1).astype(np.float32)
    deep = [(W1, np.zeros(32, np.float32)), (W2, np.zeros(16, np.float32))]
    logits = [(W3, np.zeros(1, np.float32))]
    cfg = dict(layer_num=L, head_num=H, use_res=True, mlp_activation="relu",
               logits_activation="sigmoid")
    il64 = {k: v.astype(np.float64) for k, v in il.items()}
    s, p = npo.autoint_forward(x0, il64, [(a.astype(np.float64), c.astype(np.float64)) for a, c in deep],
                               [(a.astype(np.float64), c.astype(np.float64)) for a, c in logits], cfg)
    loss = npo.cross_entropy(labels.astype(np.float64), p)
    return dict(seed=seed, table=table, ids=ids, labels=labels, row_base=row_base, bucket=bucket,
                rows=rows, x0=x0, il_W=W, W1=W1, W2=W2, W3=W3, s=s, p=p, loss=np.float64(loss))


def lookup_case(seed, B=9, F=4, dim=8, vocab=31):
    rng = np.random.default_rng(seed)
    table = rng.normal(size=(F * vocab, dim)).astype(np.float32)
    lens = rng.integers(0, 4, size=B * F)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ids = rng.integers(-(1 << 62), 1 << 62, size=int(offsets[-1]), dtype=np.int64)
    row_base = np.arange(F, dtype=np.int64) * vocab
    bucket = np.full(F, vocab, dtype=np.int64)
    out = {}
    for mode in ("mod", "splitmix"):
        for comb in ("mean", "sum", "sqrtn"):
            o, rows = npo.embedding_lookup(ids, offsets, B, F, row_base, bucket,
                                           table.astype(np.float64), mode, comb)
            out[f"out_{mode}_{comb}"] = o
            out[f"rows_{mode}"] = rows
    dout = rng.normal(size=(B, F, dim))
    g = npo.sparse_grad_sum(out["rows_mod"], offsets, B, F, dout, "mean")
    keys = np.array(sorted(g), dtype=np.int64)
    return dict(seed=seed, table=table, ids=ids, offsets=offsets, row_base=row_base, bucket=bucket,
                dout=dout, grad_rows=keys, grad_vals=np.stack([g[k] for k in keys]), **out)


def din_case(seed, variant, B=6, T=9, H=16):
    rng = np.random.default_rng(seed)
    q = rng.uniform(-0.5, 0.5, size=(B, H)).astype(np.float32)
    k = rng.uniform(-0.5, 0.5, size=(B, T, H)).astype(np.float32)
    nb = 3 if variant == 0 else 4
    W1 = glorot(rng, nb * H, 16).astype(np.float32)
    b1 = rng.uniform(-0.1, 0.1, size=16).astype(np.float32)
    W2 = glorot(rng, 16, 1).astype(np.float32)
    b2 = np.array([0.05], dtype=np.float32)
    f64 = lambda a: a.astype(np.float64)
    if variant == 0:
        v = rng.uniform(-0.5, 0.5, size=(B, T, H)).astype(np.float32)
        lens = rng.integers(0, T + 1, size=B).astype(np.int32)
        lens[0] = T
        out = npo.din_pool(f64(q), f64(k), f64(v), lens, f64(W1), f64(b1), f64(W2), f64(b2))
        return dict(seed=seed, q=q, keys=k, values=v, lengths=lens, W1=W1, b1=b1, W2=W2, b2=b2, out=out)
    mask = rng.uniform(size=(B, T)) < 0.6
    mask[1] = False
    out, probs = npo.din_softmax_pool(f64(q), f64(k), mask, f64(W1), f64(b1), f64(W2), f64(b2),
                                      return_probs=True)
    return dict(seed=seed, q=q, facts=k, mask=mask, W1=W1, b1=b1, W2=W2, b2=b2, out=out, probs=probs)


def seq_case(seed, B=7, T=5, dim=8, vocab=23):
    rng = np.random.default_rng(seed)
    table = rng.normal(size=(vocab, dim)).astype(np.float32)
    lens = rng.integers(0, T + 3, size=B)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ids = rng.integers(-(1 << 62), 1 << 62, size=int(offsets[-1]), dtype=np.int64)
    emb, mask, rows = npo.sequence_lookup(ids, offsets, B, T, 0, vocab, table.astype(np.float64),
                                          "splitmix")
    return dict(seed=seed, table=table, ids=ids, offsets=offsets, T=np.int64(T), emb=emb, mask=mask,
                rows=rows)


def main():
    os.makedirs(HERE, exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "il_config2.npz"), **il_case(101, 4, 26, 16, 16, 2, 3, True))
    np.savez_compressed(os.path.join(HERE, "il_defaults_u128.npz"), **il_case(102, 2, 26, 16, 128, 1, 1, True))
    np.savez_compressed(os.path.join(HERE, "il_dropout.npz"), **il_case(103, 3, 26, 16, 16, 2, 2, True, 0.2))
    np.savez_compressed(os.path.join(HERE, "il_multihead_u8.npz"), **il_case(104, 3, 19, 8, 8, 2, 1, True))
    np.savez_compressed(os.path.join(HERE, "autoint_config2.npz"), **autoint_case(105))
    np.savez_compressed(os.path.join(HERE, "lookup_ragged.npz"), **lookup_case(106))
    np.savez_compressed(os.path.join(HERE, "din_relu_sum.npz"), **din_case(107, 0))
    np.savez_compressed(os.path.join(HERE, "din_staytime_softmax.npz"), **din_case(108, 1))
    np.savez_compressed(os.path.join(HERE, "sequence_lookup.npz"), **seq_case(109))
    np.savez_compressed(os.path.join(HERE, "splitmix64_kat.npz"),
                        # SplitMix64 generator seeded with 0: outputs k = mix(state + gamma) with
                        # state = k * gamma; our finaliser adds gamma itself, so the inputs are
                        # k * gamma.  Published known answers for the first three outputs:
                        seeds=np.array([0, 0x9E3779B97F4A7C15, 0x3C6EF372FE94F82A], dtype=np.uint64),
                        expect=np.array([0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4,
                                         0x06C45D188009454F], dtype=np.uint64))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
