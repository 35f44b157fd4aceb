"""CPU ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package recommendsystem_amd/).

A numpy restatement of the reference's CTR feature-interaction path, written line by line from
the cited reference sources, in float64 by default (pass dtype=np.float32 for fp32 runs).

PARITY STATUS: UNPINNED.  The reference (TensorFlow/Keras + tensornet model plugins) cannot be
imported or run here: TensorFlow, keras and tensornet are absent (ordinary ModuleNotFoundError,
nothing was refused), the hot-path modules also import files missing from the reference
(layer_normalization, common_module.*, src.*), and the reference ships no tests, fixtures or
golden vectors.  This oracle is therefore an independent restatement; the
golden fixtures under tests/golden/ are generated FROM it (tests/golden/make_golden.py) and pin
regressions, not the reference.  Decisions the reference leaves open are pinned and documented
(DESIGN.md "Pinned decisions"): keras-layer-normalization LN (eps 1e-14), MultiLayerDense =
Dense(u, act) per unit, the id->row hash, the dropout mask, the tensornet optimizer forms.
"""
from __future__ import annotations

import numpy as np

U64 = np.uint64
MASK64 = (1 << 64) - 1


# ------------------------------------------------------------------------------------------
# hashing (tensornet category_column id -> row; pinned, see csrc/embedding.hip)
# ------------------------------------------------------------------------------------------
def splitmix64(z: np.ndarray) -> np.ndarray:
    """SplitMix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + U64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> U64(30))) * U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> U64(27))) * U64(0x94D049BB133111EB)
        return z ^ (z >> U64(31))


def hash_rows(ids: np.ndarray, fields: np.ndarray, row_base, bucket, mode: str = "mod") -> np.ndarray:
    """row = row_base[f] + H(id) % bucket[f]; H = identity ('mod') or splitmix64 ('splitmix').
    ids are int64 reinterpreted as uint64 (two's complement), as in the kernel."""
    u = np.asarray(ids, dtype=np.int64).view(np.uint64)
    if mode == "splitmix":
        u = splitmix64(u)
    rb = np.asarray(row_base, dtype=np.int64)[fields]
    bk = np.asarray(bucket, dtype=np.uint64)[fields]
    return (rb + (u % bk).astype(np.int64)).astype(np.int64)


def embedding_lookup(ids, offsets, B, F, row_base, bucket, table, mode="mod", combiner="mean"):
    """EmbeddingFeatures + embedding_column(combiner) + expand/Concatenate(axis=1)
    (rank/ctr/base_model.py:203-217, autoint:22-26).  Returns (out [B, F, dim], rows [nnz])."""
    table = np.asarray(table)
    dim = table.shape[1]
    ids = np.asarray(ids, dtype=np.int64).reshape(-1)
    if offsets is None:
        offsets = np.arange(B * F + 1, dtype=np.int64)
    offsets = np.asarray(offsets, dtype=np.int64)
    seg_field = np.repeat(np.arange(B * F) % F, np.diff(offsets))
    rows = hash_rows(ids, seg_field, row_base, bucket, mode)
    out = np.zeros((B * F, dim), dtype=table.dtype)
    for s in range(B * F):
        a, b = offsets[s], offsets[s + 1]
        n = b - a
        if n == 0:
            continue
        acc = np.zeros(dim, dtype=table.dtype)
        for k in range(a, b):  # fp sum in id order
            acc = acc + table[rows[k]]
        if combiner == "mean":
            acc = acc / table.dtype.type(n)
        elif combiner == "sqrtn":
            acc = acc / np.sqrt(table.dtype.type(n))
        out[s] = acc
    return out.reshape(B, F, dim), rows


def combiner_scale(n: int, combiner: str, dtype=np.float64):
    if n <= 0:
        return dtype(0)
    if combiner == "mean":
        return dtype(1) / dtype(n)
    if combiner == "sqrtn":
        return dtype(1) / np.sqrt(dtype(n))
    return dtype(1)


def sparse_grad_sum(rows, offsets, B, F, dout, combiner="mean"):
    """Backward of the lookup as a tensornet push: {row: sum over its occurrences of
    scale(segment) * dout[segment]} summed in occurrence order."""
    dout = np.asarray(dout).reshape(B * F, -1)
    if offsets is None:
        offsets = np.arange(B * F + 1)
    out: dict[int, np.ndarray] = {}
    for s in range(B * F):
        a, b = int(offsets[s]), int(offsets[s + 1])
        sc = combiner_scale(b - a, combiner, dout.dtype.type)
        for k in range(a, b):
            r = int(rows[k])
            g = dout[s] * sc
            out[r] = out[r] + g if r in out else g.copy()
    return out


# ------------------------------------------------------------------------------------------
# Keras building blocks
# ------------------------------------------------------------------------------------------
def relu(x):
    return np.maximum(x, 0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


ACTS = {None: lambda x: x, "linear": lambda x: x, "relu": relu, "sigmoid": sigmoid}


def dense(x, W, b, activation=None):
    """tf.keras.layers.Dense: tensordot(x, W, [[rank-1], [0]]) + b, then activation."""
    return ACTS[activation](np.tensordot(x, W, axes=[[x.ndim - 1], [0]]) + b)


def layer_norm(x, gamma, beta, eps=1e-14):
    """keras-layer-normalization LayerNormalization.call (the module imported at
    InteractingLayer.py:4 is absent; pinned): mean/var over the last axis,
    (x - mean) / sqrt(var + eps) * gamma + beta."""
    mean = np.mean(x, axis=-1, keepdims=True)
    var = np.mean(np.square(x - mean), axis=-1, keepdims=True)
    std = np.sqrt(var + eps)
    return (x - mean) / std * gamma + beta


def dropout_keep(seed: int, b, h, i, j, rate: float) -> np.ndarray:
    """Counter-based dropout mask shared bit-for-bit with csrc/common.hpp::dropout_keep."""
    b = np.asarray(b, dtype=np.uint64)
    key = (U64(seed & MASK64) ^ ((b << U64(32)) | (np.asarray(h, np.uint64) << U64(24))
                                 | (np.asarray(i, np.uint64) << U64(12)) | np.asarray(j, np.uint64)))
    r = splitmix64(key)
    u = (r >> U64(40)).astype(np.float64) * (1.0 / 16777216.0)
    return u >= np.float32(rate)


def layer_seed(seed: int, it: int) -> int:
    return int(splitmix64(np.array([(seed + it) & MASK64], dtype=np.uint64))[0])


def softmax(x, axis=-1):
    """tf.nn.softmax: exp(x - max) * (1 / sum)."""
    e = np.exp(x - np.max(x, axis=axis, keepdims=True))
    return e * (1.0 / np.sum(e, axis=axis, keepdims=True))


# ------------------------------------------------------------------------------------------
# H3 InteractingLayer (InteractingLayer.py:37-61)
# ------------------------------------------------------------------------------------------
def interacting_layer(x, W, bias, gamma, beta, layer_num=1, head_num=1, use_res=True,
                      eps=1e-14, drop_rate=0.0, seed=0, return_inputs=False):
    """x [B, F, E]; W [E, 4U] = [Wq|Wk|Wv|Wr]; bias [4U]; gamma, beta [U]."""
    x = np.asarray(x)
    dt = x.dtype.type
    U = W.shape[1] // 4
    H = head_num
    Wq, Wk, Wv, Wr = (W[:, j * U:(j + 1) * U] for j in range(4))
    bq, bk, bv, br = (bias[j * U:(j + 1) * U] for j in range(4))
    if x.ndim != 3:  # :38-39
        raise ValueError("The rank of input of InteractingLayer must be 3, but now is %d" % x.ndim)
    output = x
    inputs = []
    B = x.shape[0]
    for it in range(layer_num):                                          # :41
        inputs.append(output)
        query = dense(output, Wq, bq, "relu")                           # :42
        key = dense(output, Wk, bk, "relu")                             # :43
        value = dense(output, Wv, bv, "relu")                           # :44
        if use_res:
            res = dense(output, Wr, br, "relu")                         # :45-46
        query = np.concatenate(np.split(query, H, axis=2), axis=0)     # :47  [H*B, F, dh]
        key = np.concatenate(np.split(key, H, axis=2), axis=0)         # :48
        value = np.concatenate(np.split(value, H, axis=2), axis=0)     # :49
        weight = np.matmul(query, np.transpose(key, [0, 2, 1]))        # :50
        weight = weight / dt(key.shape[-1] ** 0.5)                     # :51
        weight = softmax(weight)                                       # :52
        if drop_rate > 0.0:                                            # :53-54
            HB, Fq, Fk = weight.shape
            hh, bb = np.divmod(np.arange(HB), B)
            ii = np.arange(Fq)
            jj = np.arange(Fk)
            keep = dropout_keep(layer_seed(seed, it), bb[:, None, None], hh[:, None, None],
                                ii[None, :, None], jj[None, None, :], drop_rate)
            weight = np.where(keep, weight * dt(1.0 / (1.0 - drop_rate)), dt(0))
        output = np.matmul(weight, value)                              # :55
        output = np.concatenate(np.split(output, H, axis=0), axis=2)   # :56  [B, F, U]
        if use_res:
            output = output + res                                      # :57-58
        output = relu(output)                                          # :59
        output = layer_norm(output, gamma, beta, eps)                  # :60
    if return_inputs:
        return output, inputs
    return output


# ------------------------------------------------------------------------------------------
# H4/H10 AutoInt model (autoint:18-56) + cross_entropy (rank/ctr/base_model.py:7-12)
# ------------------------------------------------------------------------------------------
def mlp(x, layers, activation):
    """MultiLayerDense (pinned): Dense(u, activation) for each (W, b) in order."""
    for W, b in layers:
        x = dense(x, W, b, activation)
    return x


def autoint_forward(x0, il, deep_layers, logit_layers, cfg):
    """x0: concatenated field embeddings [B, F, E] (autoint:22-26).  Returns (s, p) where s is the
    logits MLP output before the clip and p = clip_by_value(s, 1e-6, 1.0) (autoint:52)."""
    B = x0.shape[0]
    y = interacting_layer(x0, il["W"], il["bias"], il["gamma"], il["beta"],
                          layer_num=cfg["layer_num"], head_num=cfg["head_num"],
                          use_res=cfg["use_res"], eps=cfg.get("ln_eps", 1e-14))    # :30-35
    autoint_out = y.reshape(B, -1)                                                  # :36
    deep = mlp(x0.reshape(B, -1), deep_layers, cfg["mlp_activation"])               # :39-41
    result = np.concatenate([deep, autoint_out], axis=1)                            # :44
    s = mlp(result, logit_layers, cfg["logits_activation"])                         # :48-50
    p = np.clip(s, 1e-6, 1.0)                                                       # :52
    return s, p


def cross_entropy(y_true, y_pred, a=1):
    """rank/ctr/base_model.py:7-12: mean over the batch of the per-row sum over axis 1."""
    y_true = np.asarray(y_true, dtype=y_pred.dtype)
    loss = -y_true * np.log(y_pred + 1e-6) - (a - y_true) * np.log(1.0 - y_pred + 1e-6)
    return np.mean(np.sum(loss, axis=1), axis=0)


# ------------------------------------------------------------------------------------------
# H11 optimizers (forms pinned in csrc/optim.hip)
# ------------------------------------------------------------------------------------------
def adam_dense(p, g, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-8):
    """tf.keras / tensornet dense Adam with bias correction at step t (1-based)."""
    lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    return p - lr_t * m / (np.sqrt(v) + eps), m, v


def adam_sparse(w, g, m, v, lr, b1=0.9, b2=0.999, eps=1e-8):
    """tensornet SparseAdamValue form: no bias correction."""
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    return w - lr * m / (eps + np.sqrt(v)), m, v


def adagrad_sparse(w, g, g2, lr):
    g2 = g2 + g * g
    return w - lr * g / np.sqrt(g2), g2
