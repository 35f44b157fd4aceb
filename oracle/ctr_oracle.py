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


def fmix32(h):
    """murmur3 32-bit finaliser on uint32 arrays (wrapping arithmetic)."""
    h = np.asarray(h, dtype=np.uint32)
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        return h ^ (h >> np.uint32(16))


def dropout_keep(seed: int, b, h, i, j, rate: float) -> np.ndarray:
    """Counter-based dropout mask shared bit-for-bit with csrc/common.hpp::dropout_keep:
    kb = fmix32(lo32(seed) ^ fmix32(hi32(seed) + b)); one draw per key pair
    r = fmix32(kb ^ (h<<24 | i<<12 | (j & ~1))); keep iff half / 2^16 >= rate with
    half = r & 0xFFFF for even j, r >> 16 for odd j."""
    seed = int(seed) & MASK64
    lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)
    with np.errstate(over="ignore"):
        kb = fmix32(lo ^ fmix32(hi + np.asarray(b, dtype=np.uint32)))
    jj = np.asarray(j, np.uint32)
    ctr = ((np.asarray(h, np.uint32) << np.uint32(24)) | (np.asarray(i, np.uint32) << np.uint32(12))
           | (jj & np.uint32(0xFFFFFFFE)))
    r = fmix32(kb ^ ctr)
    half = np.where((jj & np.uint32(1)) != 0, r >> np.uint32(16), r & np.uint32(0xFFFF))
    u = half.astype(np.float64) * (1.0 / 65536.0)
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


# ------------------------------------------------------------------------------------------
# N2 owner-sharded tables (owner = row % N; tensornet's PS split its tables by
# key on the host, rank/ctr/base_model.py:89-102).  Pinned routing of csrc/sharded.hip.
# ------------------------------------------------------------------------------------------
def owner_route(rows, world: int, table_rows: int):
    """rows int [n] (-1 or >= table_rows: no row) -> (send_local, send_pos, counts): the valid
    rows stably ordered by owner (row % world), local index row // world, original position, and
    the per-owner counts."""
    rows = np.asarray(rows, dtype=np.int64)
    pos = np.arange(rows.size)
    ok = (rows >= 0) & (rows < table_rows)
    key = np.where(ok, rows % world, world)
    order = np.argsort(key, kind="stable")
    order = order[ok[order]]
    counts = np.bincount(key[ok], minlength=world)[:world]
    return (rows[order] // world).astype(np.int32), pos[order].astype(np.int32), counts.astype(np.int32)


def owner_route_fixed(rows, world: int, table_rows: int, cap: int):
    """The fixed-capacity route (rs_owner_route_fixed; the sync-free form of owner_route, no
    reference counterpart -- tensornet's PS client sends variable-size requests): owner w's k-th
    valid row (owner_route's stable order) goes to slot w * cap + k if k < cap.
    -> (send_local [world * cap] int32 (row // world, -1 pads), slot [n] int32 (-1: invalid row or
    past its owner's cap), peak = the largest per-owner count)."""
    rows = np.asarray(rows, dtype=np.int64)
    send_local, send_pos, counts = owner_route(rows, world, table_rows)
    out = np.full(world * cap, -1, dtype=np.int32)
    slot = np.full(rows.size, -1, dtype=np.int32)
    i = 0
    for w in range(world):
        for k in range(int(counts[w])):
            if k < cap:
                out[w * cap + k] = send_local[i]
                slot[send_pos[i]] = w * cap + k
            i += 1
    return out, slot, int(counts.max()) if counts.size else 0


def sharded_lookup_reference(rows_per_rank, world: int, table_rows: int, table):
    """Every rank's per-id rows gathered through the owners (what the route + all-to-all + gather
    + scatter sequence computes): table[rows] with zero rows where rows < 0."""
    out = []
    for rows in rows_per_rank:
        rows = np.asarray(rows, dtype=np.int64)
        e = np.zeros((rows.size, table.shape[1]), dtype=table.dtype)
        ok = (rows >= 0) & (rows < table_rows)
        e[ok] = table[rows[ok]]
        out.append(e)
    return out


# ------------------------------------------------------------------------------------------
# H1 sequence lookup (tn embedding_column(combiner=None, seq_max_len) -> (emb3d, mask);
# staytime/VideoDnn.py:217-244, consumed at :58-68).  Pinned: the first seq_max_len ids of a
# sample are kept, positions past the sample's length are zero rows with mask False.
# ------------------------------------------------------------------------------------------
def sequence_lookup(ids, offsets, B, T, row_base, bucket, table, mode="mod"):
    """ids [nnz] int64, offsets [B+1]; returns (emb [B, T, dim], mask [B, T] bool,
    rows [B, T] int64 with -1 at padded positions)."""
    table = np.asarray(table)
    offsets = np.asarray(offsets, dtype=np.int64)
    ids = np.asarray(ids, dtype=np.int64).reshape(-1)
    emb = np.zeros((B, T, table.shape[1]), dtype=table.dtype)
    mask = np.zeros((B, T), dtype=bool)
    rows = np.full((B, T), -1, dtype=np.int64)
    for b in range(B):
        n = min(int(offsets[b + 1] - offsets[b]), T)
        if n == 0:
            continue
        r = hash_rows(ids[offsets[b]:offsets[b] + n], np.zeros(n, dtype=np.int64), [row_base],
                      [bucket], mode)
        rows[b, :n] = r
        emb[b, :n] = table[r]
        mask[b, :n] = True
    return emb, mask, rows


# ------------------------------------------------------------------------------------------
# H6 DIN (din.py:18-47): ReLU-MLP scores, masked to zero, no softmax, weighted sum of values.
# ------------------------------------------------------------------------------------------
def sequence_mask(lengths, maxlen=None):
    """tf.sequence_mask: maxlen defaults to max(lengths) (din.py:24)."""
    lengths = np.asarray(lengths)
    if maxlen is None:
        maxlen = int(lengths.max()) if lengths.size else 0
    return np.arange(maxlen)[None, :] < lengths[:, None]


def din_pool(queries, keys, values, seq_length, W1, b1, W2, b2):
    """queries [B, H], keys/values [B, T, H], seq_length [B] (None = no mask); W1 [3H, 16],
    b1 [16], W2 [16, 1], b2 [1] (din_nn_0 / din_nn_1, both relu, din.py:12-15)."""
    q = np.expand_dims(queries, axis=1)                                   # :19  [B, 1, H]
    from_len, to_len = q.shape[1], keys.shape[1]                          # :21-22
    q = np.expand_dims(q, axis=2)                                         # :26  [B, 1, 1, H]
    k = np.expand_dims(keys, axis=1)                                      # :27  [B, 1, T, H]
    q = np.tile(q, [1, 1, to_len, 1])                                     # :28
    k = np.tile(k, [1, from_len, 1, 1])                                   # :29
    deep = np.concatenate([q, k, q * k], axis=-1)                         # :31  [B, 1, T, 3H]
    deep = dense(deep, W1, b1, "relu")                                    # :33-34
    deep = dense(deep, W2, b2, "relu")
    deep = np.squeeze(deep, axis=-1)                                      # :37  [B, 1, T]
    if seq_length is not None:
        masks = sequence_mask(seq_length, to_len)                         # :24 (maxlen = T)
        masks = np.tile(np.expand_dims(masks, 1), [1, from_len, 1])       # :40-41
        deep = np.where(masks, deep, np.zeros_like(deep))                 # :42
    out = np.matmul(deep, values)                                         # :44  [B, 1, H]
    return np.squeeze(out, 1)                                             # :45


# ------------------------------------------------------------------------------------------
# H7 staytime DIN (staytime/layer.py:16-41): [q, f, q-f, q*f] -> Dense(16, sigmoid) ->
# Dense(1) -> masked (-2**32+1) softmax over T -> weighted sum of facts.
# ------------------------------------------------------------------------------------------
DIN_PAD = -2.0 ** 32 + 1


def din_softmax_pool(query, facts, mask, W1, b1, W2, b2, return_probs=False):
    """query [B, H], facts [B, T, H], mask [B, >=T] bool (None = no mask); W1 [4H, 16], b1 [16],
    W2 [16, 1], b2 [1]."""
    B, T, H = facts.shape
    dt = facts.dtype.type
    queries = np.tile(query, [1, T]).reshape(facts.shape)                 # :20-21
    din_all = np.concatenate([queries, facts, queries - facts, queries * facts], axis=-1)  # :22-23
    d1 = dense(din_all, W1, b1, "sigmoid")                                # :24
    d2 = dense(d1, W2, b2, None)                                          # :25
    scores = d2.reshape(-1, 1, T)                                         # :26-27
    if mask is not None:
        key_masks = np.expand_dims(np.asarray(mask)[:, :T], 1)            # :30-31
        paddings = np.ones_like(scores) * dt(DIN_PAD)                     # :32
        scores = np.where(key_masks, scores, paddings)                    # :34
    probs = softmax(scores)                                               # :35
    out = np.matmul(probs, facts)                                         # :36
    out = np.squeeze(out, 1)                                              # :40
    if return_probs:
        return out, probs[:, 0, :]
    return out


# ------------------------------------------------------------------------------------------
# N1  staytime parse_input_func labels (staytime/parse.py:16-71), fp32 in the TF graph's op order
# ------------------------------------------------------------------------------------------
STAYTIME_LANDING_RE = r".*video_homepage_landing.*"                       # parse.py:64


def staytime_parse_labels(watch_ms, extra_info, bins, sigma=4, left=-19, right=180.5):
    """watch_ms int64 [B], extra_info list of str [B], bins [nbins] (config.py:18 bin_list) ->
    (staytime_label [B, nbins + 1] f32, short [B] f32, long [B] f32, sample_weight [B] f32).
    Each step is one fp32 TF op, in order; the Python-float constants become fp32 tensors."""
    import math
    import re
    f32 = np.float32
    wt_i = np.asarray(watch_ms, dtype=np.int64)
    short = np.where(wt_i > 7000, 1, 0).astype(f32)                      # :31-34
    long_ = np.where(wt_i > 18000, 1, 0).astype(f32)                     # :37-38
    wt = wt_i.astype(f32)                                                 # :40
    wt = np.divide(wt, f32(1000.0))                                       # :41
    wt = np.where(wt > f32(160.0), f32(160.0), wt).astype(f32)            # :42
    b = np.asarray(bins, dtype=f32)[None, :]                              # :45-46
    dist = np.subtract(b, wt[:, None])                                    # :48-52
    sq = np.square(np.abs(dist))                                          # :53
    nb = b.shape[1]
    width = (right - left) / (nb - 1)                                     # :55-57
    div_num = f32(math.sqrt(2 * math.pi) * sigma)                         # :59
    label = np.divide(np.exp(np.divide(sq, f32(-2 * math.pow(sigma, 2)))), div_num)  # :60
    label = np.multiply(label, f32(width))                                # :61
    stay = np.concatenate([label, wt[:, None]], -1).astype(f32)           # :62
    pat = re.compile(STAYTIME_LANDING_RE)
    sw = np.array([5.0 if pat.fullmatch(s) else 1.0 for s in extra_info], dtype=f32)  # :64
    return stay, short, long_, sw


def keras_auc(p, y, w=None, num_thresholds=200):
    """tf.keras.metrics.AUC() (defaults: ROC, summation 'interpolation') as its update_state /
    result compute it, in numpy (Keras thresholds: [-1e-7, i / (n - 1) for i = 1 .. n - 2,
    1 + 1e-7] as fp32; a prediction is positive at t when p > t; y cast to bool); the metric sites
    are rank/ctr/base_model.py:183-190, rough_rank/model.py:215-219, rank/multi_head/model.py:55.
    Accumulated in float64 (Keras keeps fp32 variables; equal for unit weights below 2^24)."""
    p = np.asarray(p, dtype=np.float32).reshape(-1)
    y = np.asarray(y).reshape(-1) != 0
    w = np.ones_like(p, dtype=np.float64) if w is None else np.asarray(w, dtype=np.float64).reshape(-1)
    n = num_thresholds
    thr = np.array([-1e-7] + [(i + 1) / (n - 1) for i in range(n - 2)] + [1.0 + 1e-7],
                   dtype=np.float32)
    above = p[None, :] > thr[:, None]                     # [n, B]
    tp = (above & y[None, :]).astype(np.float64) @ w
    fp = (above & ~y[None, :]).astype(np.float64) @ w
    P, N = float(w[y].sum()), float(w[~y].sum())
    tpr = tp / P if P > 0 else np.zeros(n)
    fpr = fp / N if N > 0 else np.zeros(n)
    return float(np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2.0))


def ctr_metrics(p, y, w=None):
    """Binary accuracy (threshold 0.5, Keras 'acc' on a one-unit output), COPC = sum(w y) / sum(w p)
    and CTR = sum(w y) / sum(w) (tensornet tn.metric.COPC / CTR: not vendored, pinned forms)."""
    p = np.asarray(p, dtype=np.float64).reshape(-1)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    w = np.ones_like(p) if w is None else np.asarray(w, dtype=np.float64).reshape(-1)
    correct = (y == (p.astype(np.float32) > np.float32(0.5)).astype(np.float64))
    return {"auc": keras_auc(p, y, w), "acc": float((w * correct).sum() / w.sum()),
            "copc": float((w * y).sum() / (w * p).sum()), "ctr": float((w * y).sum() / w.sum()),
            "pctr": float((w * p).sum() / w.sum())}
