"""CPU ORACLE (autograd twin) — test infrastructure only; see oracle/ctr_oracle.py for status.

The same TF-semantics restatement as ctr_oracle.py, written with torch CPU ops op-for-op
(split/concat head shuffles, materialised [H*B, F, F] softmax, separate Dense/ReLU/LN ops), so
that:
  * torch autograd in float64 gives the reference gradients (TF's ReluGrad `x > 0`, ClipByValue
    pass-through inside [lo, hi] and SigmoidGrad are what torch's relu/clamp/sigmoid backward
    do), cross-checked against finite differences in tests/test_oracle.py;
  * run in float32 with all host threads it is the unfused TF-CPU-style train step that
    bench.py times as the CPU baseline ("kind": "port").
PARITY STATUS: UNPINNED (no runnable reference, no reference fixtures).
"""
from __future__ import annotations

import torch

from . import ctr_oracle as npo


def round_bf16(t):
    """Round to the nearest bf16 (ties to even) and back to t's dtype: the operand rounding of
    the library's bf16 math mode (v_cvt_pk_bf16_f32).  fp64 inputs are rounded via fp32 first,
    as the kernels hold fp32 values."""
    return t.to(torch.float32).to(torch.bfloat16).to(t.dtype)


class _Bf16MatMul(torch.autograd.Function):
    """x @ W with both operands rounded to bf16 (exact products, accumulation in x's dtype).
    bwd_round: the backward GEMMs round theirs too (dx = r(g) r(W)^T, dW = r(x)^T r(g)) -- what
    the library's MFMA backward does; False: exact backward (the head's VALU layer-2 backward)."""

    @staticmethod
    def forward(ctx, x, W, bwd_round):
        ctx.save_for_backward(x, W)
        ctx.bwd_round = bwd_round
        return torch.tensordot(round_bf16(x), round_bf16(W), dims=([x.dim() - 1], [0]))

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        r = round_bf16 if ctx.bwd_round else (lambda t: t)
        gr, xr, Wr = r(g), r(x), r(W)
        dx = torch.tensordot(gr, Wr, dims=([g.dim() - 1], [1]))
        dW = torch.tensordot(xr.reshape(-1, x.shape[-1]), gr.reshape(-1, g.shape[-1]),
                             dims=([0], [0]))
        return dx, dW, None


def dense(x, W, b, activation=None, bf16=None):
    """Keras Dense.  bf16: None (fp32/fp64 math), "fwd_bwd" or "fwd" (operand rounding of the
    library's bf16 math mode; see _Bf16MatMul)."""
    if bf16 is None:
        y = torch.tensordot(x, W, dims=([x.dim() - 1], [0])) + b
    else:
        y = _Bf16MatMul.apply(x, W, bf16 == "fwd_bwd") + b
    if activation == "relu":
        return torch.relu(y)
    if activation == "sigmoid":
        return torch.sigmoid(y)
    return y


def layer_norm(x, gamma, beta, eps=1e-14):
    mean = x.mean(dim=-1, keepdim=True)
    var = (x - mean).square().mean(dim=-1, keepdim=True)
    return (x - mean) / torch.sqrt(var + eps) * gamma + beta


def interacting_layer(x, W, bias, gamma, beta, layer_num=1, head_num=1, use_res=True, eps=1e-14,
                      drop_rate=0.0, seed=0, bf16=False, torch_mask=False):
    """InteractingLayer.py:37-61, op for op (tied weights across layer_num iterations).
    bf16: the projections round their operands as the library's bf16 math mode does (forward and
    backward GEMMs); attention, LN and everything else unchanged."""
    mm = "fwd_bwd" if bf16 else None
    U = W.shape[1] // 4
    H = head_num
    Wq, Wk, Wv, Wr = (W[:, j * U:(j + 1) * U] for j in range(4))
    bq, bk, bv, br = (bias[j * U:(j + 1) * U] for j in range(4))
    B = x.shape[0]
    out = x
    for it in range(layer_num):
        q = dense(out, Wq, bq, "relu", mm)
        k = dense(out, Wk, bk, "relu", mm)
        v = dense(out, Wv, bv, "relu", mm)
        res = dense(out, Wr, br, "relu", mm) if use_res else None
        q = torch.cat(torch.split(q, U // H, dim=2), dim=0)
        k = torch.cat(torch.split(k, U // H, dim=2), dim=0)
        v = torch.cat(torch.split(v, U // H, dim=2), dim=0)
        w = torch.matmul(q, k.transpose(1, 2))
        w = w / float((U // H) ** 0.5)
        w = torch.softmax(w, dim=-1)
        if drop_rate > 0.0 and torch_mask:  # CPU baseline: TF-style RNG mask (throughput only)
            w = torch.where(torch.rand_like(w) >= drop_rate, w * (1.0 / (1.0 - drop_rate)),
                            torch.zeros_like(w))
        elif drop_rate > 0.0:
            HB, Fq, Fk = w.shape
            hh, bb = divmod(torch.arange(HB).numpy(), B)
            keep = npo.dropout_keep(npo.layer_seed(seed, it), bb[:, None, None], hh[:, None, None],
                                    torch.arange(Fq).numpy()[None, :, None],
                                    torch.arange(Fk).numpy()[None, None, :], drop_rate)
            w = torch.where(torch.from_numpy(keep), w * (1.0 / (1.0 - drop_rate)), torch.zeros_like(w))
        o = torch.matmul(w, v)
        o = torch.cat(torch.split(o, B, dim=0), dim=2)
        if use_res:
            o = o + res
        o = torch.relu(o)
        out = layer_norm(o, gamma, beta, eps)
    return out


def interacting_layer_kinks(x, W, bias, gamma, beta, layer_num, head_num, use_res=True,
                            eps=1e-14, flips=()):
    """interacting_layer (InteractingLayer.py:37-61, no dropout) with the projection ReLUs
    written as z * mask so that single ReLU derivatives can be flipped.

    Returns (y, margins): margins[it] = |z| / (sum_e |x_e W_ec| + |b_c|) per [B, F, 4U]
    projection input of iteration it -- the distance of each ReLU input from its kink in units
    of the magnitude of the sum that forms it (fp32 rounding of that sum is ~6e-8 of it, plus
    the propagated fp32 difference of the iteration's input).  relu(O + R) has no kink to
    track: O and R are post-ReLU, so O + R >= 0.
    flips: (it, b, f, c) entries whose ReLU derivative is inverted (c indexes [Q|K|V|R])."""
    U = W.shape[1] // 4
    dh = U // head_num
    out, margins = x, []
    for it in range(layer_num):
        z = torch.tensordot(out, W, dims=([out.dim() - 1], [0])) + bias            # [B, F, 4U]
        scale = torch.tensordot(out.detach().abs(), W.detach().abs(),
                                dims=([out.dim() - 1], [0])) + bias.detach().abs()
        margins.append((z.detach().abs() / scale))
        keep = (z.detach() > 0).to(z.dtype)
        for (fi, b, f, c) in flips:
            if fi == it:
                keep[b, f, c] = 1.0 - keep[b, f, c]
        pr = z * keep
        q, k, v, r = (pr[..., j * U:(j + 1) * U] for j in range(4))
        heads = []
        for h in range(head_num):
            sl = slice(dh * h, dh * (h + 1))
            w = torch.softmax(q[..., sl] @ k[..., sl].transpose(1, 2) / float(dh ** 0.5), dim=-1)
            heads.append(w @ v[..., sl])
        o = torch.cat(heads, dim=-1)
        if use_res:
            o = o + r
        out = layer_norm(torch.relu(o), gamma, beta, eps)
    return out, margins


def mlp(x, layers, activation, bf16=None):
    """bf16: per-layer operand-rounding modes (see dense), or None."""
    for i, (W, b) in enumerate(layers):
        x = dense(x, W, b, activation, bf16[i] if bf16 else None)
    return x


def autoint_forward(x0, il, deep_layers, logit_layers, cfg):
    """cfg["bf16"]: the library's bf16 math mode -- IL projections rounded forward and backward;
    the fused head's deep layer 1 rounded forward and backward (MFMA dx0 / dW1), layer 2 forward
    only (its backward is fp32 VALU), logits exact (head.hip)."""
    B = x0.shape[0]
    bf = bool(cfg.get("bf16", False))
    y = interacting_layer(x0, il["W"], il["bias"], il["gamma"], il["beta"], cfg["layer_num"],
                          cfg["head_num"], cfg["use_res"], cfg.get("ln_eps", 1e-14), bf16=bf)
    deep_modes = (["fwd_bwd"] + ["fwd"] * (len(deep_layers) - 1)) if bf else None
    deep = mlp(x0.reshape(B, -1), deep_layers, cfg["mlp_activation"], deep_modes)
    result = torch.cat([deep, y.reshape(B, -1)], dim=1)
    s = mlp(result, logit_layers, cfg["logits_activation"])
    return s, torch.clamp(s, 1e-6, 1.0)


def cross_entropy(y_true, y_pred, a=1):
    y_true = y_true.to(y_pred.dtype)
    loss = -y_true * torch.log(y_pred + 1e-6) - (a - y_true) * torch.log(1.0 - y_pred + 1e-6)
    return torch.mean(torch.sum(loss, dim=1), dim=0)


class AutoIntCPU:
    """Unfused TF-CPU-style AutoInt train step: embedding gather (index_select + per-row sparse
    gradient), InteractingLayer x layer_num, deep + logits MLP, clip, cross_entropy, backward,
    dense Adam (bias-corrected) and sparse Adam on the touched rows (tensornet form)."""

    def __init__(self, table, row_base, buckets, il, deep, logits, cfg, lr_dense=5e-5, lr_sparse=5e-5,
                 dtype=torch.float32):
        self.dtype = dtype
        self.table = torch.as_tensor(table, dtype=dtype).clone()
        self.m_tab = torch.zeros_like(self.table)
        self.v_tab = torch.zeros_like(self.table)
        self.row_base = torch.as_tensor(row_base, dtype=torch.int64)
        self.buckets = torch.as_tensor(buckets, dtype=torch.int64)
        self.cfg = cfg
        self.params = {}
        for k, v in il.items():
            self.params["il_" + k] = torch.as_tensor(v, dtype=dtype).clone().requires_grad_(True)
        self.deep = [(torch.as_tensor(W, dtype=dtype).clone().requires_grad_(True),
                      torch.as_tensor(b, dtype=dtype).clone().requires_grad_(True)) for W, b in deep]
        self.logits = [(torch.as_tensor(W, dtype=dtype).clone().requires_grad_(True),
                        torch.as_tensor(b, dtype=dtype).clone().requires_grad_(True)) for W, b in logits]
        self.dense_list = list(self.params.values()) + [t for l in self.deep + self.logits for t in l]
        self.m = [torch.zeros_like(p) for p in self.dense_list]
        self.v = [torch.zeros_like(p) for p in self.dense_list]
        self.t = 0
        self.lr_dense, self.lr_sparse = lr_dense, lr_sparse

    def rows(self, ids):
        F = ids.shape[1]
        return self.row_base[None, :] + torch.remainder(ids, self.buckets[None, :])

    def step(self, ids, labels):
        B, F = ids.shape
        rows = self.rows(ids).reshape(-1)
        x0 = self.table.index_select(0, rows).reshape(B, F, -1).requires_grad_(True)
        il = {k[3:]: v for k, v in self.params.items()}
        _, p = autoint_forward(x0, il, self.deep, self.logits, self.cfg)
        loss = cross_entropy(labels.reshape(B, -1), p)
        grads = torch.autograd.grad(loss, [x0] + self.dense_list)
        gx, gd = grads[0], grads[1:]
        with torch.no_grad():
            self.t += 1
            b1, b2, eps = 0.9, 0.999, 1e-8
            lr_t = self.lr_dense * (1 - b2 ** self.t) ** 0.5 / (1 - b1 ** self.t)
            for p_, g, m, v in zip(self.dense_list, gd, self.m, self.v):
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                p_.sub_(lr_t * m / (v.sqrt() + eps))
            uniq, inv = torch.unique(rows, return_inverse=True)
            gsum = torch.zeros(uniq.numel(), self.table.shape[1], dtype=self.dtype)
            gsum.index_add_(0, inv, gx.reshape(B * F, -1))
            m = self.m_tab[uniq].mul_(b1).add_(gsum, alpha=1 - b1)
            v = self.v_tab[uniq].mul_(b2).addcmul_(gsum, gsum, value=1 - b2)
            self.m_tab[uniq] = m
            self.v_tab[uniq] = v
            self.table[uniq] -= self.lr_sparse * m / (eps + v.sqrt())
        return float(loss)


def din_pool(queries, keys, values, seq_length, W1, b1, W2, b2):
    """din.py:18-47 op for op (tile + concat + two relu Dense + where + matmul)."""
    T = keys.shape[1]
    q = queries[:, None, None, :].expand(-1, 1, T, -1)
    k = keys[:, None, :, :]
    deep = torch.cat([q, k, q * k], dim=-1)
    deep = dense(deep, W1, b1, "relu")
    deep = dense(deep, W2, b2, "relu").squeeze(-1)              # [B, 1, T]
    if seq_length is not None:
        m = (torch.arange(T)[None, :] < torch.as_tensor(seq_length)[:, None])[:, None, :]
        deep = torch.where(m, deep, torch.zeros_like(deep))
    return torch.matmul(deep, values).squeeze(1)


def din_softmax_pool(query, facts, mask, W1, b1, W2, b2):
    """staytime/layer.py:16-41 op for op."""
    B, T, H = facts.shape
    q = query[:, None, :].expand(-1, T, -1)
    din_all = torch.cat([q, facts, q - facts, q * facts], dim=-1)
    d2 = dense(dense(din_all, W1, b1, "sigmoid"), W2, b2, None)
    scores = d2.reshape(-1, 1, T)
    if mask is not None:
        km = torch.as_tensor(mask)[:, :T][:, None, :]
        scores = torch.where(km, scores, torch.full_like(scores, npo.DIN_PAD))
    return torch.matmul(torch.softmax(scores, dim=-1), facts).squeeze(1)


# ==========================================================================================
# H8 rough_rank layers (rough_rank/layer.py), H9 staytime towers (staytime/VideoDnn.py,
# staytime/layer.py), H5 multi_head gates (rank/multi_head/multidnn.py), H10 losses.
# Written op for op with torch CPU ops (float64 in the tests); weights are passed in.
# ==========================================================================================
def _act(x, activation):
    if activation in (None, "linear"):
        return x
    if activation == "relu":
        return torch.relu(x)
    if activation == "sigmoid":
        return torch.sigmoid(x)
    if activation == "softmax":
        return torch.softmax(x, dim=-1)
    raise ValueError(activation)


def dnn(x, kernels, biases, activation="relu", output_activation=None):
    """DNN.call (rough_rank/layer.py:99-107): tensordot + bias_add + Activation per layer; the
    last layer uses output_activation when given (:86-91).  No BN / dropout (the call sites use
    use_bn=False, dropout_rate=0)."""
    n = len(kernels)
    for i, (W, b) in enumerate(zip(kernels, biases)):
        x = torch.tensordot(x, W, dims=([x.dim() - 1], [0])) + b
        act = output_activation if (output_activation and i == n - 1) else activation
        x = _act(x, act)
    return x


def mmoe(x, experts, gates, expert_activation="relu"):
    """MMOE.call (rough_rank/layer.py:149-162): experts = [(kernels, biases)] DNNs, gates = DNNs
    with softmax output; task_out = sum_e gate_e * expert_e."""
    eo = torch.stack([dnn(x, k, b, expert_activation) for k, b in experts], dim=-2)   # :150-151
    outs = []
    for k, b in gates:
        g = dnn(x, k, b, "relu", "softmax").unsqueeze(-1)                          # :154-155
        outs.append(torch.sum(eo * g, dim=-2))                                       # :158
    return outs


def ple(x, shared, specific, gates, expert_activation="relu"):
    """PLE.call (rough_rank/layer.py:212-226)."""
    so = [dnn(x, k, b, expert_activation) for k, b in shared]                     # :213
    outs = []
    for t, (gk, gb) in enumerate(gates):
        sp = [dnn(x, k, b, expert_activation) for k, b in specific[t]]            # :216
        eo = torch.stack(so + sp, dim=-2)                                           # :217-218
        g = dnn(x, gk, gb, "relu", "softmax").unsqueeze(-1)                        # :219,222
        outs.append(torch.sum(eo * g, dim=-2))                                      # :223
    return outs


def crossnet(x, kernels, biases):
    """CrossNet.call (rough_rank/layer.py:252-260): kernels [D, 1], biases [D, 1]."""
    x0 = x.unsqueeze(2)
    xl = x0
    for W, b in zip(kernels, biases):
        xw = torch.tensordot(xl, W, dims=([1], [0]))     # [B, 1, 1]
        dot_ = torch.matmul(x0, xw)                      # [B, D, 1]
        xl = dot_ + b + xl
    return xl.squeeze(2)


def deep_cross_layer(x, Ws, bs):
    """DeepCrossLayer.call (staytime/layer.py:65-71): W_i [D, 1], b_i [D]."""
    cross = None
    for i, (W, b) in enumerate(zip(Ws, bs)):
        if i == 0:
            cross = x * torch.matmul(x, W) + b + x
        else:
            cross = x * torch.matmul(cross, W) + b + cross
    return cross


def kd_loss(student, teacher):
    """KDLoss (rough_rank/layer.py:272-279): MeanSquaredError(reduction=NONE)(teacher, student)
    = mean over the last axis of (teacher - student)^2."""
    return torch.mean(torch.square(teacher - student), dim=-1)


def similarity(u, i, use_sigmoid=False):
    """Similarity.call (rough_rank/layer.py:19-24)."""
    out = torch.sum(u * i, dim=-1, keepdim=True)
    return torch.sigmoid(out) if use_sigmoid else out


def fm_layer(x):
    """FMLayer.call (staytime/layer.py:99-112): x [B, F, E] -> [B, 1]."""
    square_of_sum = torch.square(torch.sum(x, dim=1, keepdim=True))
    sum_of_square = torch.sum(x * x, dim=1, keepdim=True)
    cross_term = square_of_sum - sum_of_square
    return 0.5 * torch.sum(cross_term, dim=-1)


def senet_fm(general, W1, b1, W2, b2):
    """staytime/VideoDnn.py:81-115: SENet on the stop-gradient concat of the general inputs
    (Dense(len/4 -> int, relu), 2 * Dense(len, sigmoid)), per-field reweight, then the FM cross
    term (vector) and fm_logit.  general: list of [B, E].  Returns (reweighted list, cross, fm)."""
    n = len(general)
    sq = torch.cat(general, dim=-1).detach()                                        # :84-86
    s1 = torch.relu(sq @ W1 + b1)                                                   # :87-88
    s2 = 2 * torch.sigmoid(s1 @ W2 + b2)                                            # :90-91
    splits = torch.split(s2, 1, dim=1)                                              # :93
    rew = [g * s for g, s in zip(general, splits)]                                  # :95-96
    sum_embs = torch.sum(torch.stack(rew), dim=0)                                   # :108
    cross = sum_embs * sum_embs - torch.sum(torch.stack([r * r for r in rew]), dim=0)  # :109-112
    fm = 0.5 * torch.sum(cross, dim=-1, keepdim=True)                               # :114
    assert n == len(rew)
    return rew, cross, fm


def ffm_block(user, item, Wx, bx, Wy, by):
    """ffm_block (staytime/VideoDnn.py:11-25) for one [x_list, y_list, dim] group: pair p =
    (i, j) over user x item fields, Dense(dim)(x_i) * Dense(dim)(y_j), concatenated in p order.
    Wx [P, E, dim], bx [P, dim] (same for y)."""
    out, p = [], 0
    for x in user:
        for y in item:
            out.append((x @ Wx[p] + bx[p]) * (y @ Wy[p] + by[p]))
            p += 1
    return torch.cat(out, dim=-1)


def multiply_relu(user, item):
    """staytime/VideoDnn.py:99-105: ReLU(concat(user) * concat(item))."""
    return torch.relu(torch.cat(user, dim=-1) * torch.cat(item, dim=-1))


def staytime_head(x, W, b, bins):
    """staytime/VideoDnn.py:168-179: softmax(Dense(400)(x)), expected bins clamped at 0,
    concatenated -> [B, 401]."""
    p = torch.softmax(x @ W + b, dim=-1)
    pred = p @ torch.as_tensor(bins, dtype=p.dtype).reshape(-1, 1)
    pred = torch.where(pred < 0.0, torch.zeros_like(pred), pred)
    return torch.cat([p, pred], dim=-1)


def custom_kl_loss(y_true, y_pred, C=400, eps=1e-7):
    """staytime/model.py:20-30 (K.epsilon() = 1e-7): per-sample KL over the first C columns."""
    yt = torch.clamp(y_true[:, :C].to(y_pred.dtype), eps, 1.0)
    yp = torch.clamp(y_pred[:, :C], eps, 1.0)
    return torch.sum(yt * torch.log(yt / yp), dim=-1)


def keras_bce(y_true, y_pred, eps=1e-7):
    """tf.keras.losses.BinaryCrossentropy() (rough_rank/model.py:211-212): clip to
    [eps, 1-eps], -(y log(p+eps) + (1-y) log(1-p+eps)), mean over the last axis, then over the
    batch."""
    p = torch.clamp(y_pred, eps, 1.0 - eps)
    bce = y_true * torch.log(p + eps) + (1 - y_true) * torch.log(1 - p + eps)
    return torch.mean(torch.mean(-bce, dim=-1))


def multi_head_gates(result, We, be, Wg, bg, n_used=7):
    """rank/multi_head/multidnn.py:77-120: 8 experts Dense(32, relu), only the first n_used
    stacked; n_tasks gates Dense(n_used, softmax); task t = sum_e gate_te * expert_e.
    We [8][K, 32], Wg [T][K, n_used]."""
    eo = torch.stack([torch.relu(result @ W + b) for W, b in zip(We, be)][:n_used], dim=1)  # :82-92
    outs = []
    for W, b in zip(Wg, bg):
        g = torch.softmax(result @ W + b, dim=-1).unsqueeze(-1)                     # :100-107
        outs.append(torch.sum(eo * g, dim=1))                                        # :109-112
    return outs


# ==========================================================================================
# H12 rank/ctr Model.model_layer and H13 rank/finish DeepFM (op for op; weights passed in as
# {keras layer name: (kernel, bias)}; test infrastructure only).
# ==========================================================================================
def rank_ctr_model_layer(structure, gate_inputs, bias, P, il, il_seed, drop_rate=0.2, eps=1e-14,
                         ppnet_units=(256, 64, 8, 256, 64, 8, 32, 16), num_experts=3,
                         expert_units=(512, 256), gate_units=(256, 32), tower_units=(64, 8)):
    """rank/ctr/model_init.py:19-162.  structure = emb_structure_input (list of [B, w_i]),
    gate_inputs = emb_gate_input, bias = emb_bias_input {type: [tensors]}, il = (W, bias, gamma,
    beta) of the InteractingLayer.  Returns the two sigmoid outputs BEFORE the clip."""
    sq = torch.cat([s.mean(dim=1, keepdim=True) for s in structure], dim=1)        # :21-26
    sq = sq.detach()                                                                 # :28
    s1 = dense(sq, *P["senet_squeeze_layer"], "relu")                               # :29
    s2 = 2 * dense(s1, *P["senet_extract_layer"], "sigmoid")                        # :32
    splits = torch.split(s2, 1, dim=1)                                               # :34
    rew = [e * sp for e, sp in zip(structure, splits)]                               # :36-40
    emb3d = [dense(r, *P[f"emb_linear_map_{i}"])[:, None, :] for i, r in enumerate(rew)]  # :43-46
    auto_in = torch.cat(emb3d, dim=1)                                                # :48
    B = auto_in.shape[0]
    auto = interacting_layer(auto_in, *il, layer_num=1, head_num=2, use_res=True, eps=eps,
                             drop_rate=drop_rate, seed=il_seed).reshape(B, -1)      # :53-59
    pp = 2 * dense(torch.cat(bias["ppnet"], dim=1), *P["dnn_ppnet_gate"], "sigmoid")  # :64-66
    gl = torch.split(pp, list(ppnet_units), dim=1)                                   # :68
    deep = torch.cat(rew, dim=1)                                                     # :72
    for i in range(2):                                                               # :74-78
        deep = torch.relu(dense(deep, *P[f"dnn_{i}"]) * gl[i + 6])
    mult = torch.relu(torch.cat(bias["multiply_user"], 1) * torch.cat(bias["multiply_item"], 1))
    result = torch.cat([deep, auto, mult], dim=1)                                    # :87
    can = dense(torch.cat(bias["can"], dim=1), *P["dnn_can"])                         # :90-91
    c = torch.split(can, [48, 6, 24, 4], dim=1)                                      # :92
    w1, b1 = c[0].reshape(-1, 8, 6), c[1].reshape(-1, 1, 6)
    w2, b2 = c[2].reshape(-1, 6, 4), c[3].reshape(-1, 1, 4)
    gate_in = torch.cat(gate_inputs, dim=1)                                          # :104
    experts = []
    for i in range(num_experts):                                                     # :105-114
        er = result
        for j, _ in enumerate(expert_units):
            g = dense(gate_in, *P[f"gate_{i}_{j}_1"], "relu")
            g = 2 * dense(g, *P[f"gate_{i}_{j}_2"], "sigmoid")
            er = dense(er, *P[f"expert_output_{i}_{j}"], "relu")
            er = g * er
        experts.append(er)
    ec = torch.stack(experts, dim=1)                                                 # :115
    outs = []
    for t in range(2):                                                               # :121-132
        go = result
        for j, _ in enumerate(gate_units):
            go = dense(go, *P[f"gate_{t}_{j}"], "relu")
        go = torch.softmax(dense(go, *P[f"gate_output_{t}"]), dim=-1)[..., None]
        r = torch.sum(ec * go, dim=1)
        for j, _ in enumerate(tower_units):                                          # :139-155
            if j == 0:
                r = torch.relu(r * gl[t * 3])
            r = dense(r, *P[f"task{t}_dnn2_{j}"])
            r = torch.relu(r * gl[t * 3 + j + 1])
            if j == len(tower_units) - 1:
                cr = torch.relu(torch.matmul(r[:, None, :], w1) + b1)
                cr = torch.relu(torch.matmul(cr, w2) + b2).squeeze(1)
                r = torch.cat([r, cr], dim=1)
        outs.append(dense(r, *P[f"output_{t}"], "sigmoid"))                          # :156
    return outs


def fm_layer_finish(x, V, w, b):
    """rank/finish FMLayer.call (videodnn.py:41-52)."""
    sum_square = torch.square(x @ V)
    square_sum = torch.square(x) @ torch.square(V)
    high = 0.5 * torch.sum(sum_square - square_sum, dim=1, keepdim=True)
    return high + dense(x, w, b)


def deepfm_sub_model(general_list, bias_list, P, hidden=(64, 32)):
    """rank/finish create_deepFM_sub_model (videodnn.py:69-137) from the per-slot inputs
    (general_list = gerneral_inputs incl. emb_1568[:, 16:], bias_list = bais_inputs)."""
    general = torch.cat(general_list, dim=1)
    fm = fm_layer_finish(general, *P["fm"])
    bias = torch.cat(bias_list, dim=1)
    x = general
    for i, unit in enumerate(hidden):
        if i == 0:
            x = dense(x, *P[f"dnn_{i}"], "relu")
        else:
            one = dense(bias, *P[f"bais_dnn_one_{i}"], "relu")
            two = dense(one, *P[f"bais_dnn_two_{i}"], "sigmoid") * 2
            x = dense(x * two, *P[f"dnn_{i}"], "relu")
    one = dense(bias, *P["bais_dnn_one_3"], "relu")
    two = dense(one, *P["bais_dnn_two_3"], "sigmoid") * 2
    x = x * two
    return dense(torch.cat([x, fm], dim=1), *P["pred"], "sigmoid")


# ==========================================================================================
# CPU train steps of configs 3 and 4 (the bench's cpu_baseline legs; kind "port"): the same
# unfused TF-semantics op sequences as above in fp32 on the host, dense Adam (tf.keras form) and
# sparse Adam on the touched rows (tensornet form), from copies of a device model's weights.
# ==========================================================================================
class _CPUTrainBase:
    def _init_opt(self, lr_dense, lr_sparse):
        self.m = [torch.zeros_like(p) for p in self.dense_list]
        self.v = [torch.zeros_like(p) for p in self.dense_list]
        self.m_tab = torch.zeros_like(self.table)
        self.v_tab = torch.zeros_like(self.table)
        self.t = 0
        self.lr_dense, self.lr_sparse = lr_dense, lr_sparse

    def _update(self, loss, leaves, rows):
        grads = torch.autograd.grad(loss, leaves + self.dense_list)
        gl, gd = grads[:len(leaves)], grads[len(leaves):]
        with torch.no_grad():
            self.t += 1
            b1, b2, eps = 0.9, 0.999, 1e-8
            lr_t = self.lr_dense * (1 - b2 ** self.t) ** 0.5 / (1 - b1 ** self.t)
            for p_, g, m, v in zip(self.dense_list, gd, self.m, self.v):
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                p_.sub_(lr_t * m / (v.sqrt() + eps))
            r = torch.cat([x.reshape(-1) for x in rows])
            g = torch.cat([x.reshape(rr.numel(), -1) for x, rr in zip(gl, rows)])
            keep = r >= 0
            r, g = r[keep], g[keep]
            uniq, inv = torch.unique(r, return_inverse=True)
            gsum = torch.zeros(uniq.numel(), self.table.shape[1]).index_add_(0, inv, g)
            m = self.m_tab[uniq].mul_(b1).add_(gsum, alpha=1 - b1)
            v = self.v_tab[uniq].mul_(b2).addcmul_(gsum, gsum, value=1 - b2)
            self.m_tab[uniq] = m
            self.v_tab[uniq] = v
            self.table[uniq] -= self.lr_sparse * m / (eps + v.sqrt())
        return float(loss.detach())


def _cpu(t):
    return t.detach().float().cpu().clone().requires_grad_(True)


class DINPoolCPU(_CPUTrainBase):
    """Config 4 (workloads.DINPool): query lookup, history lookup, din.py DIN pool, Dense(1,
    sigmoid) on [pooled, q], cross_entropy (rank/multi_head/model.py:18-22), backward, Adam."""

    def __init__(self, model, lr_dense=5e-5, lr_sparse=5e-5):
        self.table = model.table.weight.detach().float().cpu().clone()
        self.vocab, self.T = model.table.rows, model.T
        d = model.din
        self.W1, self.b1, self.W2, self.b2 = (_cpu(p) for p in (d.W1, d.b1, d.W2, d.b2))
        self.Wo, self.bo = _cpu(model.out.kernel), _cpu(model.out.bias)
        self.dense_list = [self.W1, self.b1, self.W2, self.b2, self.Wo, self.bo]
        self._init_opt(lr_dense, lr_sparse)

    def prepare(self, qids, hids, hoffs, labels):
        """Host-side batch (the pre-generated input): query rows [B], padded history rows [B, T]
        (-1 past the length), lengths [B], labels."""
        q = torch.as_tensor(qids).long() % self.vocab
        h, o = torch.as_tensor(hids).long() % self.vocab, torch.as_tensor(hoffs).long()
        B = q.numel()
        lens = torch.clamp(o[1:] - o[:-1], max=self.T)
        pos = torch.arange(self.T)[None, :]
        idx = torch.clamp(o[:-1, None] + pos, max=max(h.numel() - 1, 0))
        rows = torch.where(pos < lens[:, None], h[idx], torch.full_like(idx, -1))
        return q, rows, lens, torch.as_tensor(labels).float().reshape(B, -1)

    def step(self, q, rows, lens, y):
        qe = self.table.index_select(0, q).requires_grad_(True)
        he = self.table.index_select(0, rows.clamp(min=0).reshape(-1)).reshape(*rows.shape, -1)
        he = torch.where((rows >= 0)[..., None], he, torch.zeros_like(he)).requires_grad_(True)
        pooled = din_pool(qe, he, he, lens, self.W1, self.b1, self.W2, self.b2)
        p = dense(torch.cat([pooled, qe], 1), self.Wo, self.bo, "sigmoid")
        loss = torch.mean(torch.sum(-y * torch.log(p + 1e-6) - (1 - y) * torch.log(1 - p + 1e-6), 1))
        return self._update(loss, [qe, he], [q, rows])


class MultiHeadCPU(_CPUTrainBase):
    """Config 3 (models.MultiHeadRanker, rank/multi_head/multidnn.py:14-259): multi-hot mean
    lookup, IL(1, 8, 2, dropout .2, res), deep Dense(32, 16), 7 experts / 7 softmax gates, 7
    sigmoid towers, cross_entropy, backward, Adam (L1L2 / L2 regularisers omitted: <1 % of the
    work)."""

    def __init__(self, model, lr_dense=1e-5, lr_sparse=5e-5):
        self.table = model.table.weight.detach().float().cpu().clone()
        self.cfg = cfg = model.cfg
        il = model.interact
        self.il = [_cpu(p) for p in (il.kernel, il.bias, il.gamma, il.beta)]
        self.eps = il.epsilon
        self.deep = [(_cpu(l.kernel), _cpu(l.bias)) for l in model.deep]
        self.Wc, self.bc = _cpu(model.mix.kernel), _cpu(model.mix.bias)
        self.TW, self.Tb = _cpu(model.towers.W), _cpu(model.towers.b)
        self.row_base = model.embedding.row_base.cpu().long()
        self.bucket = model.embedding.bucket.cpu().long()
        self.dense_list = self.il + [t for l in self.deep for t in l] + [self.Wc, self.bc, self.TW, self.Tb]
        self._init_opt(lr_dense, lr_sparse)

    def prepare(self, ids, offsets, labels):
        ids, offs = torch.as_tensor(ids).long(), torch.as_tensor(offsets).long()
        F = self.cfg.num_fields
        nseg = offs.numel() - 1
        cnt = offs[1:] - offs[:-1]
        seg = torch.repeat_interleave(torch.arange(nseg), cnt)
        f = seg % F
        rows = self.row_base[f] + torch.remainder(ids, self.bucket[f])
        return rows, seg, cnt.clamp(min=1).float(), torch.as_tensor(labels).float()

    def step(self, rows, seg, cnt, y):
        cfg = self.cfg
        B, F, E = y.shape[0], cfg.num_fields, cfg.embed_dim
        e = self.table.index_select(0, rows).requires_grad_(True)
        x0 = (torch.zeros(B * F, E).index_add(0, seg, e) / cnt[:, None]).reshape(B, F, E)
        auto = interacting_layer(x0, *self.il, 1, 2, True, self.eps, drop_rate=cfg.dropout_rate,
                                 torch_mask=True).reshape(B, -1)
        deep = mlp(x0.reshape(B, -1), self.deep, "relu")
        result = torch.cat([deep, auto], 1)
        D, NE, ns = 32, 7, 7
        We = [self.Wc[:, k * D:(k + 1) * D] for k in range(NE)]
        be = [self.bc[k * D:(k + 1) * D] for k in range(NE)]
        Wg = [self.Wc[:, NE * D + t * ns:NE * D + (t + 1) * ns] for t in range(7)]
        bg = [self.bc[NE * D + t * ns:NE * D + (t + 1) * ns] for t in range(7)]
        outs = multi_head_gates(result, We, be, Wg, bg, 7)
        preds = torch.cat([torch.sigmoid(o @ self.TW[t] + self.Tb[t]).reshape(B, 1)
                           for t, o in enumerate(outs)], 1)
        loss = cross_entropy(y, preds)
        return self._update(loss, [e], [rows])
