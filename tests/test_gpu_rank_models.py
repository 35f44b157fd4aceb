"""GPU parity of the rank/ctr production model (H12, with the H2 device front end) and rank/finish
DeepFM + FMLayer(Dense) (H13) against op-for-op float64 restatements (oracle/torch_ref.py
rank_ctr_model_layer / deepfm_sub_model) built from the same weights.  The rank/ctr layout is
the shipped rank/ctr/model_parameter.json (tests/golden/rank_ctr_feature_slot.json, made by
tests/golden/make_rank_ctr_fixture.py): 176 slots of width 96, 175 structure fields (2500
columns), 14 gate fields, bias groups ppnet 272 / can 176 / multiply_user 48 / multiply_item 48.
Tolerances: outputs 2e-5, losses 1e-5 relative, gradients tests/_tol.py.  Parity unpinned
against TF itself (oracle/ctr_oracle.py header)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo
from oracle import torch_ref as tr
from _tol import assert_close, assert_grad_close, to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def c64(t, grad=True):
    return torch.tensor(to_np(t), dtype=torch.float64, requires_grad=grad)


def _randomise_biases(model, rng, scale=0.05):
    with torch.no_grad():
        for name, p in model.named_parameters():
            if p.dim() == 1 or "bias" in name:
                p.copy_(torch.from_numpy(rng.uniform(-scale, scale, size=tuple(p.shape)).astype(np.float32)))


# ------------------------------------------------------------------------------------------
# front-end kernels against torch fp64
# ------------------------------------------------------------------------------------------
def test_front_end_kernels():
    from recommendsystem_amd._lib import call, ptr, stream_handle
    rng = np.random.default_rng(7)
    B, S = 37, 50
    src = torch.from_numpy(rng.normal(size=(B, S)).astype(np.float32)).to(DEV)
    cols = torch.tensor([5, 0, 49, 7, 8, 9, 30], dtype=torch.int32, device=DEV)
    out = torch.empty(B, 7, device=DEV)
    call("rs_gather_columns", stream_handle(), ptr(src), S, B, ptr(cols), 7, ptr(out), 7)
    assert torch.equal(out, src[:, cols.long()])
    dsrc = torch.ones(B, S, device=DEV)
    call("rs_scatter_add_columns", stream_handle(), ptr(out), 7, B, ptr(cols), 7, ptr(dsrc), S)
    want = torch.ones(B, S, device=DEV)
    want[:, cols.long()] += src[:, cols.long()]
    assert torch.equal(dsrc, want)
    # a plan naming columns twice: both gradients arrive
    dup = torch.tensor([3, 3, 11, 3, 11], dtype=torch.int32, device=DEV)
    g = torch.from_numpy(rng.normal(size=(B, 5)).astype(np.float32)).to(DEV)
    dsrc = torch.zeros(B, S, device=DEV)
    call("rs_scatter_add_columns", stream_handle(), ptr(g), 5, B, ptr(dup), 5, ptr(dsrc), S)
    g64 = g.double()
    torch.testing.assert_close(dsrc[:, 3].double(), g64[:, 0] + g64[:, 1] + g64[:, 3], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(dsrc[:, 11].double(), g64[:, 2] + g64[:, 4], rtol=1e-6, atol=1e-6)
    assert int((dsrc != 0).sum()) == 2 * B
    # segments incl. an empty one
    seg = torch.tensor([0, 3, 3, 10, 50], dtype=torch.int32, device=DEV)
    m = torch.empty(B, 4, device=DEV)
    call("rs_segment_mean", stream_handle(), ptr(src), S, B, ptr(seg), 4, ptr(m), 4)
    s64 = src.double().cpu()
    ref = torch.stack([s64[:, 0:3].mean(1), torch.zeros(B, dtype=torch.float64), s64[:, 3:10].mean(1),
                       s64[:, 10:50].mean(1)], 1)
    assert_close(to_np(m), ref.numpy(), 1e-6, what="segment mean")
    # CAN per-sample matmuls: forward and gradients vs torch autograd
    r = torch.from_numpy(rng.normal(size=(B, 8)).astype(np.float32)).to(DEV).requires_grad_(True)
    p = torch.from_numpy(rng.normal(size=(B, 82)).astype(np.float32) * 0.5).to(DEV).requires_grad_(True)
    from recommendsystem_amd.rank_models import can_block
    y = can_block(r, p)
    g = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(DEV)
    y.backward(g)
    r64, p64 = c64(r), c64(p)
    c = torch.split(p64, [48, 6, 24, 4], dim=1)
    h = torch.relu(torch.matmul(r64[:, None, :], c[0].reshape(-1, 8, 6)) + c[1].reshape(-1, 1, 6))
    y64 = torch.relu(torch.matmul(h, c[2].reshape(-1, 6, 4)) + c[3].reshape(-1, 1, 4)).squeeze(1)
    y64.backward(g.double().cpu())
    assert_close(to_np(y), to_np(y64), 1e-5, what="can")
    assert_grad_close(to_np(r.grad), r64.grad.numpy(), "can dr")
    assert_grad_close(to_np(p.grad), p64.grad.numpy(), "can dp")


# ------------------------------------------------------------------------------------------
# H12 rank/ctr Model
# ------------------------------------------------------------------------------------------
def _rank_ctr_P(m):
    """Keras layer name -> (kernel, bias) fp64 leaves (views of the fused blocks' leaves), plus the
    (parameter, leaf) pairs whose gradients are checked."""
    cfg = m.cfg
    L = {}
    pairs = []

    def leaf(p):
        t = c64(p)
        pairs.append((p, t))
        return t

    def dense(layer):
        return leaf(layer.kernel), leaf(layer.bias)

    P = {"senet_squeeze_layer": dense(m.senet_sq), "senet_extract_layer": dense(m.senet_ex),
         "dnn_ppnet_gate": dense(m.ppnet), "dnn_can": dense(m.can)}
    for i, l in enumerate(m.deep):
        P[f"dnn_{i}"] = dense(l)
    Kf, Bf = leaf(m.field_map.kernel), leaf(m.field_map.bias)
    seg = m.field_map.seg.cpu().numpy()
    for f in range(m.field_map.F):
        P[f"emb_linear_map_{f}"] = (Kf[seg[f]:seg[f + 1]], Bf[f])
    NE, EU, GU = cfg.num_experts, list(cfg.expert_units), list(cfg.gate_units)
    K1, B1 = leaf(m.first.kernel), leaf(m.first.bias)
    offs = np.cumsum([0] + m.first.units)
    for i in range(NE):
        P[f"expert_output_{i}_0"] = (K1[:, offs[i]:offs[i + 1]], B1[offs[i]:offs[i + 1]])
    for t in range(2):
        q = NE + t
        P[f"gate_{t}_0"] = (K1[:, offs[q]:offs[q + 1]], B1[offs[q]:offs[q + 1]])
    Kp, Bp = leaf(m.pp1.kernel), leaf(m.pp1.bias)
    offs = np.cumsum([0] + m.pp1.units)
    k = 0
    for i in range(NE):
        for j in range(len(EU)):
            q = i * len(EU) + j
            P[f"gate_{i}_{j}_1"] = (Kp[:, offs[q]:offs[q + 1]], Bp[offs[q]:offs[q + 1]])
            P[f"gate_{i}_{j}_2"] = dense(m.pp2[q])
            if j > 0:
                P[f"expert_output_{i}_{j}"] = dense(m.exp_rest[k])
                k += 1
    for t in range(2):
        P[f"gate_{t}_1"] = dense(m.gate_l2[t])
        P[f"gate_output_{t}"] = dense(m.gate_out[t])
        for j, l in enumerate(m.towers[t]):
            P[f"task{t}_dnn2_{j}"] = dense(l)
        P[f"output_{t}"] = dense(m.outputs[t])
    il = m.interact
    ilw = tuple(leaf(p) for p in (il.kernel, il.bias, il.gamma, il.beta))
    return P, ilw, pairs


@pytest.mark.parametrize("B", [5, 96])
def test_rank_ctr_model_matches_oracle(B):
    from recommendsystem_amd.feature_config import GATE_FEATURE_LIST
    from recommendsystem_amd.rank_models import RankCtrConfig, RankCtrModel
    rng = np.random.default_rng(71)
    mc = json.load(open(os.path.join(GOLDEN, "rank_ctr_feature_slot.json")))
    bucket = 500
    m = RankCtrModel(mc, RankCtrConfig(bucket_size=bucket), device=DEV, seed=5)
    _randomise_biases(m, rng)
    fe, L = m.front, m.layout
    F = len(fe.features)
    assert F == 176 and L.max_embed_size == 96 and m.struct_dim == 2500 and m.n_struct == 175
    lens = rng.integers(1, 4, size=B * F)
    lens[:F] = 1
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ids = rng.integers(0, 5 * bucket, size=int(offs[-1])).astype(np.int64)
    labels = (rng.uniform(size=(B, 2)) < 0.3).astype(np.float32)
    idt, offt, lbt = (torch.from_numpy(a).to(DEV) for a in (ids, offs, labels))
    il = m.interact
    seed = (il.seed * 1000003 + il._calls) & 0xFFFFFFFFFFFFFFFF   # the forward's dropout seed
    loss = m.loss(idt, offt, lbt)
    loss.backward()
    torch.cuda.synchronize()
    # ---- oracle ----
    W = fe.table.weight.detach().cpu().numpy().astype(np.float64)
    x0n, rows = npo.embedding_lookup(ids, offs, B, F, fe.embedding.row_base.cpu().numpy(),
                                     fe.embedding.bucket.cpu().numpy(), W, "mod", "mean")
    e64 = torch.tensor(x0n, requires_grad=True)
    emb = {s: e64[:, i] for i, s in enumerate(fe.features)}
    structure = [emb[s][:, a:b] for s, a, b in L.structure_intervals()]
    gate = [emb[s][:, a:b] for s, a, b in L.gate_intervals(GATE_FEATURE_LIST)]
    bias = {k: [emb[s][:, a:b] for s, a, b in v] for k, v in L.bias_intervals().items()}
    P, ilw, pairs = _rank_ctr_P(m)
    outs = tr.rank_ctr_model_layer(structure, gate, bias, P, ilw, seed, il.dropout_rate, il.epsilon)
    y = torch.from_numpy(labels).double()
    ref_loss = sum(tr.cross_entropy(y[:, t:t + 1], torch.clamp(outs[t], 1e-6, 1.0)) for t in range(2))
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss))), \
        (float(loss), float(ref_loss))
    for t in range(2):
        assert_close(to_np(m.last_outputs[t]), to_np(outs[t]), 2e-5, what=f"rank/ctr output {t}")
    ref_loss.backward()
    for p, r in pairs:
        assert_grad_close(to_np(p.grad), r.grad.numpy(), f"rank/ctr param {tuple(p.shape)}")
    g = npo.sparse_grad_sum(rows, offs, B, F, e64.grad.numpy().reshape(B * F, -1), "mean")
    keys = np.array(sorted(g))
    assert_grad_close(fe.table.grad.cpu().numpy()[keys], np.stack([g[k] for k in keys]), "rank/ctr push")


def test_rank_ctr_predict_and_outputs():
    """The clipped named outputs (model_init.py:157-161) equal the oracle's at use_dropout
    inference settings: forward with the IL in eval (dropout off)."""
    from recommendsystem_amd.feature_config import GATE_FEATURE_LIST
    from recommendsystem_amd.rank_models import RankCtrConfig, RankCtrModel
    rng = np.random.default_rng(72)
    mc = json.load(open(os.path.join(GOLDEN, "rank_ctr_feature_slot.json")))
    m = RankCtrModel(mc, RankCtrConfig(bucket_size=300), device=DEV, seed=6)
    _randomise_biases(m, rng)
    m.interact.train(False)  # Keras inference: no dropout
    fe, L = m.front, m.layout
    B, F = 16, len(fe.features)
    offs = np.arange(B * F + 1, dtype=np.int32)
    ids = rng.integers(0, 3000, size=B * F).astype(np.int64)
    pred = m.predict(torch.from_numpy(ids).to(DEV), torch.from_numpy(offs).to(DEV))
    assert list(pred) == list(m.cfg.task_names)
    W = fe.table.weight.detach().cpu().numpy().astype(np.float64)
    x0n, _ = npo.embedding_lookup(ids, offs, B, F, fe.embedding.row_base.cpu().numpy(),
                                  fe.embedding.bucket.cpu().numpy(), W, "mod", "mean")
    e64 = torch.tensor(x0n)
    emb = {s: e64[:, i] for i, s in enumerate(fe.features)}
    P, ilw, _ = _rank_ctr_P(m)
    outs = tr.rank_ctr_model_layer([emb[s][:, a:b] for s, a, b in L.structure_intervals()],
                                   [emb[s][:, a:b] for s, a, b in L.gate_intervals(GATE_FEATURE_LIST)],
                                   {k: [emb[s][:, a:b] for s, a, b in v] for k, v in L.bias_intervals().items()},
                                   P, ilw, 0, 0.0, m.interact.epsilon)
    for name, o in zip(m.cfg.task_names, outs):
        assert_close(to_np(pred[name]), torch.clamp(o, 1e-6, 1.0).detach().numpy(), 2e-5, what=name)


# ------------------------------------------------------------------------------------------
# H13 rank/finish FMLayer(Dense) + DeepFM
# ------------------------------------------------------------------------------------------
def test_fm_layer_dense_matches_oracle():
    from recommendsystem_amd.rank_models import FMLayer
    rng = np.random.default_rng(73)
    B, D = 300, 912
    x = torch.from_numpy(rng.normal(size=(B, D)).astype(np.float32) * 0.2).to(DEV).requires_grad_(True)
    fm = FMLayer(seed=3, device=DEV)
    y = fm(x)
    g = torch.from_numpy(rng.normal(size=(B, 1)).astype(np.float32)).to(DEV)
    y.backward(g)
    x64, V64 = c64(x), c64(fm.fm_matrix)
    w64, b64 = c64(fm.linear.kernel), c64(fm.linear.bias)
    y64 = tr.fm_layer_finish(x64, V64, w64, b64)
    y64.backward(g.double().cpu())
    assert_close(to_np(y), to_np(y64), 2e-5, 1e-5, what="FMLayer")
    assert_grad_close(to_np(x.grad), x64.grad.numpy(), "FMLayer dx")
    assert_grad_close(to_np(fm.fm_matrix.grad), V64.grad.numpy(), "FMLayer dV")
    assert_grad_close(to_np(fm.linear.kernel.grad), w64.grad.numpy(), "FMLayer dW linear")


def test_deepfm_matches_oracle():
    from recommendsystem_amd.rank_models import DeepFM, DeepFMConfig
    rng = np.random.default_rng(74)
    cfg = DeepFMConfig(bucket_size=1000)
    m = DeepFM(cfg, device=DEV, seed=9)
    _randomise_biases(m, rng)
    S = len(m.slots)
    assert S == 64 and m.gen_cols.numel() == 56 * 16 and m.bias_cols.numel() == 9 * 16
    B = 128
    ids = rng.integers(0, 20000, size=(B, S)).astype(np.int64)
    labels = (rng.uniform(size=(B, 1)) < 0.3).astype(np.float32)
    idt, lbt = torch.from_numpy(ids).to(DEV), torch.from_numpy(labels).to(DEV)
    loss = m.loss(idt, None, lbt)
    loss.backward()
    out = m(idt)
    W = m.table.weight.detach().cpu().numpy().astype(np.float64)
    x0n, rows = npo.embedding_lookup(ids, None, B, S, m.embedding.row_base.cpu().numpy(),
                                     m.embedding.bucket.cpu().numpy(), W, "mod", "mean")
    e64 = torch.tensor(x0n, requires_grad=True)
    emb = {s: e64[:, i] for i, s in enumerate(m.slots)}
    general = [emb[s][:, 0:16] for s in m.slots if s in set(cfg.general_slots)] + [emb["1568"][:, 16:]]
    bias = [emb[s][:, 0:16] for s in m.slots if s in set(cfg.bias_slots)]
    pairs = []

    def leaf(p):
        t = c64(p)
        pairs.append((p, t))
        return t

    P = {"fm": (leaf(m.fm.fm_matrix), leaf(m.fm.linear.kernel), leaf(m.fm.linear.bias)),
         "pred": (leaf(m.pred.kernel), leaf(m.pred.bias))}
    for i, l in enumerate(m.dnn):
        P[f"dnn_{i}"] = (leaf(l.kernel), leaf(l.bias))
    H = list(cfg.dnn_hidden_units)
    for q, (one, two) in enumerate(zip(m.b_one, m.b_two)):
        suffix = str(q + 1) if q < len(H) - 1 else "3"
        P[f"bais_dnn_one_{suffix}"] = (leaf(one.kernel), leaf(one.bias))
        P[f"bais_dnn_two_{suffix}"] = (leaf(two.kernel), leaf(two.bias))
    ref = tr.deepfm_sub_model(general, bias, P, tuple(H))
    ref_loss = tr.cross_entropy(torch.from_numpy(labels).double(), ref)
    assert_close(to_np(out), to_np(ref), 2e-5, what="DeepFM output")
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    ref_loss.backward()
    for p, r in pairs:
        assert_grad_close(to_np(p.grad), r.grad.numpy(), f"DeepFM param {tuple(p.shape)}")
    g = npo.sparse_grad_sum(rows, None, B, S, e64.grad.numpy().reshape(B * S, -1), "mean")
    keys = np.array(sorted(g))
    assert_grad_close(m.table.grad.cpu().numpy()[keys], np.stack([g[k] for k in keys]), "DeepFM push")
