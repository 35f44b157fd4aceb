"""CPU: the oracle itself — known answers, self-consistency (numpy vs torch autograd twin),
finite-difference gradients, and the committed golden fixtures (regression pins)."""
import os

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo
from oracle import torch_ref as tr

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def test_fmix32_known_answers():
    """murmur3 fmix32 (the dropout-mask finaliser): published values fmix32(0) = 0,
    fmix32(1) = 0x514E28B7."""
    out = npo.fmix32(np.array([0, 1], dtype=np.uint32))
    assert out.tolist() == [0, 0x514E28B7]


def test_dropout_mask_rate():
    keep = npo.dropout_keep(npo.layer_seed(7, 0), np.arange(64)[:, None, None, None], 1,
                            np.arange(40)[None, :, None, None], np.arange(40)[None, None, :, None], 0.2)
    assert abs(1.0 - keep.mean() - 0.2) < 0.01


def test_dropout_integer_threshold_is_exact():
    """csrc/common.hpp::dropout_thr16: the many-field forward compares the 16-bit half draw
    against ceil(rate * 2^16) (float32 arithmetic, as the device computes it) instead of
    half * 2^-16 >= rate: the two decisions agree for every draw, including the draws at and next
    to each threshold."""
    for rate in (0.1, 0.2, 0.25, 1.0 / 3.0, 0.5, 0.7, 0.999, 1e-7, 0.0):
        r32 = np.float32(rate)
        thr = np.uint32(np.ceil(np.float32(r32 * np.float32(65536.0))))
        draws = np.arange(0, 1 << 16, dtype=np.uint32)  # every half-draw value
        ref = draws.astype(np.float32) * np.float32(1.0 / 65536.0) >= r32
        assert np.array_equal(draws >= thr, ref), rate


def test_splitmix64_known_answers():
    d = gold("splitmix64_kat.npz")
    assert np.array_equal(npo.splitmix64(d["seeds"]), d["expect"])


def test_hash_rows_mod_and_negative_ids():
    ids = np.array([0, 5, 100001, -1, (1 << 63) - 1], dtype=np.int64)
    f = np.zeros(5, dtype=np.int64)
    rows = npo.hash_rows(ids, f, [7], [100000], "mod")
    u = ids.view(np.uint64)
    assert rows.tolist() == [7 + int(v % 100000) for v in u]


@pytest.mark.parametrize("combiner", ["mean", "sum", "sqrtn"])
def test_embedding_lookup_bruteforce(combiner):
    rng = np.random.default_rng(0)
    B, F, dim, vocab = 5, 3, 4, 11
    table = rng.normal(size=(F * vocab, dim))
    lens = rng.integers(0, 4, size=B * F)
    offs = np.concatenate([[0], np.cumsum(lens)])
    ids = rng.integers(0, 1000, size=offs[-1])
    out, rows = npo.embedding_lookup(ids, offs, B, F, np.arange(F) * vocab, [vocab] * F, table,
                                     "mod", combiner)
    for s in range(B * F):
        f = s % F
        seg = ids[offs[s]:offs[s + 1]]
        if len(seg) == 0:
            assert np.all(out.reshape(B * F, dim)[s] == 0)
            continue
        acc = sum(table[f * vocab + (i % vocab)] for i in seg)
        sc = {"mean": 1 / len(seg), "sum": 1.0, "sqrtn": 1 / np.sqrt(len(seg))}[combiner]
        assert np.allclose(out.reshape(B * F, dim)[s], acc * sc, atol=1e-12)


def test_golden_lookup_and_sparse_push():
    d = gold("lookup_ragged.npz")
    B, F = 9, 4
    for mode in ("mod", "splitmix"):
        for comb in ("mean", "sum", "sqrtn"):
            o, rows = npo.embedding_lookup(d["ids"], d["offsets"], B, F, d["row_base"], d["bucket"],
                                           d["table"].astype(np.float64), mode, comb)
            assert np.array_equal(rows, d[f"rows_{mode}"])  # index work: bit-exact
            assert np.array_equal(o, d[f"out_{mode}_{comb}"])
    g = npo.sparse_grad_sum(d["rows_mod"], d["offsets"], B, F, d["dout"], "mean")
    assert np.array_equal(np.array(sorted(g)), d["grad_rows"])
    assert np.array_equal(np.stack([g[k] for k in sorted(g)]), d["grad_vals"])


@pytest.mark.parametrize("name", ["il_config2.npz", "il_defaults_u128.npz", "il_dropout.npz",
                                  "il_multihead_u8.npz"])
def test_golden_interacting_layer(name):
    d = gold(name)
    B, F, E, U, H, L, res = (int(v) for v in d["shape"])
    y = npo.interacting_layer(d["x"].astype(np.float64), d["W"].astype(np.float64),
                              d["bias"].astype(np.float64), d["gamma"].astype(np.float64),
                              d["beta"].astype(np.float64), L, H, bool(res),
                              drop_rate=float(d["drop"]), seed=int(d["seed"]))
    assert np.array_equal(y, d["y"])


def test_golden_autoint_forward_and_loss():
    d = gold("autoint_config2.npz")
    B, F, E = d["ids"].shape[0], 26, 16
    x0, rows = npo.embedding_lookup(d["ids"], None, B, F, d["row_base"], d["bucket"],
                                    d["table"].astype(np.float64))
    assert np.array_equal(rows, d["rows"])
    il = dict(W=d["il_W"].astype(np.float64), bias=np.zeros(64), gamma=np.ones(16), beta=np.zeros(16))
    deep = [(d["W1"].astype(np.float64), np.zeros(32)), (d["W2"].astype(np.float64), np.zeros(16))]
    logits = [(d["W3"].astype(np.float64), np.zeros(1))]
    cfg = dict(layer_num=3, head_num=2, use_res=True, mlp_activation="relu", logits_activation="sigmoid")
    s, p = npo.autoint_forward(x0, il, deep, logits, cfg)
    assert np.array_equal(p, d["p"])
    assert npo.cross_entropy(d["labels"].astype(np.float64), p) == float(d["loss"])


@pytest.mark.parametrize("L,H,res,drop", [(1, 1, True, 0.0), (3, 2, True, 0.0), (2, 2, False, 0.0),
                                          (2, 2, True, 0.3)])
def test_numpy_vs_torch_twin(L, H, res, drop):
    rng = np.random.default_rng(L * 10 + H)
    B, F, E, U = 3, 7, 8, 8
    x = rng.uniform(-0.5, 0.5, (B, F, E))
    W = rng.normal(size=(E, 4 * U)) * 0.4
    b = rng.normal(size=4 * U) * 0.1
    g = rng.uniform(0.5, 1.5, U)
    be = rng.normal(size=U) * 0.1
    a = npo.interacting_layer(x, W, b, g, be, L, H, res, drop_rate=drop, seed=9)
    t = tr.interacting_layer(*(torch.tensor(v) for v in (x, W, b, g, be)), L, H, res,
                             drop_rate=drop, seed=9).numpy()
    assert np.max(np.abs(a - t)) < 1e-12


def test_torch_twin_gradients_finite_differences():
    """The autograd twin's gradients (the GPU backward's reference) vs central differences."""
    torch.manual_seed(0)
    B, F, E, U, H, L = 2, 5, 4, 4, 2, 2
    x = (torch.rand(B, F, E, dtype=torch.float64) - 0.5).requires_grad_(True)
    W = (torch.randn(E, 4 * U, dtype=torch.float64) * 0.5).requires_grad_(True)
    b = (torch.randn(4 * U, dtype=torch.float64) * 0.1 + 0.05).requires_grad_(True)
    g = (torch.rand(U, dtype=torch.float64) + 0.5).requires_grad_(True)
    be = (torch.randn(U, dtype=torch.float64) * 0.1).requires_grad_(True)
    fn = lambda *a: tr.interacting_layer(*a, L, H, True, 1e-6)  # noqa: E731
    assert torch.autograd.gradcheck(fn, (x, W, b, g, be), eps=1e-6, atol=1e-5)


def test_cross_entropy_and_clip_gradient():
    s = torch.tensor([[-0.1], [0.5], [1.2], [1e-7]], dtype=torch.float64, requires_grad=True)
    y = torch.tensor([[1.0], [0.0], [1.0], [0.0]], dtype=torch.float64)
    p = torch.clamp(s, 1e-6, 1.0)
    loss = tr.cross_entropy(y, p)
    loss.backward()
    ref = npo.cross_entropy(y.numpy(), np.clip(s.detach().numpy(), 1e-6, 1.0))
    assert abs(float(loss) - ref) < 1e-15
    # ClipByValue gradient: zero outside [1e-6, 1]
    assert s.grad[0, 0] == 0 and s.grad[2, 0] == 0 and s.grad[3, 0] == 0 and s.grad[1, 0] != 0


def test_adam_forms():
    p, g = np.array([1.0, -2.0]), np.array([0.5, -0.25])
    p1, m, v = npo.adam_dense(p, g, np.zeros(2), np.zeros(2), 1, 0.1)
    # first bias-corrected Adam step moves each weight by ~lr * sign(g)
    assert np.allclose(p - p1, 0.1 * np.sign(g), rtol=1e-5)
    w1, m, v = npo.adam_sparse(p, g, np.zeros(2), np.zeros(2), 0.1)
    assert np.allclose(p - w1, 0.1 * 0.1 * g / (1e-8 + np.sqrt(0.001 * g * g)))
    w2, g2 = npo.adagrad_sparse(p, g, np.full(2, 0.1), 0.1)
    assert np.allclose(w2, p - 0.1 * g / np.sqrt(0.1 + g * g))


# ------------------------------------------------------------------------------------------
# H6/H7 DIN pools and the H1 sequence lookup
# ------------------------------------------------------------------------------------------
def test_golden_din_pools():
    d = gold("din_relu_sum.npz")
    f64 = lambda k: d[k].astype(np.float64)  # noqa: E731
    out = npo.din_pool(f64("q"), f64("keys"), f64("values"), d["lengths"], f64("W1"), f64("b1"),
                       f64("W2"), f64("b2"))
    assert np.array_equal(out, d["out"])
    d = gold("din_staytime_softmax.npz")
    f64 = lambda k: d[k].astype(np.float64)  # noqa: E731
    out, probs = npo.din_softmax_pool(f64("q"), f64("facts"), d["mask"], f64("W1"), f64("b1"),
                                      f64("W2"), f64("b2"), return_probs=True)
    assert np.array_equal(out, d["out"]) and np.array_equal(probs, d["probs"])


def test_golden_sequence_lookup():
    d = gold("sequence_lookup.npz")
    T = int(d["T"])
    B = d["offsets"].size - 1
    emb, mask, rows = npo.sequence_lookup(d["ids"], d["offsets"], B, T, 0, d["table"].shape[0],
                                          d["table"].astype(np.float64), "splitmix")
    assert np.array_equal(emb, d["emb"]) and np.array_equal(mask, d["mask"])
    assert np.array_equal(rows, d["rows"])
    lens = np.diff(d["offsets"])
    assert np.array_equal(mask.sum(1), np.minimum(lens, T))


def test_din_semantics():
    """din.py: masked positions contribute nothing (their keys/values are irrelevant);
    staytime/layer.py: a fully masked row is the uniform mean of the facts, and masked facts
    are ignored otherwise."""
    rng = np.random.default_rng(3)
    B, T, H = 4, 6, 16
    q, k, v = rng.normal(size=(B, H)), rng.normal(size=(B, T, H)), rng.normal(size=(B, T, H))
    W1, b1 = rng.normal(size=(3 * H, 16)) * 0.3, rng.normal(size=16) * 0.1
    W2, b2 = rng.normal(size=(16, 1)), np.array([0.1])
    lens = np.array([6, 2, 0, 4])
    a = npo.din_pool(q, k, v, lens, W1, b1, W2, b2)
    k2, v2 = k.copy(), v.copy()
    k2[1, 2:] = 99.0
    v2[1, 2:] = -99.0
    assert np.allclose(a, npo.din_pool(q, k2, v2, lens, W1, b1, W2, b2))
    assert np.all(a[2] == 0)
    W1s = rng.normal(size=(4 * H, 16)) * 0.3
    mask = np.ones((B, T), bool)
    mask[0] = False
    mask[3, 4:] = False
    o = npo.din_softmax_pool(q, k, mask, W1s, b1, W2, b2)
    assert np.allclose(o[0], k[0].mean(0))
    k3 = k.copy()
    k3[3, 4:] = 5.0
    o3 = npo.din_softmax_pool(q, k3, mask, W1s, b1, W2, b2)
    assert np.allclose(o3[3], o[3]) and np.allclose(o3[:3], o[:3])


@pytest.mark.parametrize("variant", [0, 1])
def test_din_twin_matches_numpy_and_finite_differences(variant):
    rng = np.random.default_rng(5 + variant)
    B, T, H = 3, 5, 4
    q, k, v = rng.normal(size=(B, H)), rng.normal(size=(B, T, H)), rng.normal(size=(B, T, H))
    nb = 3 if variant == 0 else 4
    W1, b1 = rng.normal(size=(nb * H, 16)) * 0.4, rng.normal(size=16) * 0.2 + 0.1
    W2, b2 = rng.normal(size=(16, 1)) * 0.5, np.array([0.3])
    lens = np.array([5, 3, 1])
    mask = np.arange(T)[None, :] < lens[:, None]
    if variant == 0:
        a = npo.din_pool(q, k, v, lens, W1, b1, W2, b2)
        fn = lambda q_, k_, v_, W1_, b1_, W2_, b2_: tr.din_pool(q_, k_, v_, lens, W1_, b1_, W2_, b2_)  # noqa: E731
        args = [q, k, v, W1, b1, W2, b2]
    else:
        a = npo.din_softmax_pool(q, k, mask, W1, b1, W2, b2)
        fn = lambda q_, k_, W1_, b1_, W2_, b2_: tr.din_softmax_pool(q_, k_, torch.from_numpy(mask),  # noqa: E731
                                                                    W1_, b1_, W2_, b2_)
        args = [q, k, W1, b1, W2, b2]
    ts = [torch.tensor(x, requires_grad=True) for x in args]
    assert np.max(np.abs(fn(*ts).detach().numpy() - a)) < 1e-12
    assert torch.autograd.gradcheck(fn, tuple(ts), eps=1e-6, atol=1e-5)


def test_keras_auc_restatement():
    """oracle keras_auc: 1 for separable scores, 0.5 for constant ones, within the 200-threshold
    binning error of the exact ROC AUC (scikit-learn) on random scores."""
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    y = (rng.uniform(size=5000) < 0.3).astype(np.float32)
    assert npo.keras_auc(np.where(y > 0, 0.9, 0.1), y) == pytest.approx(1.0)
    assert npo.keras_auc(np.full(5000, 0.4), y) == pytest.approx(0.5)
    p = np.clip(rng.beta(2, 5, size=5000) + 0.15 * y, 0, 1)
    assert abs(npo.keras_auc(p, y) - roc_auc_score(y, p)) < 3e-3
    w = rng.uniform(0.5, 2, size=5000)
    assert abs(npo.keras_auc(p, y, w) - roc_auc_score(y, p, sample_weight=w)) < 3e-3
    m = npo.ctr_metrics(p, y)
    assert m["ctr"] == pytest.approx(y.mean()) and m["copc"] == pytest.approx(y.sum() / p.sum())
