"""Config 2's bf16 compute mode (BASELINE.json configs[1] "batch 4096 bf16"; rs_set_math_mode):
the InteractingLayer projections / dW / dx and the fused head's layer-1/2 GEMMs take bf16-rounded
operands with fp32 accumulation; master weights, table and optimizer state stay fp32.

Two oracles, both fp64 (oracle/torch_ref.py):
  * the bf16-EMULATING oracle (cfg["bf16"]: the same operands rounded to bf16 at the same GEMMs,
    forward and backward) -- the kernels must agree with it to fp32 accumulation noise, except
    where an fp32-vs-fp64 difference of ~1e-7 in an operand flips its bf16 rounding (probability
    ~2^-16 per rounded operand; a flip moves that operand by one bf16 ulp, 2^-8 relative).
    Tolerance: p within BF16_EMU_ATOL everywhere, within 1e-5 for >= 90 % of samples, median
    within 1e-6 (measured on MI355X, B = 512: max 7.3e-5, 97.7 % within 1e-5, median 2.8e-8).
  * the fp32-semantics oracle (the reference's math) -- the documented accuracy of the mode:
    p within BF16_ATOL, loss within BF16_LOSS_RTOL relative.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import torch_ref as tr
from _tol import to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"

BF16_EMU_ATOL = 1e-3     # p vs the bf16-emulating oracle (rare rounding flips), first step
BF16_EMU_ATOL_LATER = 1e-2  # later steps: Adam's sign-like first update turns flip-sized gradient
                            # differences into lr-sized weight differences (measured 2.0e-3)
BF16_ATOL = 2e-2         # p vs the fp32-semantics oracle: the bf16 mode's accuracy
BF16_LOSS_RTOL = 5e-3    # loss vs the fp32-semantics oracle


def _zipf(rng, shape, vocab, a=1.2):
    return np.minimum(rng.zipf(a, size=shape) - 1, vocab - 1).astype(np.int64)


def _setup(B, seed=0, vocab=100_000):
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    cfg = AutoIntConfig(vocab_per_field=vocab, compute_dtype="bf16")
    model = AutoInt(cfg, device=DEV, seed=seed, max_batch=B)
    trainer = AutoIntTrainer(model, B)
    il = {"W": to_np(model.interact.kernel), "bias": to_np(model.interact.bias),
          "gamma": to_np(model.interact.gamma), "beta": to_np(model.interact.beta)}
    deep = [(to_np(l.kernel), to_np(l.bias)) for l in model.deep.layers]
    logits = [(to_np(l.kernel), to_np(l.bias)) for l in model.logits.layers]
    ocfg = dict(layer_num=cfg.layer_num, head_num=cfg.head_num, use_res=cfg.use_res,
                mlp_activation=cfg.mlp_activation, logits_activation=cfg.logits_activation)

    def oracle(bf16):
        return tr.AutoIntCPU(model.table.weight.cpu().numpy(),
                             to_np(model.embedding.row_base).astype(np.int64),
                             to_np(model.embedding.bucket).astype(np.int64), il, deep, logits,
                             dict(ocfg, bf16=bf16), lr_dense=cfg.lr_dense,
                             lr_sparse=cfg.lr_sparse, dtype=torch.float64)
    return cfg, model, trainer, oracle


def _oracle_p(ref, ids, labels):
    B, F = ids.shape
    rows = ref.rows(ids).reshape(-1)
    x0 = ref.table.index_select(0, rows).reshape(B, F, -1)
    ilr = {n[3:]: v for n, v in ref.params.items()}
    with torch.no_grad():
        _, p = tr.autoint_forward(x0, ilr, ref.deep, ref.logits, ref.cfg)
        loss = tr.cross_entropy(labels.double(), p)
    return p.numpy().reshape(-1), float(loss)


def test_bf16_mode_rejects_unsupported_shapes():
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    cfg = AutoIntConfig(num_fields=40, vocab_per_field=100, compute_dtype="bf16")
    with pytest.raises(ValueError, match="bf16"):
        AutoIntTrainer(AutoInt(cfg, device=DEV, max_batch=64), 64)


def test_bf16_il_entry_point_refuses_fp32_only_shapes():
    """A shape without bf16 kernels returns RS_ERR_UNSUPPORTED in bf16 mode (never fp32)."""
    from recommendsystem_amd import _lib
    from recommendsystem_amd._lib import RecsysKernelError, call, ptr, stream_handle
    B, F, E, U, H = 8, 40, 16, 16, 2
    x = torch.randn(B, F, E, device=DEV)
    W = torch.randn(E, 4 * U, device=DEV)
    b, g, be = torch.zeros(4 * U, device=DEV), torch.ones(U, device=DEV), torch.zeros(U, device=DEV)
    y = torch.empty(B, F * U, device=DEV)
    args = (stream_handle(), ptr(x), B, F, E, U, H, 1, ptr(W), ptr(b), ptr(g), ptr(be), 1e-14, 1,
            0.0, 0, ptr(y), F * U, None)
    call("rs_il_fwd", *args)  # fp32: fine
    with _lib.math_mode("bf16"):
        with pytest.raises(RecsysKernelError, match="-2"):
            call("rs_il_fwd", *args)
    assert _lib.load().rs_get_math_mode() == 0


@pytest.mark.parametrize("B", [512, 4096])
def test_bf16_step_matches_emulating_oracle(B):
    cfg, model, trainer, oracle = _setup(B)
    rng, lab_rng = np.random.default_rng(5), np.random.default_rng(6)
    F = cfg.num_fields
    pool_cpu = [(torch.from_numpy(_zipf(rng, (B, F), cfg.vocab_per_field)),
                 torch.from_numpy((lab_rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)))
                for _ in range(2)]
    pool = [(i.to(DEV), l.to(DEV)) for i, l in pool_cpu]
    emu, f32 = oracle(True), oracle(False)
    trainer.capture_pool(pool, warmup=0)
    for k, (ids_c, lab_c) in enumerate(pool_cpu):
        p_emu, loss_emu = _oracle_p(emu, ids_c, lab_c)
        p_f32, loss_f32 = _oracle_p(f32, ids_c, lab_c)
        trainer.step_pool(k)
        torch.cuda.synchronize()
        p = to_np(trainer.p).reshape(-1)
        d_emu, d_f32 = np.abs(p - p_emu), np.abs(p - p_f32)
        print(f"B={B} step {k}: |p-p_emu| max {d_emu.max():.3e} p99 {np.quantile(d_emu, .99):.3e} "
              f"median {np.median(d_emu):.3e}; |p-p_f32| max {d_f32.max():.3e} median "
              f"{np.median(d_f32):.3e}; loss {float(trainer.loss):.7f} emu {loss_emu:.7f} "
              f"f32 {loss_f32:.7f}")
        assert d_emu.max() <= (BF16_EMU_ATOL if k == 0 else BF16_EMU_ATOL_LATER), d_emu.max()
        if k == 0:
            assert np.mean(d_emu <= 1e-5) >= 0.90, np.mean(d_emu <= 1e-5)
        assert np.median(d_emu) <= 1e-6, np.median(d_emu)
        assert abs(float(trainer.loss) - loss_emu) <= 1e-5 + 1e-5 * abs(loss_emu)
        assert d_f32.max() <= BF16_ATOL, d_f32.max()
        assert abs(float(trainer.loss) - loss_f32) <= BF16_LOSS_RTOL * abs(loss_f32)
        emu.step(ids_c, lab_c)   # both oracles follow the step (same batches, own math)
        f32.step(ids_c, lab_c)
    # after two steps the weights track the emulating oracle (Adam's first steps are sign-like:
    # loose absolute bound, lr = 5e-5 per step)
    got = torch.cat([q.detach().reshape(-1).double().cpu() for q in model.parameters()]).numpy()
    want = torch.cat([q.detach().reshape(-1) for q in emu.dense_list]).numpy()
    frac_bad = np.mean(np.abs(got - want) > 2e-6 + 1e-4 * np.abs(want))
    print(f"dense params off the emulating oracle after 2 steps: {frac_bad:.4f}")
    assert frac_bad <= 0.1, frac_bad


def test_bf16_training_tracks_fp32():
    """40 steps over 4 batches (lr 1e-3, memorising them: loss 0.89 -> 0.08): the bf16-mode loss
    curve stays within 5 % of the fp32 one at every step (measured: 2.4 %)."""
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    B = 1024
    rng = np.random.default_rng(11)
    losses = {}
    for dt in ("f32", "bf16"):
        cfg = AutoIntConfig(vocab_per_field=2000, compute_dtype=dt, lr_dense=1e-3, lr_sparse=1e-3)
        model = AutoInt(cfg, device=DEV, seed=4, max_batch=B)
        trainer = AutoIntTrainer(model, B)
        r = np.random.default_rng(11)
        pool = [(torch.from_numpy(_zipf(r, (B, 26), 2000)).to(DEV),
                 torch.from_numpy((r.uniform(size=(B, 1)) < 0.25).astype(np.float32)).to(DEV))
                for _ in range(4)]
        trainer.capture_pool(pool, warmup=1)
        ls = []
        for i in range(40):
            ls.append(float(trainer.step_pool(i)))
        losses[dt] = np.array(ls)
    del rng
    rel = np.abs(losses["bf16"] - losses["f32"]) / losses["f32"]
    print("loss f32", losses["f32"][[0, 9, 19, 39]], "bf16", losses["bf16"][[0, 9, 19, 39]])
    assert rel.max() <= 5e-2, rel.max()
    assert losses["bf16"][-4:].mean() < losses["bf16"][:4].mean()  # it trains
