"""Parity at the benchmarked sizes (VERDICT r01 "pin the benchmarked step").

* config 2: the EXACT step bench.py times -- AutoIntTrainer at B = 4096 over AutoIntConfig()
  (26 fields x 100k rows, lr 5e-5), Zipf(1.2) ids, Bernoulli(0.25) labels, one captured HIP graph
  per pool batch (capture_pool / step_pool) -- against the fp64 oracle (oracle/torch_ref.py
  AutoIntCPU) for two steps on two different batches:
    - predictions p (clip(sigmoid logits)) within 1e-5 absolute  (north_star "fp32 logits within
      1e-5"),  loss within 1e-5;
    - the step-1 dense gradient (left in the arena by the fused reduce) within the gradient
      tolerance of tests/_tol.py;  hashed rows bit-exact;
    - dense parameters and the whole 2.6M-row table after each step within 2e-6 + 1e-4 |ref|,
      except where Adam turns fp32 rounding of an ill-conditioned gradient into a visible
      update difference (|g| below 1e-6 of the largest |g| of its tensor, or -- table rows --
      a row gradient whose contributions cancel to under 1 % of their summed magnitude): those
      entries are counted and must be rare.
Parity unpinned against TF itself (oracle/ctr_oracle.py header).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo
from oracle import torch_ref as tr
from _tol import adam_close as _adam_close, assert_close, assert_grad_close, to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _zipf(rng, shape, vocab, a=1.2):
    return np.minimum(rng.zipf(a, size=shape) - 1, vocab - 1).astype(np.int64)


@pytest.mark.parametrize("B", [4096, 512, 1000])
def test_bench_step_matches_oracle_full_size(B):
    """B = 4096: the one-wave IL backward (bwd4); B = 512 / 1000 (per-GPU batches of the
    strong-scaling series): the wide IL kernels (il_wide.hpp) under the same trainer."""
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    cfg = AutoIntConfig()
    model = AutoInt(cfg, device=DEV, seed=0, max_batch=B)
    trainer = AutoIntTrainer(model, B)
    rng, lab_rng = np.random.default_rng(2), np.random.default_rng(3)
    F = cfg.num_fields
    pool_cpu = [(torch.from_numpy(_zipf(rng, (B, F), cfg.vocab_per_field)),
                 torch.from_numpy((lab_rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)))
                for _ in range(2)]
    pool = [(i.to(DEV), l.to(DEV)) for i, l in pool_cpu]
    # the oracle starts from the same weights (fp64 copies), before any step
    il = {"W": to_np(model.interact.kernel), "bias": to_np(model.interact.bias),
          "gamma": to_np(model.interact.gamma), "beta": to_np(model.interact.beta)}
    deep = [(to_np(l.kernel), to_np(l.bias)) for l in model.deep.layers]
    logits = [(to_np(l.kernel), to_np(l.bias)) for l in model.logits.layers]
    ocfg = dict(layer_num=cfg.layer_num, head_num=cfg.head_num, use_res=cfg.use_res,
                mlp_activation=cfg.mlp_activation, logits_activation=cfg.logits_activation)
    ref = tr.AutoIntCPU(model.table.weight.cpu().numpy(), to_np(model.embedding.row_base).astype(np.int64),
                        to_np(model.embedding.bucket).astype(np.int64), il, deep, logits, ocfg,
                        lr_dense=cfg.lr_dense, lr_sparse=cfg.lr_sparse, dtype=torch.float64)
    # warmup=0: nothing runs before the graphs are recorded; replay k = training step k
    trainer.capture_pool(pool, warmup=0)
    ill_p = ill_t = None
    for k, (ids_c, lab_c) in enumerate(pool_cpu):
        # ---- oracle forward + gradients of this step (before its update) ----
        rows = ref.rows(ids_c).reshape(-1)
        x0 = ref.table.index_select(0, rows).reshape(B, F, -1).requires_grad_(True)
        ilr = {n[3:]: v for n, v in ref.params.items()}
        _, p_ref = tr.autoint_forward(x0, ilr, ref.deep, ref.logits, ocfg)
        loss_ref = tr.cross_entropy(lab_c.double(), p_ref)
        gx, *g_ref = torch.autograd.grad(loss_ref, [x0] + ref.dense_list)
        g_tab = torch.zeros_like(ref.table).index_add_(0, rows, gx.reshape(B * F, -1))
        g_abs = torch.zeros_like(ref.table).index_add_(0, rows, gx.abs().reshape(B * F, -1))
        # ---- GPU step k: one graph replay ----
        trainer.step_pool(k)
        torch.cuda.synchronize()
        assert_close(to_np(trainer.p), p_ref.detach().numpy(), 1e-5, what=f"step {k}: p")
        assert abs(float(trainer.loss) - float(loss_ref)) < 1e-5, (float(trainer.loss), float(loss_ref))
        if k == 0:
            got_rows = trainer.rows.cpu().numpy().astype(np.int64)
            assert np.array_equal(got_rows, rows.numpy()), "hashed rows differ from the oracle"
        g_got = to_np(model.arena.grad)
        off = 0
        for gr in g_ref:
            n = gr.numel()
            assert_grad_close(g_got[off:off + n], gr.numpy().reshape(-1), f"step {k}: dense grad")
            off += n
        # ---- oracle update, then compare the updated state ----
        ref.step(ids_c, lab_c)
        got_p = torch.cat([p.detach().reshape(-1).double().cpu() for p in model.parameters()]).numpy()
        want_p = torch.cat([p.detach().reshape(-1) for p in ref.dense_list]).numpy()
        gcat = np.concatenate([g.numpy().reshape(-1) for g in g_ref])
        ill_p = _adam_close(got_p, want_p, gcat, f"step {k}: dense params", prev_ill=ill_p)
        # the table: every row (untouched rows keep their values exactly)
        ill_t = _adam_close(model.table.weight.cpu().numpy(), ref.table.numpy(), g_tab.numpy(),
                            f"step {k}: table", grad_abs=g_abs.numpy(), prev_ill=ill_t)
