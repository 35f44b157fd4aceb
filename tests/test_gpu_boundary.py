"""GPU checks of the C-ABI's defensive behaviour:

* a (row_base, bucket) pair that points outside the table: rs_embedding_lookup_fwd and
  rs_il_fwd_gather never read past the table -- the id contributes a zero row and its row index
  is -1 (skipped by every push);
* a list-mode push that claims more rows than the touched list holds: the sparse optimizer
  updates only the first touched_cap rows and SparseTable.check_overflow() raises.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_lookup_rows_outside_table_are_zero_and_minus_one():
    from recommendsystem_amd._lib import call, ptr, stream_handle
    rows_n, dim, B, F = 100, 16, 8, 3
    table = torch.rand(rows_n, dim, device=DEV)
    row_base = torch.tensor([0, 50, 90], dtype=torch.int64, device=DEV)
    bucket = torch.tensor([50, 40, 30], dtype=torch.int64, device=DEV)  # field 2 reaches row 119
    ids = torch.arange(B * F, dtype=torch.int64, device=DEV).reshape(B, F) * 7
    out = torch.full((B, F, dim), 9.0, device=DEV)
    rows = torch.empty(B * F, dtype=torch.int32, device=DEV)
    call("rs_embedding_lookup_fwd", stream_handle(), ptr(ids), None, B, F, ptr(row_base), ptr(bucket),
         0, 0, ptr(table), rows_n, dim, ptr(out), F * dim, dim, ptr(rows))
    torch.cuda.synchronize()
    want = (row_base[None, :] + ids % bucket[None, :]).reshape(-1).cpu().numpy()
    bad = want >= rows_n
    assert bad.any() and (~bad).any()
    got = rows.cpu().numpy()
    assert np.array_equal(got[~bad], want[~bad]) and np.all(got[bad] == -1)
    o = out.reshape(B * F, dim).cpu()
    assert torch.all(o[torch.from_numpy(bad)] == 0)
    assert torch.equal(o[torch.from_numpy(~bad)], table.cpu()[torch.from_numpy(want[~bad])])


def test_il_fwd_gather_rows_outside_table():
    from recommendsystem_amd._lib import call, ptr, stream_handle
    B, F, E, U, H, L = 4, 26, 16, 16, 2, 3
    rows_n = 26 * 10
    table = torch.rand(rows_n, E, device=DEV)
    row_base = torch.arange(0, 260, 10, dtype=torch.int64, device=DEV)
    bucket = torch.full((F,), 10, dtype=torch.int64, device=DEV)
    bucket[-1] = 1000  # the last field can hash past the end
    ids = torch.randint(0, 5000, (B, F), dtype=torch.int64, device=DEV)
    ids[:, -1] = torch.tensor([3, 500, 7, 999])
    W = torch.rand(E, 4 * U, device=DEV) * 0.2
    bias, gamma, beta = (torch.zeros(4 * U, device=DEV), torch.ones(U, device=DEV),
                         torch.zeros(U, device=DEV))
    x = torch.empty(B, F * E, device=DEV)
    rows = torch.empty(B * F, dtype=torch.int32, device=DEV)
    y = torch.empty(B, F * U, device=DEV)
    xs = torch.empty(L - 1, B, F, U, device=DEV)
    call("rs_il_fwd_gather", stream_handle(), ptr(ids), ptr(row_base), ptr(bucket), 0, ptr(table),
         rows_n, ptr(x), ptr(rows), B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta),
         1e-14, 1, 0.0, 0, ptr(y), F * U, ptr(xs))
    torch.cuda.synchronize()
    r = rows.reshape(B, F).cpu().numpy()
    assert list(r[:, -1]) == [253, -1, 257, -1]
    xr = x.reshape(B, F, E).cpu()
    assert torch.all(xr[1, -1] == 0) and torch.all(xr[3, -1] == 0)
    assert torch.equal(xr[0, -1], table[253].cpu())
    assert torch.isfinite(y).all()


def test_touched_list_overflow_is_reported_and_recovered():
    """A push claiming more rows than the touched list holds: every claimed row is still updated
    (exactly once per step: the list launch takes the first cap rows, the gated recovery sweep
    the rest), flags and gradient rows are released, the overflow is reported, and a later
    step without overflow updates its rows normally."""
    from recommendsystem_amd.embedding import SparseAdam, SparseTable
    t = SparseTable(1000, 8, SparseAdam(1e-2), device=DEV, seed=1, max_touched=4)
    B, F = 10, 1
    rows = torch.arange(0, 100, 10, dtype=torch.int32, device=DEV)  # 10 distinct rows > cap 4
    dout = torch.ones(B, 8, device=DEV)
    w0 = t.weight.clone()
    t.accumulate(rows, None, B, F, dout, 8, 8, 0)
    t.step()
    torch.cuda.synchronize()
    changed = (t.weight != w0).any(dim=1).nonzero().reshape(-1).cpu().tolist()
    assert sorted(changed) == rows.cpu().tolist()
    # first sparse Adam step without bias correction: w -= lr * m / (eps + sqrt(v)), m = .1 g,
    # v = .001 g^2 -> lr * .1 / sqrt(.001) for g = 1
    step = float((w0 - t.weight)[rows.long()].mean())
    assert abs(step - 1e-2 * 0.1 / (1e-8 + 0.001 ** 0.5)) < 1e-6
    assert bool((t.flag == -1).all()) and bool((t.grad == 0).all())
    assert int(t.n_touched[0]) == 0
    with pytest.raises(RuntimeError, match="overflow"):
        t.check_overflow()
    t.check_overflow()  # the sticky word was cleared by the report
    w1 = t.weight.clone()
    t.accumulate(rows[:3], None, 3, F, dout[:3], 8, 8, 0)
    t.step()
    torch.cuda.synchronize()
    changed = (t.weight != w1).any(dim=1).nonzero().reshape(-1).cpu().tolist()
    assert sorted(changed) == rows[:3].cpu().tolist()
    t.check_overflow()
