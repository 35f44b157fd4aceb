"""CPU checks of the autograd glue that replaces per-view backward chains in the composed models
(models.py split_cols / _EmbFanoutFn): same gradients as plain slicing, in float64."""
import torch

from recommendsystem_amd.models import _EmbFanoutFn, split_cols


def test_split_cols_grad_matches_slicing():
    torch.manual_seed(0)
    y = torch.randn(5, 12, dtype=torch.float64, requires_grad=True)
    sizes = [3, 5, 4]

    def loss(parts):
        return (parts[0].sin().sum() + (parts[2] ** 2).sum() * 0.5)  # parts[1] unused: None grad

    loss(split_cols(y, sizes)).backward()
    g1 = y.grad.clone()
    y.grad = None
    loss(list(torch.split(y, sizes, dim=1))).backward()
    assert torch.equal(g1, y.grad)
    assert torch.autograd.gradcheck(lambda t: tuple(split_cols(t, sizes)), (y.detach().requires_grad_(),))


def test_emb_fanout_grad_matches_views():
    torch.manual_seed(1)
    emb = torch.randn(3, 9, 32, dtype=torch.float64, requires_grad=True)
    bias = torch.tensor([0, 4, 4, 8])   # repeated field: index_add accumulates
    q = [2, 7, 7]

    def loss(gen, gate, qs):
        return (gen.cos().sum() + (gate ** 2).sum() * 0.3 + sum((x * (i + 1)).sum() for i, x in enumerate(qs))
                + emb.reshape(3, -1)[:, ::5].sum())

    gen, gate, *qs = _EmbFanoutFn.apply(emb, bias, q)
    loss(gen, gate, qs).backward()
    g1 = emb.grad.clone()
    emb.grad = None
    gen = emb[:, :, 0:16]
    loss(gen, emb.index_select(1, bias)[:, :, 16:32].reshape(3, -1), [gen[:, i, :] for i in q]).backward()
    assert torch.allclose(g1, emb.grad, rtol=0, atol=1e-12)
