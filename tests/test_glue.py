"""CPU checks of the autograd glue that replaces per-view backward chains in the composed models
(models.py split_cols; the staytime front end is tested on the GPU in
tests/test_gpu_glue.py): same gradients as plain slicing, in float64."""
import torch

from recommendsystem_amd.models import split_cols


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
