"""Flat parameter blocks and the model-wide dense parameter arena.

Every layer allocates its parameters as views into ONE flat fp32 block (params) with a twin block
for gradients, so the fused kernels can write a layer's whole gradient (e.g. the InteractingLayer's
[dW | db | dgamma | dbeta]) with one store stream and accumulate it in place.  `ParamArena.pack`
then moves every dense parameter of a model into a single flat buffer: the dense optimizer is one
launch (rs_dense_adam) and the data-parallel gradient all-reduce is one bucket.
"""
from __future__ import annotations

import math
from typing import Iterable, Sequence

import torch
from torch import nn


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator | None) -> None:
    """Keras 'glorot_uniform' (the Dense default kernel_initializer): U(-l, l), l = sqrt(6/(in+out))."""
    limit = math.sqrt(6.0 / float(fan_in + fan_out))
    with torch.no_grad():
        t.copy_((torch.rand(t.shape, generator=gen, dtype=torch.float64) * 2.0 - 1.0) * limit)


class FlatBlock:
    """Contiguous param + grad storage for one layer; hands out Parameter views in order."""

    def __init__(self, shapes: Sequence[Sequence[int]], device, dtype=torch.float32):
        self.shapes = [tuple(s) for s in shapes]
        self.sizes = [math.prod(s) for s in self.shapes]
        n = sum(self.sizes)
        self.data = torch.zeros(n, device=device, dtype=dtype)
        self.grad = torch.zeros(n, device=device, dtype=dtype)

    def params(self) -> list[nn.Parameter]:
        out, off = [], 0
        for shp, sz in zip(self.shapes, self.sizes):
            p = nn.Parameter(self.data[off:off + sz].view(shp))
            p.grad = self.grad[off:off + sz].view(shp)
            out.append(p)
            off += sz
        return out


def grads_contiguous(params: Sequence[nn.Parameter]) -> torch.Tensor | None:
    """If the params' .grad tensors are consecutive in one storage (a FlatBlock or the arena),
    return a flat view covering all of them, else None."""
    gs = [p.grad for p in params]
    if any(g is None or not g.is_contiguous() for g in gs):
        return None
    base = gs[0]
    expect = base.data_ptr()
    for g in gs:
        if g.data_ptr() != expect or g.untyped_storage().data_ptr() != base.untyped_storage().data_ptr():
            return None
        expect += g.numel() * g.element_size()
    n = sum(g.numel() for g in gs)
    off = base.storage_offset()
    return base.as_strided((n,), (1,), off)


class ParamArena:
    """One flat buffer for all dense parameters of a model (+ grads + Adam moments)."""

    def __init__(self, params: Iterable[nn.Parameter], device=None, align: int = 1):
        """align > 1: each LAYER's parameters (a run of params adjacent in one storage, e.g. one
        FlatBlock: [kernel, bias] or a packed [W1 b1 W2 b2]) led by a weight matrix start at a
        multiple of ``align`` floats; parameters inside a layer stay packed.  The GEMM engine takes its vectorised
        (float4) operand path only for 16-byte aligned weights, so the generic Trainer uses 16
        (64 B); the gaps hold zeros in data, grad and the Adam moments (a zero gradient leaves
        them zero).  The AutoInt step keeps align = 1 (its fused kernels address the arena
        by packed offsets)."""
        self.params = [p for p in params]
        if not self.params:
            raise ValueError("ParamArena needs at least one parameter")
        device = device or self.params[0].device
        offs, off, prev = [], 0, None
        for p in self.params:
            st = (p.untyped_storage().data_ptr(), p.storage_offset())
            same_layer = prev is not None and st[0] == prev[0] and st[1] == prev[1]
            if align > 1 and not same_layer and p.dim() >= 2:  # a layer led by a weight matrix
                off = (off + align - 1) // align * align
            offs.append(off)
            off += p.numel()
            prev = (st[0], st[1] + p.numel())
        self.n = off
        self.data = torch.zeros(self.n, device=device, dtype=torch.float32)
        self.grad = torch.zeros(self.n, device=device, dtype=torch.float32)
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                sz = p.numel()
                self.data[off:off + sz].copy_(p.detach().reshape(-1))
                p.data = self.data[off:off + sz].view(p.shape)
                p.grad = self.grad[off:off + sz].view(p.shape)

    def zero_grad(self) -> None:
        self.grad.zero_()
