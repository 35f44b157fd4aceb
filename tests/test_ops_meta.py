"""CPU: the torch.ops.ctr custom ops register and their fake (meta) kernels produce the right
output shapes without a GPU (what torch.compile / FakeTensor tracing sees)."""
import torch

from recommendsystem_amd import ops  # noqa: F401


def test_meta_shapes():
    m = dict(device="meta")
    x, W = torch.empty(4, 26, 16, **m), torch.empty(16, 64, **m)
    b, g, be = torch.empty(64, **m), torch.empty(16, **m), torch.empty(16, **m)
    y, xs, sv = torch.ops.ctr.interacting_fwd(x, W, b, g, be, 3, 2, True, 1e-14, 0.0, 0)
    assert y.shape == (4, 26, 16) and xs.shape == (2, 4, 26, 16)
    assert sv.shape == (3 * 4 * (26 * 16 + 2 * 2 * 26),)  # the saved pair's O + softmax stats
    dx, dW, db, dg, dbe = torch.ops.ctr.interacting_bwd(y, x, xs, sv, W, b, g, be, 3, 2, True, 1e-14,
                                                        0.0, 0)
    assert dx.shape == x.shape and dW.shape == W.shape and dbe.shape == be.shape
    d = torch.ops.ctr.dense(torch.empty(5, 7, **m), torch.empty(7, 3, **m), torch.empty(3, **m), 1)
    assert d.shape == (5, 3)
    q, k = torch.empty(5, 16, **m), torch.empty(5, 9, 16, **m)
    out, probs = torch.ops.ctr.din_pool(q, k, k, None, None, torch.empty(64, 16, **m),
                                        torch.empty(16, **m), torch.empty(16, 1, **m),
                                        torch.empty(1, **m), 1)
    assert out.shape == (5, 16) and probs.shape == (5, 9)
    o, r = torch.ops.ctr.embedding_lookup(torch.empty(6, 4, dtype=torch.int64, **m), None,
                                          torch.empty(4, dtype=torch.int64, **m),
                                          torch.empty(4, dtype=torch.int64, **m), 0, 1,
                                          torch.empty(100, 16, **m))
    assert o.shape == (6, 4, 16) and r.shape == (24,) and r.dtype == torch.int32


def test_seed_roundtrip():
    from recommendsystem_amd.ops import _seed, _signed
    for s in (0, 1, 2**63 - 1, 2**63, 2**64 - 1, 12345678901234567890):
        assert _seed(_signed(s)) == s % 2**64
