import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommendsystem_amd.layers import InteractingLayer
from oracle import torch_ref as tr
B, F, E, U, H, L = int(os.environ.get("B", 64)), 26, 16, 16, 2, int(os.environ.get("L", 3))
rng = np.random.default_rng(6)
x = rng.uniform(-0.5, 0.5, size=(B, F, E)).astype(np.float32)
dy = rng.normal(size=(B, F, U)).astype(np.float32)
il = InteractingLayer(L, U, H, use_res=True, seed=8, device="cuda"); il.build((B, F, E), device="cuda")
with torch.no_grad():
    il.bias.uniform_(-0.1, 0.1); il.gamma.uniform_(0.5, 1.5); il.beta.uniform_(-0.2, 0.2)
xd = torch.from_numpy(x).cuda().requires_grad_(True)
il(xd).backward(torch.from_numpy(dy).cuda())
torch.cuda.synchronize()
P = [torch.from_numpy(t.detach().double().cpu().numpy()).requires_grad_(True) for t in (il.kernel, il.bias, il.gamma, il.beta)]
xr = torch.from_numpy(x).double().requires_grad_(True)
tr.interacting_layer(xr, *P, L, H, True).backward(torch.from_numpy(dy).double())
gW = il.kernel.grad.double().cpu().numpy(); rW = P[0].grad.numpy()
err = np.abs(gW - rW)
np.set_printoptions(precision=2, linewidth=200)
print("dx maxerr", np.abs(xd.grad.double().cpu().numpy() - xr.grad.numpy()).max())
print("dW maxerr", err.max(), "ref absmax", np.abs(rW).max())
print("per column-group max err (q,k,v,r):", [err[:, g*16:(g+1)*16].max() for g in range(4)])
print("per e max err:", err.max(axis=1))
print("rel err per group:", [ (err[:, g*16:(g+1)*16] / (np.abs(rW[:, g*16:(g+1)*16]) + 1e-3)).max() for g in range(4)])
for name, i in (("db", 1), ("dgamma", 2), ("dbeta", 3)):
    g = (il.bias, il.gamma, il.beta)[i - 1].grad.double().cpu().numpy()
    print(name, "maxerr", np.abs(g - P[i].grad.numpy()).max(), "absmax", np.abs(P[i].grad.numpy()).max())
