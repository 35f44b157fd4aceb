"""The scan-mode sparse Adam sweep alone (rs_sparse_adam_scan, dim 16) at a given table size and
number of marked rows, for kernel-duration measurement under rocprofv3 (--kernel-trace --stats):
  python tools/sweep_bench.py ROWS MARKED [REPS]
Each rep re-marks the rows (torch index_fill) before the sweep."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle


def main(nrows=2_600_000, k=0, reps=50, dim=16):
    _lib.load()
    dev = torch.device("cuda")
    tab, m, v, g = (torch.zeros(nrows, dim, device=dev) for _ in range(4))
    flag = torch.full((nrows,), -1, dtype=torch.int32, device=dev)
    idx = torch.randperm(nrows, device=dev)[:k]
    for _ in range(reps):
        if k:
            flag.index_fill_(0, idx, -2)
        call("rs_sparse_adam_scan", stream_handle(), ptr(tab), ptr(m), ptr(v), ptr(g), ptr(flag),
             nrows, dim, 1e-3, 0.9, 0.999, 1e-8, 1.0)
    torch.cuda.synchronize()
    assert int((flag == -2).sum()) == 0
    print(nrows, k, "ok")


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a)
