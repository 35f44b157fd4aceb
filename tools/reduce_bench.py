"""Time rs_partials_reduce_adam alone (back-to-back launches, HIP events) on config-2 partial
shapes: IL (1024 x 1120), head (256 x 14306), both, with and without the Adam update."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import stream_handle


def time_graph(fn, reps):
    """Device time per launch: `reps` launches captured into one graph, replayed (no host gaps)."""
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 2)


def main(reps=50):
    _lib.load()
    dev = torch.device("cuda")
    il = torch.randn(1024, 1120, device=dev)
    hd = torch.randn(256, 14306, device=dev)
    n = 1120 + 14305
    p, m, v, g = (torch.zeros(n, device=dev) for _ in range(4))
    loss = torch.zeros(1, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    done = torch.zeros(288, dtype=torch.int32, device=dev)
    segs_il = [(il.data_ptr(), 1120, 1024, 1120, g.data_ptr(), 1.0, 0)]
    segs_hd = [(hd.data_ptr(), 14306, 256, 14305, g.data_ptr() + 4 * 1120, 1.0, 1120),
               (hd.data_ptr() + 4 * 14305, 14306, 256, 1, loss.data_ptr(), 1.0 / 4096, -1)]
    out = {}
    for name, segs in (("il", segs_il), ("head", segs_hd), ("both", segs_il + segs_hd)):
        for adam in (False, True):
            fn = lambda: _lib.partials_reduce_adam(stream_handle(), segs, p, m, v, step, done, 1e-3,
                                                   0.9, 0.999, 1e-8, 1.0, adam)
            out[f"{name}{'_adam' if adam else ''}_us"] = time_graph(fn, reps)
    from recommendsystem_amd._lib import call, ptr
    out["floor_tiny_kernel_us"] = time_graph(
        lambda: call("rs_l1l2_grad", stream_handle(), ptr(p), ptr(g), 16, 0.0, 0.0), reps)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
