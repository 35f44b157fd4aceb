"""Headline benchmark: AutoInt CTR training samples/sec (BASELINE.json metric; configs[1]:
26 fields x 16-dim embeddings, batch 4096 per GPU, embedding + 3 x InteractingLayer + MLP).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: launched by torch.distributed.run, one process per GPU, RCCL over xGMI)

A step = one full training step on one synthetic batch: embedding lookup, IL x3, deep + logits
MLP, clip + cross_entropy, backward, (N > 1: dense all-reduce + sparse row exchange), dense Adam
and sparse Adam on the touched rows.  Batches (Zipf(1.2) ids over 26 x 100k vocab, Bernoulli(0.25)
labels) are pre-generated in HBM; each has its own captured HIP graph that reads it in place.
Prints ONE JSON line on rank 0 (value = samples/s over all ranks).

Batch semantics (SURVEY §8(c) decision 6): the primary series is STRONG scaling -- the global
batch (--global-batch, default 4096 = configs[1]) is split over the N ranks, per-GPU 4096 / N --
and the same run also times the WEAK series (per-GPU --batch, default 4096) as a nested "weak"
object.  At N = 1 the two are the same workload and only one is timed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# SURVEY §8(d) / BASELINE.md: algorithmic work of config 2
IL_FWD_FLOPS_PER_SAMPLE = 289_536          # 3 iterations x (proj 53,248 + QK^T 21,632 + PV 21,632)
TRAIN_FLOPS_PER_SAMPLE = 954_144           # IL 868,608 + MLP 85,536 (train = 3 x fwd)
FP32_PEAK_TFLOPS = 157.3                   # MI355X dense fp32 (MFMA == vector rate)
BF16_PEAK_TFLOPS = 2500.0                  # MI355X dense bf16 MFMA (BASELINE.md §3 basis)
HBM_PEAK_GBS = 8000.0
STEP_BYTES_PER_SAMPLE = 3_540              # ids + label + gather + row grads
ADAM_BYTES_PER_ROW = 384                   # + 6 x 16 x 4 B per unique touched row (sparse Adam)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only "
                         "to rehearse the DP path with several ranks on one GPU)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096,
                    help="per-GPU batch of the weak-scaling series (config 2: 4096)")
    ap.add_argument("--global-batch", type=int, default=4096,
                    help="global batch of the strong-scaling series (the primary line): per-GPU "
                         "batch = global / N")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="which series is the line's value (the other is nested unless --no-other)")
    ap.add_argument("--no-other", action="store_true",
                    help="N > 1: skip the nested other-scaling series")
    ap.add_argument("--pool", type=int, default=8, help="distinct pre-generated batches")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="bounded CPU sample: run whole train steps until this much time passed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="configs 3-5: run the autograd step eagerly instead of replaying graphs")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--trace-markers", action="store_true",
                    help="launch a marker kernel (torch.cuda._sleep: 'spin_kernel') right before "
                         "and right after the timed loop, outside the timed region, so a rocprofv3 "
                         "kernel trace can be cut to the timed steps (tools/prof_steps.py)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="config 2 compute mode of the headline line (f32 = the reference's math)")
    ap.add_argument("--no-bf16", action="store_true",
                    help="skip the nested bf16-mode result of the f32 run")
    ap.add_argument("--shard-table", action="store_true",
                    help="staytime at N > 1: owner-shard the 10M x 32 table over the ranks (N2, "
                         "all-to-all lookups and pushes) instead of replicating it")
    ap.add_argument("--workload", default="autoint",
                    choices=["autoint", "multi_head", "din", "staytime"],
                    help="autoint = the headline (configs[1]); the others are configs 3-5 at their "
                         "per-GPU batch (global batch / stated DP degree), same timing contract")
    return ap.parse_args()


def trace(msg):
    if os.environ.get("RS_BENCH_TRACE"):
        print(f"[bench rank {os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def zipf_ids(rng, B, F, vocab, a=1.2):
    z = rng.zipf(a, size=(B, F)) - 1
    return np.minimum(z, vocab - 1).astype(np.int64)


def time_kernel(fn, reps):
    """Average device duration of one launch of `fn` (HIP events on torch's current stream, which
    is the stream the kernel is enqueued on)."""
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3  # seconds


def cpu_baseline(cfg, model, batches_cpu, seconds):
    """the fp32 torch-CPU restatement (oracle/torch_ref.py::AutoIntCPU, TF op
    order) on the host cores, all cores and 1 thread, median of 3 runs each.  Bounded: each run
    takes whole train steps until seconds / 6 have passed (>= 2 steps)."""
    from oracle import torch_ref as tr
    # the box's CPU share (OMP_NUM_THREADS is set to it; affinity shows the whole machine)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    il = {k: v.detach().double().cpu().numpy() for k, v in
          dict(W=model.interact.kernel, bias=model.interact.bias, gamma=model.interact.gamma,
               beta=model.interact.beta).items()}
    deep = [(l.kernel.detach().cpu().numpy(), l.bias.detach().cpu().numpy()) for l in model.deep.layers]
    logits = [(l.kernel.detach().cpu().numpy(), l.bias.detach().cpu().numpy()) for l in model.logits.layers]
    ocfg = dict(layer_num=cfg.layer_num, head_num=cfg.head_num, use_res=cfg.use_res,
                mlp_activation=cfg.mlp_activation, logits_activation=cfg.logits_activation)
    ref = tr.AutoIntCPU(model.table.weight.cpu().numpy(), model.embedding.row_base.cpu().numpy(),
                        model.embedding.bucket.cpu().numpy(), il, deep, logits, ocfg,
                        dtype=torch.float32)
    B = batches_cpu[0][0].shape[0]
    per_run = max(seconds / 6.0, 0.5)

    def runs(n_threads):
        torch.set_num_threads(n_threads)
        ref.step(*batches_cpu[0])  # warm-up
        rates, steps_total = [], 0
        for _ in range(3):
            t0 = time.perf_counter()
            n = 0
            while n < 2 or time.perf_counter() - t0 < per_run:
                ref.step(*batches_cpu[n % len(batches_cpu)])
                n += 1
            rates.append(B * n / (time.perf_counter() - t0))
            steps_total += n
        return float(np.median(rates)), steps_total

    multi, n_multi = runs(threads)
    single, n_single = runs(1)
    torch.set_num_threads(threads)
    return {"value": round(multi, 1), "unit": "samples/sec", "cores": threads, "kind": "port",
            "single_thread": {"value": round(single, 1), "cores": 1},
            "sample": f"AutoInt train steps at batch {B} (26x16, IL x3, MLP, dense + sparse Adam) of "
                      f"the TF-semantics fp32 torch-CPU restatement (oracle/torch_ref.py): median of 3 "
                      f"runs of >= {per_run:.1f} s each, {n_multi} steps on {threads} threads and "
                      f"{n_single} steps on 1 thread"}


def config1_leg(seconds, dev):
    """configs[0]: InteractingLayer.py's forward on the host CPU --
    x ~ U(-0.05, 0.05) [256, 26, 16] (seed 0), glorot-uniform weights (seed 1), no dropout -- with
    the constructor defaults (layer_num 1, unit_num 128, head_num 1, use_res) and the AutoInt
    setting (3, 16, 2, use_res).  "For config 1 the CPU path is the measurement": the fp32
    TF-op-order restatement (oracle/torch_ref.py::interacting_layer, kind "port") timed on the
    box's host cores (all threads, median of 3 bounded runs) and on 1 thread; beside it, the same
    forward through rs_il_fwd on the GPU (HIP events, for reference)."""
    from oracle import torch_ref as tr
    from recommendsystem_amd._lib import call, ptr, stream_handle
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    B, F, E = 256, 26, 16
    x = np.random.default_rng(0).uniform(-0.05, 0.05, size=(B, F, E)).astype(np.float32)
    out = {"workload": "configs[0]: InteractingLayer forward, 26 fields x emb 16, batch 256 "
                       "(x ~ U(-0.05, 0.05) seed 0, glorot-uniform weights seed 1, no dropout)",
           "unit": "samples/sec", "kind": "port", "cores": threads}
    per = max(seconds / 12.0, 0.25)
    for name, (L, U, H) in (("ctor_defaults", (1, 128, 1)), ("autoint", (3, 16, 2))):
        lim = (6.0 / (E + U)) ** 0.5
        w = np.random.default_rng(1).uniform(-lim, lim, size=(E, 4 * U)).astype(np.float32)
        args = (torch.from_numpy(w), torch.zeros(4 * U), torch.ones(U), torch.zeros(U), L, H, True)
        xt = torch.from_numpy(x)

        def rate(n_threads):
            torch.set_num_threads(n_threads)
            with torch.no_grad():
                tr.interacting_layer(xt, *args)
                rs = []
                for _ in range(3):
                    t0, k = time.perf_counter(), 0
                    while k < 2 or time.perf_counter() - t0 < per:
                        tr.interacting_layer(xt, *args)
                        k += 1
                    rs.append(B * k / (time.perf_counter() - t0))
            return float(np.median(rs))

        multi, single = rate(threads), rate(1)
        torch.set_num_threads(threads)
        # the same forward on the GPU (fp32, one launch)
        xd = torch.from_numpy(x).to(dev)
        wd, bd = torch.from_numpy(w).to(dev), torch.zeros(4 * U, device=dev)
        gd, bed = torch.ones(U, device=dev), torch.zeros(U, device=dev)
        y = torch.empty(B, F * U, device=dev)
        xs = torch.empty(max(L - 1, 1), B, F, U, device=dev)
        t = time_kernel(lambda: call("rs_il_fwd", stream_handle(), ptr(xd), B, F, E, U, H, L,
                                     ptr(wd), ptr(bd), ptr(gd), ptr(bed), 1e-14, 1, 0.0, 0,
                                     ptr(y), F * U, ptr(xs) if L > 1 else None), 50)
        out[name] = {"layer": f"IL(layer_num={L}, unit_num={U}, head_num={H}, use_res=True)",
                     "cpu_value": round(multi, 1), "cpu_single_thread": round(single, 1),
                     "gpu_value": round(B / t, 1), "gpu_us_per_forward": round(t * 1e6, 2)}
    return out


WORKLOADS = {
    # name: (config index, per-GPU batch, description)
    "multi_head": (2, 4096, "configs[2]: rank/multi_head AUTOINT train (200 fields x dim 8 multi-hot, "
                            "IL(1,8,2,dropout .2) + 7 experts/gates + 7 towers), global 8192 / DP2"),
    "din": (3, 1024, "configs[3]: din.py DIN pool train (seq 100, 1M x 16 table, query ++ pool -> "
                     "Dense(1)), global 4096 / DP4"),
    "staytime": (4, 2048, "configs[4]: staytime mtl_net + rough_rank DSSM joint train, 10M x 32 "
                          "hashed table, global 16384 / DP8"),
}


# algorithmic work of the configs-3-5 dominant kernels
IL200_FWD_FLOPS_PER_SAMPLE = 1_382_400   # F=200, E=U=8, H=2: proj 102 400 + QK^T 640 000 + PV 640 000
PUSH_BYTES_PER_ID = 4 + 64 + 128 + 4     # row index, dout row, grad row read + write, flag
PUSH_BYTES_PER_SLOT = 4                  # every (sample, position) slot's row index is read


def workload_roofline(args, model, pool, B, dev):
    """Dominant kernel of configs 3-5 (rocprof, profiles/r02/prof_*), timed live with HIP events on
    torch's current stream (the stream it is launched on) with the workload's own shapes:
      multi_head  rs_il::large::bwd_kernel  -- InteractingLayer backward, F = 200 (48 % of the step)
      din         sparse_grad_accum_kernel  -- the history push, B x 100 slots (28 %)
      staytime    gemm_kernel (rs_dense_*)  -- the GEMM engine, on the widest expert layer
                  [B, 1712] x [1712, 256] (the GEMMs are ~40 % of the step, spread over shapes)"""
    from recommendsystem_amd import _lib
    from recommendsystem_amd._lib import call, ptr, stream_handle
    lib = _lib.load()
    s = stream_handle()
    g = torch.Generator(device=dev).manual_seed(7)
    if args.workload == "multi_head":
        F, E, U, H = model.cfg.num_fields, model.cfg.embed_dim, model.cfg.embed_dim, 2
        il = model.interact
        x = torch.rand(B, F, E, device=dev, generator=g) - 0.5
        dy = torch.randn(B, F * U, device=dev, generator=g)
        dx = torch.empty_like(x)
        wsn = int(lib.rs_il_bwd_workspace_floats(B, E, U))
        ws = torch.empty(wsn, device=dev)
        # the layer's path: the forward saves O / softmax stats / keep bits, the backward reads them
        ns = int(lib.rs_il_attn_save_floats(B, F, U, H, 1))
        asave = torch.empty(ns, device=dev)
        y = torch.empty(B, F * U, device=dev)
        call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, 1, ptr(il.kernel), ptr(il.bias),
             ptr(il.gamma), ptr(il.beta), il.epsilon, 1, il.dropout_rate, 11, ptr(y), F * U, None,
             ptr(asave), ns)
        t = time_kernel(lambda: call(
            "rs_il_bwd_saved", s, ptr(x), None, ptr(dy), F * U, B, F, E, U, H, 1, ptr(il.kernel),
            ptr(il.bias), ptr(il.gamma), ptr(il.beta), il.epsilon, 1, il.dropout_rate, 11, ptr(dx),
            0, None, 0, ptr(ws), wsn, ptr(asave), ns), args.kernel_reps)
        fl = 2 * IL200_FWD_FLOPS_PER_SAMPLE * B
        return {"bound": "mfma", "kernel": "rs_il::large::bwd_kernel<LC<8,8,2>> (IL backward over the "
                "forward's attention save, F=200, dropout .2)", "achieved": round(fl / t / 1e12, 3), "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(fl / t / 1e12 / FP32_PEAK_TFLOPS, 4), "traffic": None,
                "launch_us": round(t * 1e6, 2), "flops_per_launch": fl}
    if args.workload == "din":
        qids, hids, hoffs, _ = pool[0]
        T, vocab = model.T, model.table.rows
        o = hoffs.long()
        lens = torch.clamp(o[1:] - o[:-1], max=T)
        pos = torch.arange(T, device=dev)[None, :]
        idx = torch.clamp(o[:-1, None] + pos, max=hids.numel() - 1)
        rows = torch.where(pos < lens[:, None], hids[idx] % vocab,
                           torch.full_like(idx, -1)).to(torch.int32).reshape(-1).contiguous()
        dout = torch.randn(B, T, model.table.dim, device=dev, generator=g)
        tab = model.table
        t = time_kernel(lambda: tab.accumulate(rows, None, B, T, dout, T * tab.dim, tab.dim, 0),
                        args.kernel_reps)
        nvalid = int(lens.sum())
        by = PUSH_BYTES_PER_SLOT * B * T + PUSH_BYTES_PER_ID * nvalid
        return {"bound": "hbm", "kernel": "sparse_grad_accum_kernel (history push, B x 100 slots, "
                f"{nvalid} ids)", "achieved": round(by / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(by / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                "launch_us": round(t * 1e6, 2), "bytes_per_launch": by}
    out = staytime_gather_roofline(model, pool, B, dev, args.kernel_reps)
    K, N = 1712, 256
    X = torch.randn(B, K, device=dev, generator=g)
    Wt = torch.randn(K, N, device=dev, generator=g) * 0.02
    bt = torch.zeros(N, device=dev)
    Y = torch.empty(B, N, device=dev)
    t = time_kernel(lambda: call("rs_dense_fwd", s, ptr(X), B, K, K, ptr(Wt), ptr(bt), N, 1, ptr(Y), N),
                    args.kernel_reps)
    fl = 2 * B * K * N
    out["gemm_roofline"] = {
        "bound": "mfma", "kernel": f"gemm_kernel via rs_dense_fwd [{B}x{K}]x[{K}x{N}] relu (staytime "
        "expert layer 1)", "achieved": round(fl / t / 1e12, 3), "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s", "frac": round(fl / t / 1e12 / FP32_PEAK_TFLOPS, 4), "traffic": None,
        "launch_us": round(t * 1e6, 2), "flops_per_launch": fl}
    return out


# config-5 gather side, algorithmic bytes (dim-32 fp32 rows = 128 B)
LOOKUP_BYTES_PER_ID = 8 + 4 + 2 * 128      # id, hashed row out, row read, output row write
SEQ_BYTES_PER_SLOT = 128 + 1 + 4           # output row (zero past the length), mask, row index
SEQ_BYTES_PER_ID = 8 + 128                 # id, row read
PUSH_BYTES_PER_ID32 = 4 + 128              # row index, dout row (per id)
ROW_BYTES_PER_UNIQUE = 2 * 128 + 4 + 6 * 128 + 4   # grad row RMW + flag (push), AdaGrad: w, g2sum,
#                                            grad read + write (zeroed), touched-list entry


def staytime_gather_roofline(model, pool, B, dev, reps):
    """Config 5's HBM-bound gather side (BASELINE.json configs[4] "HBM-bound gather roofline"),
    timed live with HIP events on torch's current stream: the step's five lookups (91 single-hot
    fields, 3 x 50-long sequences, 52 DSSM fields; rs_embedding_lookup_fwd /
    rs_sequence_lookup_fwd), their five pushes into the gradient table (list mode: election +
    claim kernels, rs_sparse_grad_accumulate_ws) and the sparse AdaGrad over the touched rows --
    exactly the table-side launches of one training step, on pool batch 0.  Algorithmic bytes:
    per id its id, row read, output write and dout read; per unique row the gradient row
    read-modify-write, flag and the optimizer's row traffic."""
    from recommendsystem_amd._lib import call, ptr, stream_handle
    from recommendsystem_amd.embedding import COMBINERS
    t = model.table
    st_ids, seq_ids, seq_offs, rr_ids = pool[0][0], pool[0][1], pool[0][2], pool[0][3]
    d = t.dim
    g = torch.Generator(device=dev).manual_seed(8)
    jobs = []  # (kind, layer, ids, offsets, F or T, out, rows, dout)
    for lay, ids in ((model.fields, st_ids), (model.rr_fields, rr_ids)):
        F = lay.num_fields
        jobs.append(("fields", lay, ids, None, F, torch.empty(B, F, d, device=dev),
                     torch.empty(B * F, device=dev, dtype=torch.int32),
                     torch.randn(B, F, d, device=dev, generator=g)))
    for lay, ids, offs in zip(model.seqs, seq_ids, seq_offs):
        T = lay.seq_max_len
        jobs.append(("seq", lay, ids, offs, T, torch.empty(B, T, d, device=dev),
                     torch.empty(B * T, device=dev, dtype=torch.int32),
                     torch.randn(B, T, d, device=dev, generator=g)))
    mask = torch.empty(B, max(j[4] for j in jobs), device=dev, dtype=torch.uint8)
    lens = torch.empty(B, device=dev, dtype=torch.int32)

    def gather_side():
        s = stream_handle()
        for kind, lay, ids, offs, F, out, rows, _ in jobs:
            if kind == "fields":
                call("rs_embedding_lookup_fwd", s, ptr(ids), None, B, F, ptr(lay.row_base),
                     ptr(lay.bucket), lay.hash_mode, lay.combiner, ptr(t.weight), t.rows, d,
                     ptr(out), F * d, d, ptr(rows))
            else:
                call("rs_sequence_lookup_fwd", s, ptr(ids), ptr(offs), B, F, lay.row_base,
                     lay.bucket, lay.hash_mode, ptr(t.weight), d, ptr(out), F * d, d, ptr(mask),
                     F, ptr(lens), ptr(rows))
        for kind, lay, ids, offs, F, out, rows, dout in reversed(jobs):
            t.accumulate(rows, None, B, F, dout, F * d, d,
                         lay.combiner if kind == "fields" else COMBINERS["sum"])
        t.step(grad_scale=1.0)

    saved = [x.clone() for x in (t.weight, t.g2sum)]
    sec = time_kernel(gather_side, reps)
    t.weight.copy_(saved[0])
    t.g2sum.copy_(saved[1])
    n_ids = n_slots_seq = n_ids_seq = 0
    all_rows = []
    for kind, lay, ids, offs, F, out, rows, _ in jobs:
        valid = rows[rows >= 0]
        all_rows.append(valid)
        if kind == "fields":
            n_ids += B * F
        else:
            n_slots_seq += B * F
            n_ids_seq += int(valid.numel())
    uniq = int(torch.unique(torch.cat(all_rows)).numel())
    by = (LOOKUP_BYTES_PER_ID * n_ids + SEQ_BYTES_PER_SLOT * n_slots_seq +
          SEQ_BYTES_PER_ID * n_ids_seq + PUSH_BYTES_PER_ID32 * (n_ids + n_ids_seq) +
          ROW_BYTES_PER_UNIQUE * uniq)
    return {"bound": "hbm", "kernel": "gather side of one step: 5 lookups (91 fields, 3 x 50 "
            "sequences, 52 DSSM fields) + 5 pushes (election + claim) + sparse AdaGrad, "
            f"{n_ids + n_ids_seq} ids, {uniq} unique rows of the 10M x 32 table",
            "achieved": round(by / sec / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(by / sec / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
            "launch_us": round(sec * 1e6, 2), "bytes_per_launch": by}


def workload_cpu_baseline(args, model, rng, B):
    """configs 3-4: the fp32 torch-CPU TF-semantics train step (oracle/torch_ref.py
    MultiHeadCPU / DINPoolCPU, kind "port") on a bounded sample of the workload (smaller batch
    for config 3: its IL materialises [2B, 200, 200] scores), median of 3 runs, all threads and
    1 thread.  Config 5: oracle/model_oracles.py StaytimeRoughRankCPU (host copy of the 10M x 32
    table, sparse AdaGrad) on device-generated staytime batches copied to the host."""
    from oracle import torch_ref as tr
    from recommendsystem_amd import workloads as W
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    if args.workload == "multi_head":
        Bc = 256
        ref = tr.MultiHeadCPU(model)
        batches = [ref.prepare(*(t.cpu() for t in W.multi_head_batch(rng, Bc, model.cfg, "cpu")))
                   for _ in range(2)]
    elif args.workload == "staytime":
        from oracle.model_oracles import StaytimeRoughRankCPU
        Bc = 256
        ref = StaytimeRoughRankCPU(model)
        batches = [ref.prepare(W.staytime_batch(rng, Bc, model, model.table.weight.device))
                   for _ in range(2)]
    else:
        Bc = B
        ref = tr.DINPoolCPU(model)
        batches = [ref.prepare(*(t.cpu() for t in W.din_batch(rng, Bc, model.T, model.table.rows, "cpu")))
                   for _ in range(2)]
    per_run = max(args.cpu_baseline_seconds / 6.0, 0.5)

    def runs(n):
        torch.set_num_threads(n)
        ref.step(*batches[0])
        rates, tot = [], 0
        for _ in range(3):
            t0, k = time.perf_counter(), 0
            while k < 2 or time.perf_counter() - t0 < per_run:
                ref.step(*batches[k % len(batches)])
                k += 1
            rates.append(Bc * k / (time.perf_counter() - t0))
            tot += k
        return float(np.median(rates)), tot

    multi, nm = runs(threads)
    single, ns = runs(1)
    torch.set_num_threads(threads)
    return {"value": round(multi, 1), "unit": "samples/sec", "cores": threads, "kind": "port",
            "single_thread": {"value": round(single, 1), "cores": 1},
            "sample": f"{args.workload} train steps at batch {Bc} of the TF-semantics fp32 torch-CPU "
                      f"restatement ({type(ref).__module__}.{type(ref).__name__}): median of 3 runs of "
                      f">= {per_run:.1f} s, {nm} steps on {threads} threads, {ns} on 1 thread"}


def run_workload(args, world, rank, dev, pg):
    """Configs 3-5 through the generic Trainer (eager autograd composition of the kernels)."""
    from recommendsystem_amd.models import MultiHeadConfig, MultiHeadRanker
    from recommendsystem_amd.trainer import Trainer
    from recommendsystem_amd import workloads as W
    ci, B, desc = WORKLOADS[args.workload]
    if args.batch != 4096:
        B = args.batch
    rng = np.random.default_rng(10 + 1000 * rank)
    if args.workload == "multi_head":
        cfg = MultiHeadConfig()
        model = MultiHeadRanker(cfg, device=dev, seed=0)
        trainer = Trainer(model, cfg.lr_dense, model.tables(), process_group=pg)
        pool = [W.multi_head_batch(rng, B, cfg, dev) for _ in range(args.pool)]
    elif args.workload == "din":
        model = W.DINPool(device=dev, seed=0)
        trainer = Trainer(model, 5e-5, [model.table], process_group=pg)
        pool = [W.din_batch(rng, B, 100, 1_000_000, dev) for _ in range(args.pool)]
    else:
        shard = pg if (world > 1 and args.shard_table) else None  # N2 owner-sharded 10M table
        model = W.StaytimeRoughRank(device=dev, seed=0, shard_group=shard)
        trainer = Trainer(model, 5e-4, [model.table], process_group=pg,
                          lr_groups=[(model.dssm, model.rr_cfg.lr_dense)])
        pool = [W.staytime_batch(rng, B, model, dev) for _ in range(args.pool)]
    sharded = getattr(model.table, "sharded", False)
    # owner-sharded tables are captured with fixed routing, their all-to-alls inside the graph:
    # RCCL only (gloo collectives are host calls)
    graphed = not args.eager and (not sharded or torch.distributed.get_backend(pg) == "nccl")
    dp_caps = None
    if graphed:  # one HIP graph per pool batch (forward + autograd backward + optimizers)
        if world > 1:
            # the sync-free captured DP step: fixed-capacity all-gathers sized from the pool's
            # own touched-row counts (max over ranks, 25 % headroom; overflow is detected);
            # owner-sharded tables get their fixed routing capacity (owner_cap) the same way
            dp_caps = trainer.measure_dp_caps(pool)
        trainer.capture_pool(pool, warmup=1, dp_caps=dp_caps)
        step = trainer.step_pool
    else:
        def step(i):
            return trainer.step(*pool[i % len(pool)])
    for i in range(args.warmup):
        step(i)
    if args.trace_markers:
        torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if args.trace_markers:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    if dp_caps is not None:
        trainer.check_dp_overflow()  # (outside the timed region)
    samples = B * args.steps * world
    roofline = workload_roofline(args, model, pool, B, dev)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_seconds > 0:
        cpu = workload_cpu_baseline(args, model, rng, B)
    out = {"metric": f"samples/sec {args.workload} train ({desc})", "value": round(samples / dt, 1),
           "unit": "samples/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (SURVEY §8d config generators; random-init weights)",
           "config": {"workload": desc, "global_batch": B * world, "per_gpu_batch": B,
                      "parallelism": f"dp{world}",
                      "table": ("owner-sharded" + (f" (fixed routing, owner_cap {model.table.owner_cap})"
                                                   if getattr(model.table, "owner_cap", None) else "")
                                if sharded else "replicated"),
                      "execution": ("one HIP graph per pool batch" + (
                          f" + sync-free fixed-capacity exchange (dp_caps {dp_caps})" if dp_caps
                          else "")) if graphed else "eager autograd"},
           "roofline": roofline, "cpu_baseline": cpu, "final_loss": round(float(loss.detach()), 6)}
    if rank == 0:
        print(json.dumps(out), flush=True)


def per_gpu_batch(args, world, scaling):
    if scaling == "weak":
        return args.batch
    if args.global_batch % world:
        raise SystemExit(f"--global-batch {args.global_batch} does not split over {world} ranks")
    return args.global_batch // world


def bench_autoint(args, world, rank, dev, pg, compute_dtype, scaling="strong"):
    """Config 2 in one compute mode ("f32": the reference's dtype; "bf16": config 2's stated
    bf16 mode, rs_set_math_mode) and one batch series (strong: global batch split over the
    ranks; weak: per-GPU batch fixed).  Returns (result dict, model, cfg, CPU batch pool)."""
    from recommendsystem_amd import _lib
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    # config 2: 26 x 16, vocab 100k/field, IL(3, 16, 2), mlp [32,16], [1]
    cfg = AutoIntConfig(compute_dtype=compute_dtype)
    B, F = per_gpu_batch(args, world, scaling), cfg.num_fields
    model = AutoInt(cfg, device=dev, seed=0, max_batch=B, world_size=world)
    trainer = AutoIntTrainer(model, B, process_group=pg)

    rng = np.random.default_rng(2 + 1000 * rank)
    lab_rng = np.random.default_rng(3 + 1000 * rank)
    pool_cpu = [(torch.from_numpy(zipf_ids(rng, B, F, cfg.vocab_per_field)),
                 torch.from_numpy((lab_rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)))
                for _ in range(args.pool)]
    pool = [(i.to(dev), l.to(dev)) for i, l in pool_cpu]

    # one HIP graph per resident batch (the step reads its batch in place: no input copy)
    trace("capturing")
    trainer.capture_pool(pool, warmup=max(1, min(args.warmup, 3)))
    trace("captured")
    for i in range(args.warmup):
        trainer.step_pool(i)
    if args.trace_markers:
        torch.cuda._sleep(1000)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    barrier()
    torch.cuda.synchronize()
    step_ev = None
    if os.environ.get("RS_BENCH_STEP_TRACE"):  # diagnostic: device time of every timed step
        step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        if step_ev is not None:
            step_ev[i].record()
        trainer.step_pool(i)
    if step_ev is not None:
        step_ev[args.steps].record()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if step_ev is not None:
        us = [round(step_ev[k].elapsed_time(step_ev[k + 1]) * 1e3, 1) for k in range(args.steps)]
        print(json.dumps({"step_trace_us": us, "graph": [k % len(trainer.pool_graphs)
                                                        for k in range(args.steps)]}),
              file=sys.stderr, flush=True)
    if args.trace_markers:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    loss = float(trainer.loss.item())
    trace(f"timed loop done, loss {loss}")

    # ---- roofline of the dominant kernel (IL backward), HIP events on its stream ----
    from recommendsystem_amd._lib import call, ptr, stream_handle
    il = model.interact
    E, U, H, L = cfg.embed_dim, cfg.unit_num, cfg.head_num, cfg.layer_num

    xt = trainer.head["xt"] if trainer.head is not None else None
    hd = trainer.head

    def il_bwd_once():
        # the exact launch the step makes: backward + fused sparse push into the gradient table
        # (scan-mode marks) + the head's deferred dW1 = x0^T dz1 rows (rs_il_bwd_push_saved_xt);
        # it adds into table.grad, which only matters after the timed region (the saved pair: it
        # reads the forward's attention save left by the last step)
        t = model.table
        xa = (ptr(trainer.x0), F * E, ptr(xt["dz1"]), hd["N1"], hd["K0"], hd["N1"],
              ptr(xt["slab"])) if xt else ()
        call("rs_il_bwd_push_saved_xt" if xt else "rs_il_bwd_push_saved", stream_handle(),
             ptr(trainer.x0), ptr(trainer.xsave),
             trainer.dcat.data_ptr() + 4 * trainer.D, trainer.CW, B, F, E, U, H, L,
             ptr(il.kernel), ptr(il.bias), ptr(il.gamma), ptr(il.beta), il.epsilon, 1, 0.0, 0,
             ptr(trainer.dx0), ptr(trainer.rows), ptr(t.grad), ptr(t.flag), None, 0,
             ptr(trainer.il_ws), trainer.il_ws_n, ptr(trainer.asave), trainer.asave_n, *xa)

    def il_fwd_once():
        call("rs_il_fwd_saved", stream_handle(), ptr(trainer.x0), B, F, E, U, H, L,
             ptr(il.kernel), ptr(il.bias), ptr(il.gamma), ptr(il.beta), il.epsilon, 1, 0.0, 0,
             trainer.cat.data_ptr() + 4 * trainer.D, trainer.CW, ptr(trainer.xsave),
             ptr(trainer.asave), trainer.asave_n)

    trace("kernel timing")
    peak = BF16_PEAK_TFLOPS if compute_dtype == "bf16" else FP32_PEAK_TFLOPS
    with _lib.math_mode(compute_dtype):
        t_bwd = time_kernel(il_bwd_once, args.kernel_reps)
        t_fwd = time_kernel(il_fwd_once, args.kernel_reps)
    # backward = 2 x the forward's matmul FLOPs, plus the deferred dW1 (2 K0 N1 per sample) the
    # launch carries when the head defers it
    bwd_flops = (2 * IL_FWD_FLOPS_PER_SAMPLE + (2 * hd["K0"] * hd["N1"] if xt else 0)) * B
    achieved = bwd_flops / t_bwd / 1e12
    # HBM traffic is not measurable inside this run (PMC needs its own rocprofv3 --pmc passes):
    # the value is the committed PMC measurement of the same launch (tools/il_traffic.py over
    # this bench's own step), labelled as such
    traffic, traffic_src = None, None
    kname = "rs_il::bwd4_kernel" if B > 1536 else "rs_il::wbwd_kernel"
    # the newest round's committed measurement (profiles/rNN/il_bwd_traffic.json)
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "il_bwd_traffic.json")) +
                   glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "*", "il_bwd_traffic.json")))
    tf_path = cands[-1] if cands else ""
    if compute_dtype == "f32" and tf_path and os.path.exists(tf_path):
        with open(tf_path) as f:
            tj = json.load(f)
        if tj.get("per_gpu_batch") == B and tj.get("kernel", "").split("<")[0] in kname and \
                tj.get("launch") == ("rs_il_bwd_push_saved_xt" if xt else "rs_il_bwd_push_saved"):
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = (f"committed rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, separate passes) "
                           f"in {os.path.relpath(tf_path, ROOT)} ({tj.get('source', '')}), not measured "
                           f"in this run")

    samples = B * args.steps * world
    # BASELINE.md §3 step roofline: max(sum bytes / HBM BW, sum flops / peak), per GPU
    rb = model.embedding.row_base.cpu().numpy()[None, :]
    uniq = int(np.mean([np.unique(rb + np.remainder(i.numpy(), cfg.vocab_per_field)).size
                        for i, _ in pool_cpu]))
    step_bytes = B * STEP_BYTES_PER_SAMPLE + ADAM_BYTES_PER_ROW * uniq
    step_flops = B * TRAIN_FLOPS_PER_SAMPLE
    t_bytes = step_bytes / (HBM_PEAK_GBS * 1e9)
    t_bf16 = step_flops / (BF16_PEAK_TFLOPS * 1e12)
    t_fp32 = step_flops / (FP32_PEAK_TFLOPS * 1e12)
    step_s = dt / args.steps
    out = {
        "metric": "samples/sec AutoInt CTR train, 26 fields×16-dim emb, batch 4096, 1/2/4/8 GPU",
        "value": round(samples / dt, 1),
        "unit": "samples/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": compute_dtype,
        "data": "synthetic (Zipf(1.2) ids over 26x100k vocab, Bernoulli(0.25) labels; random-init weights)",
        "config": {"workload": "configs[1]: AutoInt full train (embedding + 3xInteractingLayer + MLP), "
                               f"26 fields x emb 16, global batch {B * world} ({scaling} scaling)",
                   "global_batch": B * world, "per_gpu_batch": B, "fields": F, "emb_dim": E,
                   "layer_num": L,
                   "head_num": H, "parallelism": f"dp{world}",
                   "execution": ("one HIP graph per pool batch" if trainer._one_graph else
                                 "forward/backward graph + eager all-gather + optimizer graph")
                                + (" (RCCL all-gather captured in the step graph)"
                                   if getattr(trainer, "dp_one_graph", False) else "")},
        "roofline": {"bound": "mfma", "kernel": kname
                     + " (InteractingLayer backward over the forward's attention save + fused sparse "
                       "push" + (" + the head's deferred dW1, counted)" if xt else ")"),
                     "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "launch_us": round(t_bwd * 1e6, 2),
                     "flops_per_launch": bwd_flops},
        "il_fwd_us": round(t_fwd * 1e6, 2),
        "step_roofline": {
            "bytes_per_step": step_bytes, "flops_per_step": step_flops, "unique_rows": uniq,
            "t_bytes_us": round(t_bytes * 1e6, 3), "t_flops_bf16_us": round(t_bf16 * 1e6, 3),
            "t_flops_fp32_us": round(t_fp32 * 1e6, 3),
            "frac_bf16_basis": round(max(t_bytes, t_bf16) / step_s, 4),
            "frac_fp32_basis": round(max(t_bytes, t_fp32) / step_s, 4),
            "note": "BASELINE.md §3: fraction = roofline time / measured step time; the bf16 "
                    "basis is the config's stated compute dtype"},
        "step_tflops": round(TRAIN_FLOPS_PER_SAMPLE * samples / dt / 1e12, 3),
        "final_loss": round(loss, 6),
        "cpu_baseline": None,
    }
    return out, model, cfg, pool_cpu


def launch_ranks(args) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start N fresh rank processes through
    torch.distributed.run and return its exit code.  The parent never touches the GPU (no HIP
    call before the children exist), so every rank initialises its own device cleanly."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per "
                         "GPU (torch.distributed.run --nproc-per-node N) or let bench.py do it")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())  # (rehearsal: several ranks per GPU)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
        pg = dist.group.WORLD
        if rank == 0:
            print(f"[bench] {dist.get_backend(pg)} world size {dist.get_world_size(pg)}",
                  file=sys.stderr, flush=True)
        assert dist.get_world_size(pg) == args.gpus

    from recommendsystem_amd import _lib
    _lib.load()
    if args.workload != "autoint":
        run_workload(args, world, rank, dev, pg)
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    out, model, cfg, pool_cpu = bench_autoint(args, world, rank, dev, pg, args.dtype, args.scaling)
    other = "weak" if args.scaling == "strong" else "strong"
    if world > 1 and not args.no_other and per_gpu_batch(args, world, other) != out["config"]["per_gpu_batch"]:
        # the other batch series in the same run (own timed region, same contract)
        o3, *_ = bench_autoint(args, world, rank, dev, pg, args.dtype, other)
        out[other] = {k: o3[k] for k in ("value", "ms_per_step", "scaling", "roofline", "il_fwd_us",
                                         "final_loss")}
        out[other]["global_batch"] = o3["config"]["global_batch"]
        out[other]["per_gpu_batch"] = o3["config"]["per_gpu_batch"]
    if args.dtype == "f32" and not args.no_bf16:
        # config 2's bf16 mode beside the fp32 line (same contract, own timed region)
        o2, *_ = bench_autoint(args, world, rank, dev, pg, "bf16", args.scaling)
        out["bf16"] = {k: o2[k] for k in ("value", "ms_per_step", "dtype", "roofline",
                                           "il_fwd_us", "step_roofline", "final_loss")}
        out["bf16"]["note"] = ("IL projections/dW/dx and head layer-1/2 GEMMs on bf16 MFMA, fp32 "
                               "accumulation and master weights; accuracy in tests/test_gpu_bf16.py")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(cfg, model, pool_cpu, args.cpu_baseline_seconds)
        out["config1"] = config1_leg(args.cpu_baseline_seconds, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
