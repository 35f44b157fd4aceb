"""Synthetic workloads of SURVEY §8d configs 3-5 (the headline config 2 lives in bench.py):
model builders over one HBM-resident table and seeded batch generators of the stated shapes.

    config 3  rank/multi_head: 200 fields x vocab 265k, dim 8, multi-hot U{1..3} (mean),
              7 Bernoulli(0.1) labels, global batch 8192 (DP 2 -> 4096 per GPU)
    config 4  din.py pool: 1M-item vocab x 16, Zipf(1.1) query + history ids, lengths U{1..100}
              with max 100, global batch 4096 (DP 4 -> 1024 per GPU).  din.py is a bare layer;
              the harness around it (pooled ++ query -> Dense(1, sigmoid) -> cross_entropy) is
              this framework's, stated in DESIGN.md.
    config 5  staytime + rough_rank joint: one 10M x 32 table (splitmix64(id) % 10M, AdaGrad
              lr .005 g2sum .1 -- staytime/VideoDnn.py:233), 91 staytime fields + 3 x 50
              sequences + 33 user / 19 item rough_rank fields (cols 0:16), 400-bin soft labels
              (staytime/parse.py:40-62), global batch 16384 (DP 8 -> 2048 per GPU).
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn

from .din import DIN
from .embedding import (EmbeddingFeatures, SequenceEmbedding, ShardedSparseTable, SparseAdaGrad,
                        SparseAdam, SparseTable)
from .layers import Dense
from .models import (DSSM, STAYTIME_BINS, DSSMConfig, MultiHeadConfig, MultiHeadRanker,
                     StaytimeConfig, StaytimeMTL)
from .parse import staytime_labels as device_staytime_labels
from .towers import cross_entropy_sum, fused_loss


def zipf_ids(rng, shape, vocab, a):
    z = rng.zipf(a, size=shape) - 1
    return np.minimum(z, vocab - 1).astype(np.int64)


# ------------------------------------------------------------------------------------------
# config 3
# ------------------------------------------------------------------------------------------
def multi_head_batch(rng, B, cfg: MultiHeadConfig, device):
    F = cfg.num_fields
    lens = rng.integers(1, 4, size=B * F)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ids = zipf_ids(rng, (int(offsets[-1]),), cfg.vocab_per_field, 1.2)
    labels = (rng.uniform(size=(B, cfg.num_label)) < 0.1).astype(np.float32)
    return (torch.from_numpy(ids).to(device), torch.from_numpy(offsets).to(device),
            torch.from_numpy(labels).to(device))


# ------------------------------------------------------------------------------------------
# config 4
# ------------------------------------------------------------------------------------------
class DINPool(nn.Module):
    """Config-4 harness around din.py's DIN: item table 1M x 16, query item lookup, history
    sequence lookup (T = 100, lengths), DIN(query, hist, hist, lengths), then
    Dense(1, sigmoid) on [pooled, query] and cross_entropy (rank/ctr/base_model.py:7-12)."""

    def __init__(self, vocab=1_000_000, dim=16, T=100, device=None, seed=0, max_touched=None):
        super().__init__()
        dev = torch.device(device or "cuda")
        self.T = T
        self.table = SparseTable(vocab, dim, SparseAdam(5e-5), device=dev, seed=seed,
                                 max_touched=max_touched)
        # 1 M rows, ~20 K touched per step at B = 1024: a 4 MB flag sweep is cheaper than the
        # pushes' row claims (Trainer applies it at world 1)
        self.table.prefer_scan = True
        self.query = EmbeddingFeatures(self.table, [vocab], combiner="sum")
        self.hist = SequenceEmbedding(self.table, vocab, T)
        self.din = DIN(seed=seed + 1, device=dev)
        self.din.build((1, T, dim), device=dev)
        self.out = Dense(1, "sigmoid", seed=seed + 2, device=dev)
        self.out.build((1, 2 * dim), device=dev)

    def regularizers(self):
        return []

    def forward(self, qids, hids, hoffs):
        q = self.query(qids.reshape(-1, 1)).reshape(qids.shape[0], -1)          # [B, 16]
        keys, _, lengths = self.hist(hids, hoffs, return_lengths=True)          # [B, T, 16]
        # din.py:18-47 pooling, then the head's concat [pooled, q]: the DIN kernel writes into the
        # concat and sums the query's two gradients in its backward (forward_concat)
        return self.out(self.din.forward_concat(q, keys, keys, lengths))

    def loss(self, qids, hids, hoffs, labels):
        return cross_entropy_sum(labels, self.forward(qids, hids, hoffs))


def din_batch(rng, B, T, vocab, device):
    q = zipf_ids(rng, (B,), vocab, 1.1)
    lens = rng.integers(1, T + 1, size=B)
    lens[0] = T
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    h = zipf_ids(rng, (int(offs[-1]),), vocab, 1.1)
    y = (rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)
    t = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
    return t(q), t(h), t(offs), t(y)


# ------------------------------------------------------------------------------------------
# config 5
# ------------------------------------------------------------------------------------------
class StaytimeRoughRank(nn.Module):
    """Config-5 joint model: StaytimeMTL + DSSM over ONE hashed table (rows 32 wide; rough_rank
    reads columns 0:16)."""

    def __init__(self, rows=10_000_000, device=None, seed=0, st_cfg=None, rr_cfg=None,
                 max_touched=None, shard_group=None):
        """shard_group: a process group -> the table is owner-sharded over its ranks
        (ShardedSparseTable, N2); None -> one replicated table."""
        super().__init__()
        dev = torch.device(device or "cuda")
        self.st_cfg = st_cfg or StaytimeConfig()
        self.rr_cfg = rr_cfg or DSSMConfig()
        if shard_group is not None:
            self.table = ShardedSparseTable(rows, self.st_cfg.emb_dim, SparseAdaGrad(), device=dev,
                                            seed=seed, max_touched=max_touched,
                                            process_group=shard_group)
        else:
            self.table = SparseTable(rows, self.st_cfg.emb_dim, SparseAdaGrad(), device=dev,
                                     seed=seed, max_touched=max_touched)
            # single GPU: the pushes mark rows with plain stores and the AdaGrad sweeps the 10 M
            # flags (40 MB) instead of electing and claiming the touched rows (same box, 30 steps:
            # 2.155 -> 2.122 ms per step; the gather side 286 -> 259 us); RS_STAYTIME_SCAN=0
            # keeps list mode (A/B)
            import os
            self.table.prefer_scan = os.environ.get("RS_STAYTIME_SCAN", "1") != "0"
        F = self.st_cfg.num_fields
        self.fields = EmbeddingFeatures(self.table, [rows] * F, row_base=[0] * F, combiner="mean",
                                        hash_mode="splitmix")
        self.seqs = nn.ModuleList(SequenceEmbedding(self.table, rows, self.st_cfg.seq_len,
                                                    hash_mode="splitmix")
                                  for _ in range(self.st_cfg.num_seq))
        nrr = self.rr_cfg.user_fields + self.rr_cfg.item_fields
        self.rr_fields = EmbeddingFeatures(self.table, [rows] * nrr, row_base=[0] * nrr,
                                           combiner="mean", hash_mode="splitmix")
        self.staytime = StaytimeMTL(self.st_cfg, device=dev, seed=seed + 1000)
        self.dssm = DSSM(self.rr_cfg, device=dev, seed=seed + 2000)

    def regularizers(self):
        return []

    def loss(self, st_ids, seq_ids, seq_offs, rr_ids, y_stay, y_short, y_long, sw, y_click, mask):
        emb = self.fields(st_ids)                                                 # [B, 91, 32]
        seqs, masks = [], []
        for s in range(self.st_cfg.num_seq):
            e, m = self.seqs[s](seq_ids[s], seq_offs[s])
            seqs.append(e)
            masks.append(m)
        st_terms = self.staytime.loss_terms(emb, seqs, masks, y_stay, y_short, y_long, sw)
        rr = self.rr_fields(rr_ids)           # [B, 52, 32]: the DSSM reads columns 0:16 per field
        # the joint total (staytime loss + DSSM loss) as ONE fused loss over the six outputs
        return fused_loss(st_terms + self.dssm.loss_terms(rr, mask, y_click), emb.shape[0])


def staytime_labels(rng, B):
    """staytime/parse.py:25-64 on synthetic watch times (LogNormal, ms)."""
    wt_ms = np.exp(rng.normal(9.5, 1.0, size=B))
    short = (wt_ms > 7000).astype(np.float32)[:, None]
    long_ = (wt_ms > 18000).astype(np.float32)[:, None]
    wt = np.minimum(wt_ms / 1000.0, 160.0)[:, None]
    bins = np.array(STAYTIME_BINS)[None, :]
    width = (180.5 - (-19)) / (400 - 1)
    lab = np.exp(np.square(np.abs(bins - wt)) / (-2 * 16.0)) / (math.sqrt(2 * math.pi) * 4) * width
    stay = np.concatenate([lab, wt], axis=1).astype(np.float32)
    sw = np.where(rng.uniform(size=B) < 0.1, 5.0, 1.0).astype(np.float32)
    return stay, short, long_, sw


def staytime_batch(rng, B, model: StaytimeRoughRank, device, id_space=1 << 40):
    st, rr = model.st_cfg, model.rr_cfg
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    st_ids = zipf_ids(rng, (B, st.num_fields), id_space, 1.2)
    seq_ids, seq_offs = [], []
    for _ in range(st.num_seq):
        lens = rng.integers(0, st.seq_len + 1, size=B)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        seq_ids.append(t(zipf_ids(rng, (int(offs[-1]),), id_space, 1.2)))
        seq_offs.append(t(offs))
    rr_ids = zipf_ids(rng, (B, rr.user_fields + rr.item_fields), id_space, 1.2)
    # labels built on the device from raw watch times (parse_input_func, staytime/parse.py:30-64)
    wt_ms = np.exp(rng.normal(9.5, 1.0, size=B)).astype(np.int64)
    landing = (rng.uniform(size=B) < 0.1).astype(np.uint8)
    stay, short, long_, sw = device_staytime_labels(t(wt_ms), t(landing))
    click = (rng.uniform(size=(B, 1)) < 0.1).astype(np.float32)
    mask = (rng.uniform(size=(B, 1)) < 0.5).astype(np.float32)
    return (t(st_ids), seq_ids, seq_offs, t(rr_ids), stay, short, long_, sw, t(click), t(mask))
