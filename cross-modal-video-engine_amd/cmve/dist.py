"""Gallery sharded across the GPUs of a node (one process per GPU, RCCL over xGMI).

SURVEY.md section 8(e).  Each rank keeps a contiguous shard of the video gallery resident
in HBM (packed once).  Per query batch:
  1. all-gather of the query embeddings (RCCL; each rank contributes its slice),
  2. exact GT scores: every rank scores the GTs that live in its shard (fp64), then an
     all-reduce(MAX) gives each query its best-GT score,
  3. local fused rank count against the shard (bf16 MFMA pass + fp64 fix-up),
  4. all-reduce(SUM) of the int32 better-than-GT counts -> global ranks / R@K.
The top-k path all-gathers each shard's exact local top-k (score, global id) and merges
(score desc, global id asc).  The reference never shards.
With world_size 1 every collective is skipped.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import engine
from . import _lib


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n_global: int, world: int, rank: int):
    """Contiguous shards of ceil(n/world) rows: [lo, hi)."""
    per = (n_global + world - 1) // world
    lo = min(n_global, rank * per)
    return lo, min(n_global, lo + per)


class ShardedGallery:
    """This rank's gallery shard, packed in HBM, plus the global row offset."""

    def __init__(self, local_embs, offset: int, n_global: int, with_lo: bool = False, eps: float = 0.0,
                 device: Optional[torch.device] = None):
        self.rank, self.world = _world()
        self.shard = engine.RowSet(local_embs, eps=eps, with_lo=with_lo, device=device)
        self.device = self.shard.device
        self.offset = int(offset)
        self.n_global = int(n_global)
        self.ws = engine.RankWorkspace(self.device, cap=1 << 22)
        self._csr_cache = None

    # ---- GT lists restricted to this shard ----
    def local_gt_csr(self, gts_global: Sequence[Sequence[int]]):
        lo, hi = self.offset, self.offset + self.shard.n
        local = [[g - lo for g in l if lo <= g < hi] for l in gts_global]
        return engine.csr(local, self.device)

    def all_gather_rows(self, x_local: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return x_local
        out = torch.empty((self.world * x_local.shape[0],) + tuple(x_local.shape[1:]), dtype=x_local.dtype,
                          device=x_local.device)
        dist.all_gather_into_tensor(out, x_local.contiguous())
        return out

    def rank_queries(self, q_local: torch.Tensor, gt_csr, n_q: int, mode: int = _lib.SIM_BF16, events=None,
                     return_host: bool = True):
        """Global 1-based GT ranks of all gathered queries (t2v direction).

        q_local: this rank's [n_local, D] query embeddings (equal n_local on every rank);
        gt_csr: (off, idx) from ``local_gt_csr`` for the GATHERED query order."""
        q_all = self.all_gather_rows(q_local)
        q = engine.RowSet(q_all, with_lo=(mode == _lib.SIM_BF16X3), device=self.device)
        off, idx = gt_csr
        sgt, _, _ = engine.gt_thresholds(q, self.shard, off, idx, mode)
        if self.world > 1:
            sgt = torch.nan_to_num(sgt, nan=-np.inf)
            dist.all_reduce(sgt, op=dist.ReduceOp.MAX)
            sgt = torch.where(torch.isinf(sgt) & (sgt < 0), torch.full_like(sgt, float('nan')), sgt)
        hi, lo = engine.rank_thresholds(q, self.shard, sgt, mode)
        cnt, _ = engine.rank_count_launch(q, self.shard, mode, row=(sgt, hi, lo), ws=self.ws, events=events)
        if self.world > 1:
            dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        no_gt = torch.isnan(sgt[:n_q])
        ranks = torch.where(no_gt, torch.full_like(cnt[:n_q], self.n_global + 1), cnt[:n_q] + 1)
        if not return_host:
            return ranks
        ncand = int(self.ws.count.item())
        if ncand > self.ws.cap:  # overflow: grow and redo (correctness first)
            self.ws.grow(ncand)
            return self.rank_queries(q_local, gt_csr, n_q, mode, None, return_host)
        return ranks.cpu().numpy().astype(np.int64)

    def topk(self, q_local: torch.Tensor, k: int, mode: int = _lib.SIM_BF16):
        """Global exact top-k (global ids, fp64 cosines) of all gathered queries."""
        q_all = self.all_gather_rows(q_local)
        q = engine.RowSet(q_all, with_lo=self.shard.has_lo, device=self.device)
        kk = min(k, self.shard.n)
        idx, sc = engine.topk(q, self.shard, kk, mode=mode)
        idx = torch.from_numpy(idx + self.offset).to(self.device)
        sc = torch.from_numpy(sc).to(self.device)
        if self.world > 1:
            idx = self.all_gather_rows(idx.unsqueeze(0).contiguous()).reshape(self.world, q.n, kk)
            sc = self.all_gather_rows(sc.unsqueeze(0).contiguous()).reshape(self.world, q.n, kk)
            idx = idx.permute(1, 0, 2).reshape(q.n, -1)
            sc = sc.permute(1, 0, 2).reshape(q.n, -1)
        idx_h = idx.cpu().numpy()
        sc_h = sc.cpu().numpy()
        out = np.empty((q.n, min(k, idx_h.shape[1])), np.int64)
        out_s = np.empty(out.shape)
        for i in range(q.n):
            order = np.lexsort((idx_h[i], -sc_h[i]))[:out.shape[1]]  # score desc, global id asc
            out[i] = idx_h[i, order]
            out_s[i] = sc_h[i, order]
        return out, out_s


def metrics_from_ranks(ranks: np.ndarray) -> List[float]:
    """(R@1, R@5, R@10, medr, meanr) -- LINAS-engine/util/metrics.py:149-157."""
    n = ranks.shape[0]
    return [100.0 * np.count_nonzero(ranks <= 1) / n, 100.0 * np.count_nonzero(ranks <= 5) / n,
            100.0 * np.count_nonzero(ranks <= 10) / n, float(np.median(ranks)), float(ranks.mean())]
