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


# ---- collective steps (device-agnostic: RCCL on the GPU path, gloo in the CPU tests) ----

def local_gt_lists(gts_global: Sequence[Sequence[int]], lo: int, hi: int):
    """GT lists restricted to the shard [lo, hi), re-indexed locally."""
    return [[g - lo for g in l if lo <= g < hi] for l in gts_global]


def merge_gt_scores(sgt_partial: torch.Tensor, world: int) -> torch.Tensor:
    """all-reduce(MAX) of per-shard best-GT scores; NaN (no GT in this shard) -> -inf -> NaN."""
    if world == 1:
        return sgt_partial
    s = torch.nan_to_num(sgt_partial, nan=-np.inf)
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    return torch.where(torch.isinf(s) & (s < 0), torch.full_like(s, float('nan')), s)


def reduce_counts(cnt: torch.Tensor, world: int) -> torch.Tensor:
    """all-reduce(SUM) of per-shard better-than-GT counts."""
    if world > 1:
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    return cnt


def gather_rows_async(x_local: torch.Tensor, out: torch.Tensor, world: int):
    """all_gather_into_tensor(out, x_local) as an async collective (RCCL runs it on its own stream):
    returns the Work to .wait() on before reading `out`, or None at world 1 (plain copy)."""
    if world == 1:
        out.copy_(x_local)
        return None
    return dist.all_gather_into_tensor(out, x_local.contiguous(), async_op=True)


def any_flag(flag: torch.Tensor, world: int) -> torch.Tensor:
    """OR of a per-rank boolean over the ranks (all-reduce MAX), so that all ranks take the same branch."""
    if world == 1:
        return flag
    o = flag.to(torch.int32).reshape(1)
    dist.all_reduce(o, op=dist.ReduceOp.MAX)
    return o[0] > 0


def ranks_from(cnt: torch.Tensor, sgt: torch.Tensor, n_q: int, n_global: int) -> torch.Tensor:
    no_gt = torch.isnan(sgt[:n_q])
    c = cnt[:n_q].to(torch.int64)
    return torch.where(no_gt, torch.full_like(c, n_global + 1), c + 1)


def pad_topk(idx: torch.Tensor, scores: torch.Tensor, k: int):
    """Pad a local [n_q, kk] top-k to k columns with empty slots (id -1, score NaN)."""
    n_q, kk = idx.shape
    if kk >= k:
        return idx, scores
    pi = torch.full((n_q, k - kk), -1, dtype=idx.dtype, device=idx.device)
    ps = torch.full((n_q, k - kk), float("nan"), dtype=scores.dtype, device=scores.device)
    return torch.cat([idx, pi], 1), torch.cat([scores, ps], 1)


def merge_topk(idx_global: torch.Tensor, scores: torch.Tensor, k: int, world: int, to_host: bool = True):
    """Gather every shard's local top-k (global ids, fp64 scores) and keep the best k per query,
    ordered (score desc, global id asc) -- on the device: a stable sort by id, then a stable sort by
    descending score.  idx_global/scores: [n_q, k_local]; id -1 marks an empty slot (score ignored).
    Returns (ids int64 [n_q, k'], scores fp64 [n_q, k']) with k' = min(k, world * k_local); slots
    past the available entries hold -1 / NaN."""
    n_q, kk = idx_global.shape
    if world == 1:  # one shard: its top-k is already in (score desc, id asc) order
        ids = idx_global.to(torch.int64)[:, :k]
        sc = scores.to(torch.float64)[:, :k]
        sc = torch.where(ids < 0, torch.full_like(sc, float("nan")), sc)
        return (ids, sc) if not to_host else (ids.cpu().numpy(), sc.cpu().numpy())
    if world > 1:
        gi = torch.empty((world * n_q, kk), dtype=idx_global.dtype, device=idx_global.device)
        gs = torch.empty((world * n_q, kk), dtype=scores.dtype, device=scores.device)
        dist.all_gather_into_tensor(gi, idx_global.contiguous())
        dist.all_gather_into_tensor(gs, scores.contiguous())
        idx_global = gi.reshape(world, n_q, kk).permute(1, 0, 2).reshape(n_q, -1)
        scores = gs.reshape(world, n_q, kk).permute(1, 0, 2).reshape(n_q, -1)
    ids = idx_global.to(torch.int64)
    sc = scores.to(torch.float64)
    empty = ids < 0
    key_id = torch.where(empty, torch.full_like(ids, torch.iinfo(torch.int64).max), ids)
    key_sc = torch.where(empty, torch.full_like(sc, -float("inf")), sc)
    o1 = torch.argsort(key_id, dim=1, stable=True)
    key_id, key_sc, empty = key_id.gather(1, o1), key_sc.gather(1, o1), empty.gather(1, o1)
    o2 = torch.argsort(-key_sc, dim=1, stable=True)
    kout = min(k, ids.shape[1])
    o2 = o2[:, :kout]
    out_id, out_sc, out_empty = key_id.gather(1, o2), key_sc.gather(1, o2), empty.gather(1, o2)
    out_id = torch.where(out_empty, torch.full_like(out_id, -1), out_id)
    out_sc = torch.where(out_empty, torch.full_like(out_sc, float("nan")), out_sc)
    if not to_host:
        return out_id, out_sc
    return out_id.cpu().numpy(), out_sc.cpu().numpy()


class ShardedGallery:
    """This rank's gallery shard, packed in HBM, plus the global row offset."""

    def __init__(self, local_embs, offset: int, n_global: int, with_lo: bool = False, eps: float = 0.0,
                 device: Optional[torch.device] = None, with_f16: bool = True):
        self.rank, self.world = _world()
        self.shard = engine.RowSet(local_embs, eps=eps, with_lo=with_lo, device=device, with_f16=with_f16)
        self.device = self.shard.device
        self.offset = int(offset)
        self.n_global = int(n_global)
        self.ws = engine.RankWorkspace(self.device, cap=1 << 22)
        self._csr_cache = None

    # ---- GT lists restricted to this shard ----
    def local_gt_csr(self, gts_global: Sequence[Sequence[int]]):
        return engine.csr(local_gt_lists(gts_global, self.offset, self.offset + self.shard.n), self.device)

    def all_gather_rows(self, x_local: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return x_local
        out = torch.empty((self.world * x_local.shape[0],) + tuple(x_local.shape[1:]), dtype=x_local.dtype,
                          device=x_local.device)
        dist.all_gather_into_tensor(out, x_local.contiguous())
        return out

    def rank_queries(self, q_local: torch.Tensor, gt_csr, n_q: int, mode: int = _lib.SIM_F16, events=None,
                     return_host: bool = True, chunks: int = 1):
        """Global 1-based GT ranks of all gathered queries (t2v direction).

        q_local: this rank's [n_local, D] query embeddings (equal n_local on every rank);
        gt_csr: (off, idx) from ``local_gt_csr`` for the GATHERED query order."""
        q_all = self.all_gather_rows(q_local)
        q = engine.RowSet(q_all, with_lo=(mode == _lib.SIM_BF16X3), with_f16=(mode == _lib.SIM_F16),
                          device=self.device)
        off, idx = gt_csr
        sgt, _, _ = engine.gt_thresholds(q, self.shard, off, idx, mode)
        sgt = merge_gt_scores(sgt, self.world)
        hi, lo = engine.rank_thresholds(q, self.shard, sgt, mode)
        cnt, _ = engine.rank_count_launch(q, self.shard, mode, row=(sgt, hi, lo), ws=self.ws, events=events,
                                          chunks=chunks)
        cnt = reduce_counts(cnt, self.world)
        ranks = ranks_from(cnt, sgt, n_q, self.n_global)
        if not return_host:
            return ranks
        if self.ws.overflowed():  # overflow: grow and redo (correctness first)
            self.ws.grow()
            return self.rank_queries(q_local, gt_csr, n_q, mode, None, return_host, chunks)
        return ranks.cpu().numpy().astype(np.int64)

    def gather_rows_async(self, x_local: torch.Tensor, out: torch.Tensor):
        """gather_rows_async for this rank's world.  Issue it BEFORE enqueueing the compute that
        should overlap it -- the collective first waits for the work already on the current stream --
        and call .wait() on the returned Work before reading `out`."""
        return gather_rows_async(x_local, out, self.world)

    def rank_queries_device(self, q_all: torch.Tensor, gt_csr, n_q: int, mode: int = _lib.SIM_F16, events=None,
                            chunks: int = 1):
        """rank_queries on already-gathered queries with no host synchronisation: returns
        (ranks int64 [n_q] on the device, overflow flag bool [] on the device).  A set flag means the
        undecided-pair list overflowed and the counts are incomplete: grow the workspace and redo."""
        q = engine.RowSet(q_all, with_lo=(mode == _lib.SIM_BF16X3), with_f16=(mode == _lib.SIM_F16),
                          device=self.device)
        off, idx = gt_csr
        sgt, _, _ = engine.gt_thresholds(q, self.shard, off, idx, mode)
        sgt = merge_gt_scores(sgt, self.world)
        hi, lo = engine.rank_thresholds(q, self.shard, sgt, mode)
        cnt, _ = engine.rank_count_launch(q, self.shard, mode, row=(sgt, hi, lo), ws=self.ws, events=events,
                                          chunks=chunks)
        ch = self.ws.chunks
        ovf = (self.ws.count[:ch] > self.ws.cap // ch).any()
        if self.world > 1:  # the overflow flag rides the counts' all-reduce(SUM): one collective, all ranks agree
            both = reduce_counts(torch.cat([cnt, ovf.to(cnt.dtype).reshape(1)]), self.world)
            cnt, ovf = both[:-1], both[-1] > 0
        return ranks_from(cnt, sgt, n_q, self.n_global), ovf

    def topk(self, q_local: torch.Tensor, k: int, mode: int = _lib.SIM_F16):
        """Global exact top-k (global ids, fp64 cosines) of all gathered queries."""
        q_all = self.all_gather_rows(q_local)
        q = engine.RowSet(q_all, with_lo=self.shard.has_lo, with_f16=self.shard.has_f16, device=self.device)
        kk = min(k, self.shard.n)
        idx, sc = engine.topk(q, self.shard, kk, mode=mode, to_host=False)
        idx = idx.to(torch.int64)
        idx = torch.where(idx >= 0, idx + self.offset, idx)
        idx, sc = pad_topk(idx, sc, k)  # every rank contributes k columns (shards may hold fewer rows)
        return merge_topk(idx, sc, k, self.world)


def recall_counts_device(ranks: torch.Tensor) -> torch.Tensor:
    """#(rank <= 1), #(rank <= 5), #(rank <= 10), sum of ranks: int64 [4] on the device (R@K counts
    without a host round trip; metrics.py:149-157 divides by n_q)."""
    return torch.stack([(ranks <= 1).sum(), (ranks <= 5).sum(), (ranks <= 10).sum(), ranks.sum()])


def metrics_from_ranks(ranks: np.ndarray) -> List[float]:
    """(R@1, R@5, R@10, medr, meanr) -- LINAS-engine/util/metrics.py:149-157."""
    n = ranks.shape[0]
    return [100.0 * np.count_nonzero(ranks <= 1) / n, 100.0 * np.count_nonzero(ranks <= 5) / n,
            100.0 * np.count_nonzero(ranks <= 10) / n, float(np.median(ranks)), float(ranks.mean())]
