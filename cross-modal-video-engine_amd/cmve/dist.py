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


_NAN_GT = -1e300  # below every cosine: "this shard's GTs all score NaN" inside the MAX all-reduce


def encode_gt_scores(sgt: torch.Tensor) -> torch.Tensor:
    """Per-shard GT scores (cmve_gt_thresholds: NaN = no GT in this shard, +inf = GTs here but every
    one scores NaN, else the best finite score) -> keys whose MAX over the shards is the global
    answer: a finite score wins over NaN GTs, which win over no GT (NaN -> -inf, +inf -> -1e300)."""
    return torch.nan_to_num(sgt, nan=-np.inf, posinf=_NAN_GT)


def decode_gt_scores(key: torch.Tensor) -> torch.Tensor:
    """Inverse of encode_gt_scores after the MAX: -inf -> NaN (no GT anywhere), -1e300 -> +inf."""
    s = torch.where(key == _NAN_GT, torch.full_like(key, float("inf")), key)
    return torch.where(torch.isinf(s) & (s < 0), torch.full_like(s, float("nan")), s)


def merge_gt_scores(sgt_partial: torch.Tensor, world: int) -> torch.Tensor:
    """all-reduce(MAX) of per-shard best-GT scores (encode / MAX / decode)."""
    if world == 1:
        return sgt_partial
    s = encode_gt_scores(sgt_partial)
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    return decode_gt_scores(s)


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
    """Global 1-based ranks on the device (cmve_gt_ranks): no GT (NaN) -> n_global + 1, every GT NaN
    (+inf) -> n_global, else count + 1."""
    return engine.gt_ranks(cnt, sgt, n_q, n_global)


def pad_topk(idx: torch.Tensor, scores: torch.Tensor, k: int):
    """Pad a local [n_q, kk] top-k to k columns with empty slots (id -1, score NaN)."""
    n_q, kk = idx.shape
    if kk >= k:
        return idx, scores
    pi = torch.full((n_q, k - kk), -1, dtype=idx.dtype, device=idx.device)
    ps = torch.full((n_q, k - kk), float("nan"), dtype=scores.dtype, device=scores.device)
    return torch.cat([idx, pi], 1), torch.cat([scores, ps], 1)


def gather_topk(idx_global: torch.Tensor, scores: torch.Tensor, world: int):
    """all-gather of every shard's local top-k: [n_q, world * k] ids (int64) / fp64 scores, shard r's
    run at columns [r*k, (r+1)*k) of each query (the layout cmve_merge_topk reads)."""
    ids = idx_global.to(torch.int64).contiguous()
    sc = scores.to(torch.float64).contiguous()
    if world == 1:
        return ids, sc
    n_q, kk = ids.shape
    gi = torch.empty((world * n_q, kk), dtype=ids.dtype, device=ids.device)
    gs = torch.empty((world * n_q, kk), dtype=sc.dtype, device=sc.device)
    dist.all_gather_into_tensor(gi, ids)
    dist.all_gather_into_tensor(gs, sc)
    return (gi.reshape(world, n_q, kk).permute(1, 0, 2).reshape(n_q, -1).contiguous(),
            gs.reshape(world, n_q, kk).permute(1, 0, 2).reshape(n_q, -1).contiguous())


def merge_sorted_topk(ids: torch.Tensor, scores: torch.Tensor, lists: int, k: int):
    """cmve_merge_topk on the device: `lists` sorted runs per query -> the best k (score desc, global
    id asc; empty slots -1 / NaN)."""
    n_q, width = ids.shape
    k_in = width // lists
    out_i = torch.empty((n_q, k), dtype=torch.int64, device=ids.device)
    out_s = torch.empty((n_q, k), dtype=torch.float64, device=ids.device)
    _lib.check(_lib.lib.cmve_merge_topk(engine.handle(ids.device), engine._ptr(ids.contiguous()),
                                        engine._ptr(scores.contiguous()), n_q, lists, k_in, k,
                                        engine._ptr(out_i), engine._ptr(out_s)), "cmve_merge_topk")
    return out_i, out_s


def merge_topk(idx_global: torch.Tensor, scores: torch.Tensor, k: int, world: int, to_host: bool = True):
    """Gather every shard's local top-k (global ids, fp64 scores; id -1 = empty slot) and keep the best
    k per query, ordered (score desc, global id asc), by the HIP k-way merge.  Returns (ids int64
    [n_q, k'], scores fp64 [n_q, k']), k' = min(k, world * k_local); slots past the available entries
    hold -1 / NaN."""
    ids, sc = gather_topk(idx_global, scores, world)
    kout = min(k, ids.shape[1])
    out_i, out_s = merge_sorted_topk(ids, sc, world, kout)
    if not to_host:
        return out_i, out_s
    return out_i.cpu().numpy(), out_s.cpu().numpy()


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
        gt_csr: (off, idx) from ``local_gt_csr`` for the GATHERED query order.  The overflow flag of
        the undecided-pair list rides the counts' all-reduce, so every rank sees the same flag: all of
        them grow their lists and redo the batch together (a rank that trusted its own flag alone would
        return incomplete counts while another waited in the next all-gather)."""
        q_all = self.all_gather_rows(q_local)
        for _attempt in range(4):
            ranks, ovf = self.rank_queries_device(q_all, gt_csr, n_q, mode, events, chunks)
            if not bool(ovf.item()):
                break
            self.ws.grow()  # every rank: the flag is the all-reduced one
        else:
            raise _lib.CmveError("ShardedGallery.rank_queries: undecided-pair list kept overflowing")
        if not return_host:
            return ranks
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
        if kk < 1:  # an empty shard (shard_bounds' last rank): contributes k empty slots
            idx = torch.full((q.n, k), -1, dtype=torch.int64, device=self.device)
            sc = torch.full((q.n, k), float("nan"), dtype=torch.float64, device=self.device)
        else:
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
