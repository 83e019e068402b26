"""Gallery sharded across GPUs: one shard per rank, RCCL over xGMI.

Each rank keeps a contiguous shard of the video gallery resident in HBM (packed once).  One
exact two-direction evaluation of a caption batch (the reference's ``cal_perf`` over
``cal_error``, ``LINAS-engine/validate.py:15-54``, ``util/metrics.py:124-157``) is:
  1. all-gather of the caption embeddings (each rank contributes its slice);
  2. t2v GT scores: every rank scores the GTs that live in its shard (fp64), an all-reduce(MAX)
     gives each caption its best-GT score;
     v2t GT scores: a video's GT captions are all present after the gather, so they are local;
  3. ONE fused rank GEMM over (all captions) x (this shard): row counts (t2v, partial: this
     shard's videos) and column counts (v2t, complete: every caption) -- fp16 MFMA + fp64 fix-up;
  4. one all-reduce(SUM) carrying the t2v counts, this shard's v2t R@K sums and the
     undecided-pair overflow flag -> global t2v ranks on every rank, global v2t R@K sums.
     The v2t ranks themselves are rank-local (medr / mAP gather them once at the end).
The top-k path all-gathers each shard's exact local top-k (score, global id) and merges them
(score desc, global id asc) on the device (cmve_merge_topk).  The reference never shards
(SURVEY.md section 0.2).

Collectives go through a communicator object: ``TorchComm`` is the torch.distributed process
group (backend "nccl" = RCCL on the GPU, gloo in the CPU tests); ``LocalGroup`` runs N shards in
ONE process, one thread and HIP stream per shard (a host driving several shards -- on one GPU or
several -- with the same coordination code).  ``ShardedGallery``'s shard-local arithmetic is a
handful of methods (``_pack``, ``_row_gt``, ``_col_gt``, ``_count``, ``_ranks``, ``_positions``)
over the HIP kernels; the coordination above them is shared by every communicator.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional, Sequence

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


# ---------------------------------------------------------------------------------------------
# communicators
# ---------------------------------------------------------------------------------------------

class _Done:
    """A completed collective (the Work of a synchronous exchange)."""

    def wait(self):
        return True


class TorchComm:
    """torch.distributed's default process group (RCCL on the GPU path, gloo in CPU tests); a
    single-process job (no process group) is world 1 and every collective is a no-op / copy."""

    def __init__(self):
        self.rank, self.world = _world()

    def all_reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        """In place; op 'sum' or 'max'."""
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
        return t

    def all_gather_into(self, out: torch.Tensor, x: torch.Tensor, async_op: bool = False):
        """out = cat over ranks of x (equal shapes); async_op returns a Work to .wait() on."""
        if self.world == 1:
            out.copy_(x)
            return _Done() if async_op else None
        w = dist.all_gather_into_tensor(out, x.contiguous(), async_op=async_op)
        return w

    def barrier(self):
        if self.world > 1:
            dist.barrier()


class CAbiComm:
    """The torch.distributed ranks over the C ABI's own RCCL communicator (``cmve_dist_*``, csrc/dist.hip): the
    collectives a host without torch would call, driven through the same ShardedGallery coordination.  The
    128-byte unique id is made on rank 0 and broadcast over the process group (``uid`` given: used as is,
    e.g. by a host with its own bootstrap); every collective is enqueued on the caller's current stream.
    At world 1 the collectives still run (identity gathers / reductions), so the path is exercised on one GPU."""

    always = True  # run the collectives at world 1 too (see _solo)
    _TYPES = {torch.float32: _lib.CMVE_F32, torch.float64: _lib.CMVE_F64, torch.int32: _lib.CMVE_I32,
              torch.int64: _lib.CMVE_I64}

    def __init__(self, device: Optional[torch.device] = None, rank: Optional[int] = None,
                 world: Optional[int] = None, uid: Optional[bytes] = None):
        import ctypes as C
        r0, w0 = _world()
        self.rank = r0 if rank is None else int(rank)
        self.world = w0 if world is None else int(world)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        self.device = torch.device(dev.type, idx)  # indexed: tensors report 'cuda:N', never bare 'cuda'
        if uid is None:
            buf = C.create_string_buffer(_lib.DIST_UNIQUE_ID_BYTES)
            if self.rank == 0:
                _lib.check(_lib.lib.cmve_dist_unique_id(buf), "cmve_dist_unique_id")
            if self.world > 1:
                obj = [bytes(buf.raw) if self.rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                buf = C.create_string_buffer(obj[0], _lib.DIST_UNIQUE_ID_BYTES)
        else:
            buf = C.create_string_buffer(bytes(uid), _lib.DIST_UNIQUE_ID_BYTES)
        h = C.c_void_p()
        _lib.check(_lib.lib.cmve_create(idx, C.c_void_p(torch.cuda.current_stream(idx).cuda_stream), C.byref(h)),
                   "cmve_create")
        self._h = h.value
        _lib.check(_lib.lib.cmve_dist_init(self._h, self.world, self.rank, buf), "cmve_dist_init")
        n, rk = C.c_int32(), C.c_int32()
        _lib.check(_lib.lib.cmve_dist_size(self._h, C.byref(n), C.byref(rk)), "cmve_dist_size")
        if (n.value, rk.value) != (self.world, self.rank):
            raise RuntimeError(f"CAbiComm: communicator is rank {rk.value} of {n.value}, expected "
                               f"{self.rank} of {self.world}")

    def _code(self, t: torch.Tensor) -> int:
        if t.dtype not in self._TYPES or not t.is_contiguous() or t.device != self.device:
            raise ValueError(f"CAbiComm: contiguous {list(self._TYPES)} tensors on {self.device} only, got "
                             f"{t.dtype} on {t.device}")
        return self._TYPES[t.dtype]

    def _on_current(self):
        import ctypes as C
        _lib.check(_lib.lib.cmve_set_stream(self._h, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "cmve_set_stream")

    def all_reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        """In place; op 'sum' or 'max'."""
        code = self._code(t)
        self._on_current()
        _lib.check(_lib.lib.cmve_dist_allreduce(self._h, engine._ptr(t), t.numel(), code,
                                                _lib.DIST_SUM if op == "sum" else _lib.DIST_MAX),
                   "cmve_dist_allreduce")
        return t

    def all_gather_into(self, out: torch.Tensor, x: torch.Tensor, async_op: bool = False):
        """out = cat over ranks of x (equal shapes), enqueued on the current stream (async_op: a completed
        Work -- the stream order already holds every later reader)."""
        x = x.contiguous()
        code = self._code(x)
        if (out.dtype != x.dtype or out.numel() != self.world * x.numel() or not out.is_contiguous()
                or out.device != self.device):
            raise ValueError(f"CAbiComm.all_gather_into: out must be world x the input, same dtype, contiguous, on "
                             f"{self.device}")
        self._on_current()
        _lib.check(_lib.lib.cmve_dist_allgather(self._h, engine._ptr(x), x.numel(), code, engine._ptr(out)),
                   "cmve_dist_allgather")
        return _Done() if async_op else None

    def barrier(self):
        t = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.all_reduce(t, "sum")
        torch.cuda.current_stream(self.device).synchronize()

    def close(self):
        if self._h:
            _lib.lib.cmve_dist_destroy(self._h)
            _lib.lib.cmve_destroy(self._h)
            self._h = None


class ThreadComm:
    """One shard's view of a ``LocalGroup``: the collectives of TorchComm between threads of one
    process.  Every exchange completes its inputs on the caller's stream first and its outputs
    before returning, so the shards may run on different HIP streams (or devices)."""

    def __init__(self, group: "LocalGroup", rank: int):
        self.group, self.rank, self.world = group, rank, group.n

    def _exchange(self, x: torch.Tensor) -> List[torch.Tensor]:
        if x.is_cuda:
            torch.cuda.current_stream(x.device).synchronize()
        g = self.group
        g.slots[self.rank] = x
        g.barrier.wait()
        vals = list(g.slots)
        return vals

    def _release(self, out: torch.Tensor):
        if out.is_cuda:
            torch.cuda.current_stream(out.device).synchronize()
        self.group.barrier.wait()  # every shard has read the deposited inputs

    def all_reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        vals = [v.to(t.device) for v in self._exchange(t)]
        st = torch.stack(vals)
        r = st.sum(0) if op == "sum" else st.max(0).values
        self._release(r)
        t.copy_(r)
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()
        return t

    def all_gather_into(self, out: torch.Tensor, x: torch.Tensor, async_op: bool = False):
        vals = [v.to(out.device) for v in self._exchange(x.contiguous())]
        r = torch.cat(vals)
        self._release(r)
        out.copy_(r.reshape(out.shape))
        if out.is_cuda:
            torch.cuda.current_stream(out.device).synchronize()
        return _Done() if async_op else None

    def barrier(self):
        self.group.barrier.wait()


class LocalGroup:
    """N shards in ONE process: ``run(fn)`` calls fn(rank, comm) on N threads, each on its own HIP
    stream (devices[rank] if given, else the current device), and returns the N results.  The
    coordination code is the same as across processes; a shard that raises aborts the group."""

    def __init__(self, n: int, devices: Optional[Sequence[torch.device]] = None, timeout: float = 600.0):
        self.n = int(n)
        self.devices = list(devices) if devices is not None else None
        self.barrier = threading.Barrier(self.n, timeout=timeout)
        self.slots: List[Optional[torch.Tensor]] = [None] * self.n

    def comm(self, rank: int) -> ThreadComm:
        return ThreadComm(self, rank)

    def run(self, fn: Callable[[int, ThreadComm], object]) -> list:
        results: list = [None] * self.n
        errors: list = [None] * self.n

        def body(r):
            try:
                dev = self.devices[r] if self.devices is not None else None
                if torch.cuda.is_available():
                    dev = dev or torch.device("cuda", torch.cuda.current_device())
                    torch.cuda.set_device(dev)
                    with torch.cuda.stream(torch.cuda.Stream(dev)):
                        results[r] = fn(r, self.comm(r))
                        torch.cuda.current_stream(dev).synchronize()
                else:
                    results[r] = fn(r, self.comm(r))
            except BaseException as e:  # noqa: BLE001 -- re-raised below; free the others
                errors[r] = e
                self.barrier.abort()

        threads = [threading.Thread(target=body, args=(r,)) for r in range(self.n)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        first = next((e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)), None)
        if first is None:
            first = next((e for e in errors if e is not None), None)
        if first is not None:
            raise first
        return results


def _solo(comm) -> bool:
    """A world-1 communicator whose collectives may be skipped (CAbiComm runs them even then: `always`)."""
    return comm.world == 1 and not getattr(comm, "always", False)


def _comm(comm):
    """A communicator from None (TorchComm), an int world size (legacy: TorchComm, which must agree),
    or a communicator object."""
    if comm is None or isinstance(comm, int):
        c = TorchComm()
        if isinstance(comm, int) and comm != c.world:
            raise ValueError(f"world {comm} given, but the process group has {c.world} ranks")
        return c
    return comm


# ---------------------------------------------------------------------------------------------
# collective steps (device-agnostic: RCCL / gloo / threads)
# ---------------------------------------------------------------------------------------------

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


def merge_gt_scores(sgt_partial: torch.Tensor, comm=None) -> torch.Tensor:
    """all-reduce(MAX) of per-shard best-GT scores (encode / MAX / decode)."""
    comm = _comm(comm)
    if _solo(comm):
        return sgt_partial
    s = encode_gt_scores(sgt_partial)
    comm.all_reduce(s, "max")
    return decode_gt_scores(s)


def reduce_counts(cnt: torch.Tensor, comm=None) -> torch.Tensor:
    """all-reduce(SUM) of per-shard better-than-GT counts."""
    return _comm(comm).all_reduce(cnt, "sum")


def gather_rows_async(x_local: torch.Tensor, out: torch.Tensor, comm=None):
    """all_gather_into_tensor(out, x_local) as an async collective (RCCL runs it on its own stream):
    returns the Work to .wait() on before reading `out`, or None at world 1 (plain copy)."""
    comm = _comm(comm)
    if _solo(comm):
        out.copy_(x_local)
        return None
    return comm.all_gather_into(out, x_local.contiguous(), async_op=True)


def all_gather_rows(x_local: torch.Tensor, comm=None) -> torch.Tensor:
    """Rows of every rank in rank order (equal row counts on every rank)."""
    comm = _comm(comm)
    if _solo(comm):
        return x_local
    out = torch.empty((comm.world * x_local.shape[0],) + tuple(x_local.shape[1:]), dtype=x_local.dtype,
                      device=x_local.device)
    comm.all_gather_into(out, x_local.contiguous())
    return out


def all_gather_var(x_local: torch.Tensor, comm=None) -> torch.Tensor:
    """Rows of every rank in rank order when ranks hold different row counts: the counts are
    gathered first, every rank pads to the largest, and the padding is dropped after the gather."""
    comm = _comm(comm)
    if _solo(comm):
        return x_local
    n = torch.tensor([x_local.shape[0]], dtype=torch.int64, device=x_local.device)
    ns = all_gather_rows(n, comm).tolist()
    m = max(ns)
    if min(ns) == m:
        return all_gather_rows(x_local, comm)
    pad = torch.zeros((m,) + tuple(x_local.shape[1:]), dtype=x_local.dtype, device=x_local.device)
    pad[:x_local.shape[0]] = x_local
    g = all_gather_rows(pad, comm)
    return torch.cat([g[r * m:r * m + ns[r]] for r in range(comm.world)])


def any_flag(flag: torch.Tensor, comm=None) -> torch.Tensor:
    """OR of a per-rank boolean over the ranks (all-reduce MAX), so that all ranks take the same branch."""
    comm = _comm(comm)
    if _solo(comm):
        return flag
    o = flag.to(torch.int32).reshape(1)
    comm.all_reduce(o, "max")
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


def gather_topk(idx_global: torch.Tensor, scores: torch.Tensor, comm=None):
    """all-gather of every shard's local top-k: [n_q, world * k] ids (int64) / fp64 scores, shard r's
    run at columns [r*k, (r+1)*k) of each query (the layout cmve_merge_topk reads)."""
    comm = _comm(comm)
    world = comm.world
    ids = idx_global.to(torch.int64).contiguous()
    sc = scores.to(torch.float64).contiguous()
    if _solo(comm):
        return ids, sc
    n_q, kk = ids.shape
    gi = all_gather_rows(ids, comm)
    gs = all_gather_rows(sc, comm)
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


def merge_topk(idx_global: torch.Tensor, scores: torch.Tensor, k: int, comm=None, to_host: bool = True):
    """Gather every shard's local top-k (global ids, fp64 scores; id -1 = empty slot) and keep the best
    k per query, ordered (score desc, global id asc), by the HIP k-way merge.  Returns (ids int64
    [n_q, k'], scores fp64 [n_q, k']), k' = min(k, world * k_local); slots past the available entries
    hold -1 / NaN."""
    comm = _comm(comm)
    ids, sc = gather_topk(idx_global, scores, comm)
    kout = min(k, ids.shape[1])
    out_i, out_s = merge_sorted_topk(ids, sc, comm.world, kout)
    if not to_host:
        return out_i, out_s
    return out_i.cpu().numpy(), out_s.cpu().numpy()


def recall_counts_device(ranks: torch.Tensor) -> torch.Tensor:
    """#(rank <= 1), #(rank <= 5), #(rank <= 10), sum of ranks: int64 [4] on the device (R@K counts
    without a host round trip; metrics.py:149-157 divides by n_q)."""
    return torch.stack([(ranks <= 1).sum(), (ranks <= 5).sum(), (ranks <= 10).sum(), ranks.sum()])


def metrics_from_ranks(ranks: np.ndarray) -> List[float]:
    """(R@1, R@5, R@10, medr, meanr) -- LINAS-engine/util/metrics.py:149-157."""
    n = ranks.shape[0]
    return [100.0 * np.count_nonzero(ranks <= 1) / n, 100.0 * np.count_nonzero(ranks <= 5) / n,
            100.0 * np.count_nonzero(ranks <= 10) / n, float(np.median(ranks)), float(ranks.mean())]


def metrics_from_recall(rec: Sequence[int], n: int) -> List[float]:
    """(R@1, R@5, R@10, meanr) from recall_counts_device sums over n queries."""
    return [100.0 * rec[0] / n, 100.0 * rec[1] / n, 100.0 * rec[2] / n, rec[3] / n]


def ap_from_positions(positions) -> float:
    """APScorer (LINAS-engine/basic/metric.py:31-46) from the positions of a list's relevant items."""
    p = np.sort(np.asarray(positions, np.float64))
    if p.size == 0:
        return 0.0
    return float(np.sum(np.arange(1, p.size + 1) / p) / p.size)


# ---------------------------------------------------------------------------------------------
# the shard
# ---------------------------------------------------------------------------------------------

class ShardedGallery:
    """This rank's gallery shard [offset, offset + n) of an n_global-video gallery, packed in HBM.

    ``comm``: a communicator (default: TorchComm over torch.distributed's process group)."""

    def __init__(self, local_embs, offset: int, n_global: int, with_lo: bool = False, eps: float = 0.0,
                 device: Optional[torch.device] = None, with_f16: bool = True, comm=None, cap: int = 1 << 22):
        self.comm = _comm(comm)
        self.rank, self.world = self.comm.rank, self.comm.world
        self.offset = int(offset)
        self.n_global = int(n_global)
        self._setup(local_embs, with_lo, eps, device, with_f16, cap)

    def _setup(self, local_embs, with_lo, eps, device, with_f16, cap):
        self.shard = engine.RowSet(local_embs, eps=eps, with_lo=with_lo, device=device, with_f16=with_f16)
        self.device = self.shard.device
        self.n = self.shard.n
        self.eps = eps
        self.ws = engine.RankWorkspace(self.device, cap=cap)

    # ---- shard-local arithmetic (HIP kernels) ----
    def _pack(self, q_all: torch.Tensor, mode: int):
        return engine.RowSet(q_all, eps=self.eps, with_lo=(mode == _lib.SIM_BF16X3), with_f16=(mode == _lib.SIM_F16),
                             device=self.device)

    def _csr(self, lists):
        return engine.csr(lists, self.device)

    def _row_gt(self, q, csr, mode: int) -> torch.Tensor:
        """Best fp64 GT score of every caption over the GTs in this shard (NaN none, +inf all NaN)."""
        off, idx = csr
        return engine.gt_thresholds(q, self.shard, off, idx, mode)[0]

    def _col_gt(self, q, csr, mode: int):
        """(best GT score, thresholds) of every shard video over its GT captions (all gathered)."""
        off, idx = csr
        return engine.gt_thresholds(self.shard, q, off, idx, mode)

    def _count(self, q, mode: int, sgt_row: Optional[torch.Tensor], col, events=None, chunks: int = 1):
        """One fused rank GEMM: (row counts [q.n_pad] | None, col counts [n_pad] | None, overflow bool [])."""
        if sgt_row is None and col is None:
            return None, None, torch.zeros((), dtype=torch.bool, device=self.device)
        row = None
        if sgt_row is not None:
            hi, lo = engine.rank_thresholds(q, self.shard, sgt_row, mode)
            row = (sgt_row, hi, lo)
        rc, cc = engine.rank_count_launch(q, self.shard, mode, row=row, col=col, ws=self.ws, events=events,
                                          chunks=chunks)
        ch = self.ws.chunks
        ovf = (self.ws.count[:ch] > self.ws.cap // ch).any()
        return rc, cc, ovf

    def _ranks(self, cnt, sgt, n: int, n_m: int) -> torch.Tensor:
        return ranks_from(cnt, sgt, n, n_m)

    def _grow(self):
        self.ws.grow()

    def _positions(self, q, lists, mode: int):
        """1-based positions of every GT caption of every shard video among all captions (v2t mAP)."""
        return engine.gt_positions_fused(self.shard, q, lists, mode=mode)

    # ---- GT lists restricted to this shard ----
    def local_gt_csr(self, gts_global: Sequence[Sequence[int]]):
        """t2v: every caption's GT videos inside this shard, re-indexed locally."""
        return self._csr(local_gt_lists(gts_global, self.offset, self.offset + self.n))

    def local_v2t_csr(self, v2t_gts_global: Sequence[Sequence[int]]):
        """v2t: the GT captions (gathered order) of this shard's videos."""
        return self._csr(self.local_v2t_lists(v2t_gts_global))

    def local_v2t_lists(self, v2t_gts_global):
        return [list(v2t_gts_global[self.offset + j]) for j in range(self.n)]

    # ---- collectives ----
    def all_gather_rows(self, x_local: torch.Tensor) -> torch.Tensor:
        return all_gather_rows(x_local, self.comm)

    def gather_rows_async(self, x_local: torch.Tensor, out: torch.Tensor):
        """gather_rows_async for this shard's communicator.  Issue it BEFORE enqueueing the compute that
        should overlap it -- the collective first waits for the work already on the current stream --
        and call .wait() on the returned Work before reading `out`."""
        return gather_rows_async(x_local, out, self.comm)

    # ---- t2v only (the gallery_shard bench leg) ----
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
            self._grow()  # every rank: the flag is the all-reduced one
        else:
            raise _lib.CmveError("ShardedGallery.rank_queries: undecided-pair list kept overflowing")
        if not return_host:
            return ranks
        return ranks.cpu().numpy().astype(np.int64)

    def rank_queries_device(self, q_all: torch.Tensor, gt_csr, n_q: int, mode: int = _lib.SIM_F16, events=None,
                            chunks: int = 1):
        """rank_queries on already-gathered queries with no host synchronisation: returns
        (ranks int64 [n_q] on the device, overflow flag bool [] on the device).  A set flag means the
        undecided-pair list overflowed and the counts are incomplete: grow the workspace and redo."""
        q = self._pack(q_all, mode)
        sgt = merge_gt_scores(self._row_gt(q, gt_csr, mode), self.comm)
        cnt, _, ovf = self._count(q, mode, sgt, None, events=events, chunks=chunks)
        if self.world > 1:  # the overflow flag rides the counts' all-reduce(SUM): one collective, all ranks agree
            both = reduce_counts(torch.cat([cnt, ovf.to(cnt.dtype).reshape(1)]), self.comm)
            cnt, ovf = both[:-1], both[-1] > 0
        return self._ranks(cnt, sgt, n_q, self.n_global), ovf

    # ---- both directions (cal_perf) ----
    def evaluate_device(self, q_all: torch.Tensor, row_csr, col_csr, n_q: int, mode: int = _lib.SIM_F16,
                        events=None, q=None):
        """One exact two-direction evaluation of the gathered captions against every shard, no host
        synchronisation.  row_csr: t2v GT lists restricted to this shard (``local_gt_csr``) or None;
        col_csr: this shard's v2t GT lists into the gathered captions (``local_v2t_csr``) or None.
        Returns (t2v ranks int64 [n_q] | None -- global, equal on every rank; v2t ranks int64 [n] | None
        -- this shard's videos; v2t recall sums int64 [4] | None -- all shards; overflow bool []).  q: the
        captions already packed (``_pack(q_all, mode)``), reused across passes over the same captions."""
        if q is None:
            q = self._pack(q_all, mode)
        sgt_r = merge_gt_scores(self._row_gt(q, row_csr, mode), self.comm) if row_csr is not None else None
        col = self._col_gt(q, col_csr, mode) if (col_csr is not None and self.n > 0) else None
        rc, cc, ovf = self._count(q, mode, sgt_r, col, events=events)
        v2t = self._ranks(cc, col[0], self.n, n_q) if col is not None else None
        if col_csr is not None and self.n == 0:  # an empty shard (shard_bounds' last rank): no videos to rank
            v2t = torch.zeros(0, dtype=torch.int64, device=ovf.device)
        parts = []
        if rc is not None:
            parts.append(rc[:n_q].to(torch.int64))
        v2t_rec = recall_counts_device(v2t) if v2t is not None else torch.zeros(4, dtype=torch.int64,
                                                                                   device=ovf.device)
        parts += [v2t_rec, ovf.to(torch.int64).reshape(1)]
        # ONE all-reduce(SUM): the t2v counts, the v2t R@K sums and the overflow flag
        both = reduce_counts(torch.cat(parts), self.comm)
        ovf = both[-1] > 0
        rec = both[-5:-1] if col_csr is not None else None
        t2v = self._ranks(both[:n_q].to(torch.int32), sgt_r, n_q, self.n_global) if row_csr is not None else None
        return t2v, v2t, rec, ovf

    def evaluate(self, q_local: torch.Tensor, t2v_gts=None, v2t_gts=None, mode: int = _lib.SIM_F16):
        """Exact global ranks of both directions, on every rank (host int64 arrays): captions = the
        rank-ordered gather of every rank's q_local (row counts may differ); t2v_gts[i] = GT video ids
        (global) of gathered caption i; v2t_gts[v] = GT caption ids (gathered order) of global video v.
        Returns (t2v ranks [n_q] | None, v2t ranks [n_global] | None)."""
        q_all = all_gather_var(q_local, self.comm)
        return self._evaluate_gathered(q_all, self._pack(q_all, mode), t2v_gts, v2t_gts, mode)

    def _evaluate_gathered(self, q_all, q, t2v_gts, v2t_gts, mode: int):
        """evaluate() on captions already gathered (q_all) and packed (q)."""
        n_q = q_all.shape[0]
        row_csr = self.local_gt_csr(t2v_gts) if t2v_gts is not None else None
        col_csr = self.local_v2t_csr(v2t_gts) if v2t_gts is not None else None
        for _attempt in range(4):
            t2v, v2t, _, ovf = self.evaluate_device(q_all, row_csr, col_csr, n_q, mode, q=q)
            if not bool(ovf.item()):
                break
            self._grow()
        else:
            raise _lib.CmveError("ShardedGallery.evaluate: undecided-pair list kept overflowing")
        t2v_h = t2v.cpu().numpy().astype(np.int64) if t2v is not None else None
        v2t_h = None
        if v2t is not None:
            self._check_layout()
            v2t_h = all_gather_var(v2t, self.comm).cpu().numpy().astype(np.int64)
        return t2v_h, v2t_h

    def _check_layout(self):
        """Gathers in rank order must reproduce the global video order: shard r = [offset_r, offset_r + n_r),
        contiguous and increasing with r."""
        if self.world == 1:
            if self.offset != 0 or self.n != self.n_global:
                raise ValueError("ShardedGallery: a world-1 shard must hold the whole gallery")
            return
        t = torch.tensor([[self.offset, self.n]], dtype=torch.int64, device=self.device)
        lay = all_gather_rows(t, self.comm).cpu().numpy()
        ends = lay[:, 0] + lay[:, 1]
        if lay[0, 0] != 0 or ends[-1] != self.n_global or not np.array_equal(lay[1:, 0], ends[:-1]):
            raise ValueError(f"ShardedGallery: shards are not contiguous in rank order: {lay.tolist()}")

    def cal_perf(self, q_local: torch.Tensor, v2t_gt, t2v_gt, mode: int = _lib.SIM_F16):
        """``LINAS-engine/validate.py:15-54`` cal_perf over the sharded gallery: the reference's two
        6-tuples (v2t (r1, r5, r10, medr, meanr, mAP), t2v (...)) on every rank.  v2t_gt: list over the
        n_global videos of GT caption ids (gathered order); t2v_gt: dict or list over the captions of GT
        video ids (metrics.get_gt's outputs).  t2v mAP is the AP of each caption's FIRST GT
        (metrics.py:61-79); v2t mAP is over every GT caption of a video (metrics.py:83-102)."""
        # the captions are gathered and packed ONCE; every pass below (both directions, the first-GT t2v pass, the
        # v2t GT positions) reuses them
        q_all = all_gather_var(q_local, self.comm)
        n_q = q_all.shape[0]
        q = self._pack(q_all, mode)
        t2v_lists = [t2v_gt[i] for i in range(n_q)]  # KeyError on a caption without GT, like metrics.py:142
        v2t_lists = [v2t_gt[j] for j in range(self.n_global)]
        t2v, v2t = self._evaluate_gathered(q_all, q, t2v_lists, v2t_lists, mode)
        firsts = [[l[0]] for l in t2v_lists]
        if all(len(l) == 1 for l in t2v_lists):
            t2v_first = t2v
        else:
            t2v_first, _ = self._evaluate_gathered(q_all, q, firsts, None, mode)
        t2v_map = float(np.mean(1.0 / t2v_first))
        local = self.local_v2t_lists(v2t_lists)
        if all(len(l) <= 1 for l in v2t_lists):
            aps = [1.0 / v2t[self.offset + j] if local[j] else 0.0 for j in range(self.n)]
        else:
            aps = [ap_from_positions(p) for p in self._positions(q, local, mode)]
        s = torch.tensor([float(np.sum(aps))], dtype=torch.float64, device=self.device)
        v2t_map = float(reduce_counts(s, self.comm).item()) / self.n_global
        return (tuple(metrics_from_ranks(v2t)) + (v2t_map,), tuple(metrics_from_ranks(t2v)) + (t2v_map,))

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
        return merge_topk(idx, sc, k, self.comm)
