"""Device-side engine: packed embedding sets in HBM and the scoring / ranking calls.

PyTorch-ROCm provides device memory and streams only; every computation is a
libcmve.so (hand-written HIP, gfx950) call.  There is no CPU fallback: without a
GPU every entry point raises.
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes as C
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import lib, check, Rows

_HANDLES: Dict[Tuple[int, int], int] = {}

# Set by an atexit hook: objects still alive when the interpreter exits (a batch table, a captured graph held by a
# module or a test's traceback) skip their HIP destroy calls in __del__ -- the HIP runtime may already be torn down
# then, and the process releases the device memory anyway.
_EXITING = False


def _mark_exiting():
    global _EXITING
    _EXITING = True


atexit.register(_mark_exiting)


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("cmve needs a ROCm GPU (MI355X / gfx950); no CPU fallback exists")


def default_device() -> torch.device:
    require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


def handle(device: Optional[torch.device] = None) -> int:
    """cmve handle bound to the CURRENT torch stream of `device`."""
    device = device or default_device()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _handle_for(idx, torch.cuda.current_stream(idx).cuda_stream)


def stream_handle(device: torch.device, stream: "torch.cuda.Stream") -> int:
    """cmve handle bound to an explicit torch stream (no current-stream switch per call)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _handle_for(idx, stream.cuda_stream)


def _handle_for(idx: int, stream: int) -> int:
    key = (idx, stream)
    h = _HANDLES.get(key)
    if h is None:
        out = C.c_void_p()
        check(lib.cmve_create(idx, C.c_void_p(stream), C.byref(out)), "cmve_create")
        h = out.value
        _HANDLES[key] = h
    return h


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.CMVE_F32
    if t.dtype == torch.float64:
        return _lib.CMVE_F64
    raise TypeError(f"cmve: unsupported dtype {t.dtype} (float32 / float64 only)")


def pack_size(n: int, d: int) -> Tuple[int, int]:
    n_pad, d_pad = C.c_int64(), C.c_int64()
    check(lib.cmve_pack_size(n, d, C.byref(n_pad), C.byref(d_pad)), "cmve_pack_size")
    return n_pad.value, d_pad.value


def to_device(x, device: Optional[torch.device] = None, dtype=None) -> torch.Tensor:
    """numpy / torch -> contiguous float32|float64 device tensor (dtype preserved unless given)."""
    device = device or default_device()
    if isinstance(x, torch.Tensor):
        t = x.detach()
    else:
        t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    elif t.dtype in (torch.float16, torch.bfloat16):
        t = t.to(torch.float32)
    elif t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    return t.to(device, non_blocking=True).contiguous()


class RowSet:
    """A packed, L2-normalised embedding set resident in HBM (``cmve_rows_t``).

    ``eps=0`` reproduces LINAS ``l2norm`` (no epsilon, ``LINAS-engine/evaluation.py:10-14``);
    ``eps=1e-12`` reproduces ``F.normalize`` (``MultiFusion/src/combiner.py:134``).
    The raw rows are kept: the exact fp64 fix-up reads them.
    """

    def __init__(self, x, eps: float = 0.0, with_lo: bool = True, device: Optional[torch.device] = None,
                 with_f16: bool = True, raw_rows: bool = False):
        device = device or default_device()
        raw = to_device(x, device)
        if raw.dim() != 2:
            raise ValueError(f"RowSet expects a 2-D [n, d] matrix, got shape {tuple(raw.shape)}")
        n, d = raw.shape
        if d == 0:
            raise ValueError("RowSet: zero-dimensional embeddings")
        n_pad, d_pad = pack_size(n, d)
        self.device = device
        self.raw = raw
        self.n, self.d, self.n_pad, self.d_pad = n, d, n_pad, d_pad
        self.eps = float(eps)
        self.hi = torch.empty((n_pad, d_pad), dtype=torch.int16, device=device)
        self.lo = torch.empty((n_pad, d_pad), dtype=torch.int16, device=device) if with_lo else None
        self.inv_norm = torch.empty(n_pad, dtype=torch.float64, device=device)
        self.err_hi = torch.empty(n_pad, dtype=torch.float32, device=device)
        self.err_hilo = torch.empty(n_pad, dtype=torch.float32, device=device)
        self.h16 = torch.empty((n_pad, d_pad), dtype=torch.int16, device=device) if with_f16 else None
        self.err_h16 = torch.empty(n_pad, dtype=torch.float32, device=device) if with_f16 else None
        self.err_max = torch.empty(3, dtype=torch.float32, device=device)
        self.desc = Rows(n=n, d=d, n_pad=n_pad, d_pad=d_pad, hi=self.hi.data_ptr(),
                         lo=self.lo.data_ptr() if self.lo is not None else None,
                         raw=raw.data_ptr() if n else None, raw_dtype=_dtype_code(raw), flags=_lib.PACK_RAW if raw_rows else 0,
                         raw_ld=raw.stride(0) if n else d, inv_norm=self.inv_norm.data_ptr(),
                         err_hi=self.err_hi.data_ptr(), err_hilo=self.err_hilo.data_ptr(),
                         err_max=self.err_max.data_ptr(), eps=self.eps,
                         h16=self.h16.data_ptr() if with_f16 else None,
                         err_h16=self.err_h16.data_ptr() if with_f16 else None)
        check(lib.cmve_pack_rows(handle(device), C.byref(self.desc)), "cmve_pack_rows")

    def repack(self, x):
        """Copy new rows of the SAME shape into the resident raw buffer and re-pack them in place
        (query batches re-scored against a resident gallery: no allocation per call)."""
        src = x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(x))
        if tuple(src.shape) != tuple(self.raw.shape):
            raise ValueError(f"RowSet.repack: expected {tuple(self.raw.shape)}, got {tuple(src.shape)}")
        self.raw.copy_(src, non_blocking=True)
        check(lib.cmve_pack_rows(handle(self.device), C.byref(self.desc)), "cmve_pack_rows")
        return self

    @property
    def has_lo(self):
        return self.lo is not None

    @property
    def has_f16(self):
        return self.h16 is not None

    def normalized(self, dtype=torch.float64) -> torch.Tensor:
        """x / max(||x||, eps) on device (K1')."""
        out = torch.empty((self.n, self.d), dtype=dtype, device=self.device)
        if self.n:
            check(lib.cmve_l2norm_rows(handle(self.device), _ptr(self.raw), _dtype_code(self.raw), self.raw.stride(0),
                                       _ptr(out), _dtype_code(out), out.stride(0), self.n, self.d, self.eps),
                  "cmve_l2norm_rows")
        return out


class PackedOperand:
    """Split-bf16 planes of a raw GEMM operand [n, d] written by a fused kernel (cmve_pack_tblocks,
    cmve_layernorm_pack) instead of cmve_pack_rows: usable wherever cmve_linear takes a RowSet
    packed with raw_rows=True (no fp32 rows behind it, no score bound)."""

    def __init__(self, n: int, d: int, device: Optional[torch.device] = None, row_multiple: int = 1):
        device = device or default_device()
        n_pad, d_pad = pack_size(n, d)
        n_pad = -(-n_pad // row_multiple) * row_multiple
        self.device, self.n, self.d, self.n_pad, self.d_pad = device, n, d, n_pad, d_pad
        self.hi = torch.empty((n_pad, d_pad), dtype=torch.int16, device=device)
        self.lo = torch.empty((n_pad, d_pad), dtype=torch.int16, device=device)
        self.err_max = torch.empty(3, dtype=torch.float32, device=device)
        self.desc = Rows(n=n, d=d, n_pad=n_pad, d_pad=d_pad, hi=self.hi.data_ptr(), lo=self.lo.data_ptr(), raw=None,
                         raw_dtype=_lib.CMVE_F32, flags=_lib.PACK_RAW, raw_ld=d, err_max=self.err_max.data_ptr())

    has_lo = True
    has_f16 = False

    @classmethod
    def from_blocks_transposed(cls, x: torch.Tensor, block_rows: int, block_cols: int):
        """Operand rows (b, c) = column c of block b of x viewed as [nb][block_rows][block_cols]
        (fp32): each row has block_rows elements (cmve_pack_tblocks)."""
        x = x.detach().float().contiguous()
        nb = x.numel() // (block_rows * block_cols)
        op = cls(nb * block_cols, block_rows, x.device, row_multiple=block_cols)
        check(lib.cmve_pack_tblocks(handle(x.device), _ptr(x), nb, block_rows, block_cols, C.byref(op.desc)),
              "cmve_pack_tblocks")
        return op

    @classmethod
    def layernorm(cls, x: torch.Tensor, weight, bias, eps: float):
        """LayerNorm(x) rows (fp64 statistics, cmve_layernorm's arithmetic) as a packed operand."""
        x = x.detach().float().contiguous()
        n, d = x.shape
        op = cls(n, d, x.device)
        w = weight.detach().float().contiguous() if weight is not None else None
        b = bias.detach().float().contiguous() if bias is not None else None
        check(lib.cmve_layernorm_pack(handle(x.device), _ptr(x), x.stride(0), n, d, _ptr(w), _ptr(b), float(eps),
                                      C.byref(op.desc)), "cmve_layernorm_pack")
        return op


def transpose_blocks_kv(x: torch.Tensor, block_rows: int, block_cols: int, d: int, T: int, gs: int,
                        B: int) -> torch.Tensor:
    """transpose_blocks whose output rows of d floats (g, t, bb) of .reshape(B // gs, T, gs, d) are
    stored at row t*B + g*gs + bb (cmve_transpose_blocks_kv): [T * B, d]."""
    x = x.detach().float().contiguous()
    nb = x.numel() // (block_rows * block_cols)
    y = torch.empty((T * B, d), dtype=torch.float32, device=x.device)
    check(lib.cmve_transpose_blocks_kv(handle(x.device), _ptr(x), nb, block_rows, block_cols, d, T, gs, B, _ptr(y)),
          "cmve_transpose_blocks_kv")
    return y


def transpose_blocks(x: torch.Tensor, block_rows: int, block_cols: int) -> torch.Tensor:
    """y[(b, c), :] = column c of block b of x viewed as [nb][block_rows][block_cols] (fp32)."""
    x = x.detach().float().contiguous()
    nb = x.numel() // (block_rows * block_cols)
    y = torch.empty((nb * block_cols, block_rows), dtype=torch.float32, device=x.device)
    check(lib.cmve_transpose_blocks(handle(x.device), _ptr(x), nb, block_rows, block_cols, _ptr(y)),
          "cmve_transpose_blocks")
    return y


def _mode_for(q: RowSet, g: RowSet, mode: Optional[int]) -> int:
    if mode is None:
        mode = _lib.SIM_BF16X3 if (q.has_lo and g.has_lo) else _lib.SIM_BF16
    if mode == _lib.SIM_BF16X3 and not (q.has_lo and g.has_lo):
        raise ValueError("BF16X3 mode needs both sets packed with lo planes")
    return mode


def sim_store(q: RowSet, g: RowSet, alpha: float = 1.0, beta: float = 0.0, mode: Optional[int] = None,
              out_dtype=torch.float32) -> torch.Tensor:
    """out[i, j] = alpha * cos(q_i, g_j) + beta on device."""
    mode = _mode_for(q, g, mode)
    out = torch.empty((q.n, g.n), dtype=out_dtype, device=q.device)
    if q.n and g.n:
        check(lib.cmve_sim_store(handle(q.device), C.byref(q.desc), C.byref(g.desc), mode, alpha, beta, _ptr(out),
                                 _dtype_code(out), out.stride(0)), "cmve_sim_store")
    return out


def pairwise(a: torch.Tensor, b: torch.Tensor, metric: int, alpha: float = 1.0, beta: float = 0.0,
             out_dtype=torch.float64) -> torch.Tensor:
    """out[i, j] = alpha * f(a_i, b_j) + beta for a non-cosine metric (K10, fp64 accumulation)."""
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"pairwise: shapes {tuple(a.shape)} and {tuple(b.shape)} do not match")
    # row-strided views go in as they are (lda >= D); anything else is made contiguous
    a = a if a.stride(1) == 1 and a.stride(0) >= a.shape[1] else a.contiguous()
    b = b if b.stride(1) == 1 and b.stride(0) >= b.shape[1] else b.contiguous()
    out = torch.empty((a.shape[0], b.shape[0]), dtype=out_dtype, device=a.device)
    if a.shape[0] and b.shape[0]:
        check(lib.cmve_pairwise(handle(a.device), _ptr(a), _dtype_code(a), a.stride(0), a.shape[0], _ptr(b),
                                _dtype_code(b), b.stride(0), b.shape[0], a.shape[1], metric, float(alpha),
                                float(beta), _ptr(out), _dtype_code(out), out.stride(0)), "cmve_pairwise")
    return out


def csr(lists: Sequence[Sequence[int]], device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Python GT lists -> (offsets int64 [n+1], indices int32) device tensors."""
    lens = np.fromiter((len(l) for l in lists), dtype=np.int64, count=len(lists))
    off = np.zeros(len(lists) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    idx = np.fromiter((int(v) for l in lists for v in l), dtype=np.int32, count=int(off[-1]))
    if idx.size == 0:
        idx = np.zeros(1, np.int32)
    return (torch.from_numpy(off).to(device), torch.from_numpy(idx).to(device))


def gt_thresholds(a: RowSet, b: RowSet, off: torch.Tensor, idx: torch.Tensor, mode: int):
    sgt = torch.empty(a.n_pad, dtype=torch.float64, device=a.device)
    hi = torch.empty(a.n_pad, dtype=torch.float32, device=a.device)
    lo = torch.empty(a.n_pad, dtype=torch.float32, device=a.device)
    check(lib.cmve_gt_thresholds(handle(a.device), C.byref(a.desc), C.byref(b.desc), mode, _ptr(off), _ptr(idx),
                                 _ptr(sgt), _ptr(hi), _ptr(lo)), "cmve_gt_thresholds")
    return sgt, hi, lo


class RankWorkspace:
    """Reusable device buffers for rank_count: the undecided-pair list (grown on overflow) and
    one int64 pair counter per gallery chunk (cmve_rank_count_overlap)."""

    def __init__(self, device, cap: int = 1 << 20):
        self.device = device
        self.cand = torch.empty(max(cap, 1), dtype=torch.int64, device=device)
        self.count = torch.zeros(_lib.MAX_CHUNKS, dtype=torch.int64, device=device)
        self.chunks = 1

    @property
    def cap(self):
        return self.cand.numel()

    def ncand(self) -> int:
        """Undecided pairs of the last launch (synchronises)."""
        return int(self.count[:self.chunks].sum().item())

    def overflowed(self) -> bool:
        """True if a chunk's list outgrew its share of the buffer (counts incomplete)."""
        return bool((self.count[:self.chunks] > self.cap // self.chunks).any().item())

    def grow(self, need: int = 0):
        need = max(need, self.ncand())
        self.cand = torch.empty(int(need * 1.25) * self.chunks + 1024 * self.chunks, dtype=torch.int64,
                                device=self.device)


def rank_thresholds(a: RowSet, b: RowSet, sgt: torch.Tensor, mode: int):
    """fp32 bracketing thresholds for given exact GT scores sgt[a.n_pad] (NaN = no GT)."""
    hi = torch.empty(a.n_pad, dtype=torch.float32, device=a.device)
    lo = torch.empty(a.n_pad, dtype=torch.float32, device=a.device)
    check(lib.cmve_rank_thresholds(handle(a.device), C.byref(a.desc), C.byref(b.desc), mode, _ptr(sgt), _ptr(hi),
                                   _ptr(lo)), "cmve_rank_thresholds")
    return hi, lo


def rank_count_launch(q: RowSet, g: RowSet, mode: int, row=None, col=None, ws: Optional[RankWorkspace] = None,
                      row_cnt=None, col_cnt=None, events=None, chunks: int = 1):
    """Enqueue the fused rank count (no sync).  row/col = (sgt, thr_hi, thr_lo) or None.
    chunks > 1: cmve_rank_count_overlap -- the gallery in `chunks` pieces, each piece's fp64
    fix-up on the handle's auxiliary stream behind the next piece's MFMA pass.
    events = (start, mid, end) torch.cuda.Event triple recorded around the MFMA pass and the
    fix-up (with chunks > 1 the two overlap: mid is recorded with end)."""
    dirs = (_lib.DIR_ROW if row is not None else 0) | (_lib.DIR_COL if col is not None else 0)
    if row is not None and row_cnt is None:
        row_cnt = torch.empty(q.n_pad, dtype=torch.int32, device=q.device)
    if col is not None and col_cnt is None:
        col_cnt = torch.empty(g.n_pad, dtype=torch.int32, device=q.device)
    r = row if row is not None else (None, None, None)
    c = col if col is not None else (None, None, None)
    h = handle(q.device)
    chunks = max(1, min(int(chunks), _lib.MAX_CHUNKS))
    ws.chunks = chunks
    if events is not None:
        events[0].record()
    if chunks > 1:
        check(lib.cmve_rank_count_overlap(h, C.byref(q.desc), C.byref(g.desc), mode, dirs, _ptr(r[0]), _ptr(r[1]),
                                          _ptr(r[2]), _ptr(c[0]), _ptr(c[1]), _ptr(c[2]), _ptr(row_cnt),
                                          _ptr(col_cnt), _ptr(ws.cand), ws.cap, _ptr(ws.count), chunks),
              "cmve_rank_count_overlap")
        if events is not None:
            events[1].record()
            events[2].record()
        return row_cnt, col_cnt
    check(lib.cmve_rank_mfma(h, C.byref(q.desc), C.byref(g.desc), mode, dirs, _ptr(r[1]), _ptr(r[2]), _ptr(c[1]),
                             _ptr(c[2]), _ptr(row_cnt), _ptr(col_cnt), _ptr(ws.cand), ws.cap, _ptr(ws.count)),
          "cmve_rank_mfma")
    if events is not None:
        events[1].record()
    check(lib.cmve_rank_fixup(h, C.byref(q.desc), C.byref(g.desc), dirs, _ptr(r[0]), _ptr(c[0]), _ptr(row_cnt),
                              _ptr(col_cnt), _ptr(ws.cand), ws.cap, _ptr(ws.count)), "cmve_rank_fixup")
    if events is not None:
        events[2].record()
    return row_cnt, col_cnt


def gt_rank_counts(q: RowSet, g: RowSet, row_gts=None, col_gts=None, mode: int = _lib.SIM_F16,
                   ws: Optional[RankWorkspace] = None, chunks: int = 1):
    """Exact GT ranks in both directions from ONE fused GEMM pass.

    row_gts[i]: GT indices into g for query row i (t2v); col_gts[j]: GT indices into q
    for gallery row j (v2t).  Returns (row_ranks, col_ranks, n_candidates) as numpy int64,
    1-based; empty GT lists give n_other + 1 (``LINAS-engine/util/metrics.py:140``).
    """
    if row_gts is None and col_gts is None:
        raise ValueError("gt_rank_counts: need row_gts and/or col_gts")
    if mode == _lib.SIM_BF16X3 and not (q.has_lo and g.has_lo):
        raise ValueError("BF16X3 needs lo planes")
    if mode == _lib.SIM_F16 and not (q.has_f16 and g.has_f16):
        mode = _lib.SIM_BF16
    ws = ws or RankWorkspace(q.device, cap=max(1 << 16, 64 * (q.n + g.n)))
    row = col = None
    if row_gts is not None:
        roff, ridx = csr(row_gts, q.device)
        row = gt_thresholds(q, g, roff, ridx, mode)
    if col_gts is not None:
        coff, cidx = csr(col_gts, q.device)
        col = gt_thresholds(g, q, coff, cidx, mode)
    for _attempt in range(4):
        rc, cc = rank_count_launch(q, g, mode, row, col, ws, chunks=chunks)
        ncand = ws.ncand()  # synchronises
        if not ws.overflowed():
            break
        ws.grow(ncand)
    else:
        raise _lib.CmveError("rank_count: candidate list kept overflowing")
    out_r = gt_ranks(rc, row[0], q.n, g.n).cpu().numpy() if row_gts is not None else None
    out_c = gt_ranks(cc, col[0], g.n, q.n).cpu().numpy() if col_gts is not None else None
    return out_r, out_c, ncand


def gt_ranks(cnt: torch.Tensor, sgt: torch.Tensor, n: int, n_m: int, out: Optional[torch.Tensor] = None,
             recall: Optional[torch.Tensor] = None) -> torch.Tensor:
    """1-based ranks int64 [n] on the device from better-than-GT counts and GT scores (cmve_gt_ranks):
    empty GT list (sgt NaN) -> n_m + 1, every GT NaN (sgt +inf) -> n_m, else count + 1
    (``LINAS-engine/util/metrics.py:137-147``).  recall: optional int64 [4] device output
    (#rank<=1, #rank<=5, #rank<=10, sum of ranks)."""
    if out is None:
        out = torch.empty(max(n, 1), dtype=torch.int64, device=cnt.device)
    check(lib.cmve_gt_ranks(handle(cnt.device), _ptr(cnt), _ptr(sgt), n, n_m, _ptr(out), _ptr(recall)),
          "cmve_gt_ranks")
    return out[:n]


class RankSession:
    """Resident exact GT-rank evaluation of a fixed problem (the reference re-runs
    ``encode_* -> cal_error -> cal_perf`` on new embeddings of the same sets every validation,
    ``LINAS-engine/validate.py:61-74``): the packed planes of both sets, the GT lists, thresholds,
    counts and the undecided-pair list are allocated once, and one evaluation is FOUR launches on
    the session's stream (``cmve_eval_ranks``, K14): pack both sets + exact GT scores, the fused rank
    GEMM (thresholds derived in-kernel), the fp64 fix-up, ranks + R@K sums.
    ``run(captions, videos)`` returns (t2v ranks, v2t ranks) exactly as ``gt_rank_counts`` does.
    Device tensors of the session's dtype are read in place (no copy); anything else is copied into
    the session's own buffers first.  An undecided-pair overflow grows the list and redoes the run.
    ``enqueue`` + ``stats`` is the non-blocking form (R@K sums / overflow on the device)."""

    def __init__(self, n_q: int, n_g: int, d: int, row_gts=None, col_gts=None, dtype=torch.float32,
                 mode: int = _lib.SIM_F16, eps: float = 0.0, device: Optional[torch.device] = None,
                 cand_cap: Optional[int] = None, stream: Optional["torch.cuda.Stream"] = None):
        if row_gts is None and col_gts is None:
            raise ValueError("RankSession: need row_gts and/or col_gts")
        if n_q < 1 or n_g < 1:
            raise ValueError("RankSession: both sets need rows")
        self.device = device or default_device()
        dev = self.device
        self.mode, self.dtype = mode, dtype
        self.q = RowSet(torch.zeros((n_q, d), dtype=dtype, device=dev), eps=eps, with_lo=(mode == _lib.SIM_BF16X3),
                        with_f16=(mode == _lib.SIM_F16), device=dev)
        self.g = RowSet(torch.zeros((n_g, d), dtype=dtype, device=dev), eps=eps, with_lo=(mode == _lib.SIM_BF16X3),
                        with_f16=(mode == _lib.SIM_F16), device=dev)
        self.row = csr(row_gts, dev) if row_gts is not None else None
        self.col = csr(col_gts, dev) if col_gts is not None else None
        # a one-to-one GT pairing (MSR-VTT-1kA: caption i <-> video p(i)) lets the evaluation's prep pack and
        # score each (caption, video) pair in one wave (CMVE_EVAL_PAIRED)
        self.paired = self._is_pairing(row_gts, col_gts, n_q, n_g)
        self._alloc(int(cand_cap) if cand_cap else max(1 << 16, 64 * (n_q + n_g)))
        self.out = torch.zeros(_lib.EVAL_OUT_HEAD + n_q + n_g, dtype=torch.int64, device=dev)
        self.host = torch.zeros(_lib.EVAL_OUT_HEAD + n_q + n_g, dtype=torch.int64).pin_memory()
        self._bound = (None, None)
        # stream: the session's own HIP stream (every launch and copy of the session goes there, with no
        # current-stream switch per evaluation: ~6 us of host time each); None = the caller's current stream
        self.stream = stream
        self._h = stream_handle(dev, stream) if stream is not None else None

    @staticmethod
    def _is_pairing(row_gts, col_gts, n_q, n_g) -> bool:
        if row_gts is None or col_gts is None or n_q != n_g:
            return False
        rows = [row_gts[i] for i in range(n_q)]
        cols = [col_gts[j] for j in range(n_g)]
        if any(len(l) != 1 for l in rows) or any(len(l) != 1 for l in cols):
            return False
        return all(0 <= int(rows[i][0]) < n_g and int(cols[int(rows[i][0])][0]) == i for i in range(n_q))

    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _alloc(self, cap: int):
        nbytes = C.c_int64()
        check(lib.cmve_eval_workspace(C.byref(self.q.desc), C.byref(self.g.desc), int(cap), C.byref(nbytes)),
              "cmve_eval_workspace")
        self.ws = torch.zeros(nbytes.value, dtype=torch.uint8, device=self.device)  # zeroed once (ABI contract)
        self.cap = int(cap)
        self._args = None
        # captured graphs bake the workspace address in: a new workspace makes them stale (EvalGraph.launch
        # refuses them), and each graph keeps the workspace it was captured with alive
        self._ws_gen = getattr(self, "_ws_gen", -1) + 1

    @property
    def ncand(self) -> int:
        """Undecided pairs of the last evaluation written into ``self.out`` (synchronises)."""
        return int(self.out[8].item())

    def _bind(self, rs: RowSet, x):
        """Point the packed set's raw rows at x (a device tensor of the session dtype, rows contiguous),
        or copy x into the set's own buffer."""
        if (torch.is_tensor(x) and x.device == self.device and x.dtype == self.dtype and x.dim() == 2
                and tuple(x.shape) == tuple(rs.raw.shape) and x.stride(1) == 1 and x.stride(0) >= x.shape[1]):
            src = x
        else:
            src_t = x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(x))
            if tuple(src_t.shape) != tuple(rs.raw.shape):
                raise ValueError(f"RankSession: expected {tuple(rs.raw.shape)}, got {tuple(src_t.shape)}")
            rs.raw.copy_(src_t, non_blocking=True)
            src = rs.raw
        rs.desc.raw = src.data_ptr()
        rs.desc.raw_ld = src.stride(0)
        return src

    def enqueue(self, captions, videos, timing_slot: int = -1, out: Optional[torch.Tensor] = None,
                _bind_only: bool = False, wait_current: bool = True):
        """Enqueue one evaluation (no host synchronisation) on the session's stream, or on the current
        stream without one.  The inputs must stay unmodified until it completes.  With a session stream the
        evaluation first waits for the work already enqueued on the caller's current stream (the producer of
        the embeddings, e.g. an encoder), and inputs read in place are recorded on the session stream for
        the caching allocator; ``wait_current=False`` skips the wait for callers whose inputs are known to
        be complete (a resident buffer the caller synchronised once).  out: optional int64 device tensor of
        ``EVAL_OUT_HEAD + n_q + n_g`` words receiving this evaluation's head + ranks instead of
        ``self.out`` (a ring of them lets pipelined evaluations be read back in batches)."""
        if out is None:
            out = self.out
        elif (out.dtype != torch.int64 or out.device != self.out.device or not out.is_contiguous()
              or out.numel() < self.out.numel()):
            raise ValueError(f"RankSession.enqueue: out must be a contiguous int64 {self.out.device} tensor of "
                             f">= {self.out.numel()} words")
        if not (self._bound[0] is captions and self._bound[1] is videos and self._args is not None
                and captions.data_ptr() == self.q.desc.raw and videos.data_ptr() == self.g.desc.raw):
            # (re)bind: the same input tensors again (a resident buffer refilled between evaluations)
            # reuse the bound descriptors and the prepared argument tuple -- the host side of an
            # evaluation is then one ctypes call
            if self.stream is not None and wait_current:
                self._order_after_current()
                wait_current = False
            with self._ctx():  # a copying bind goes on the session's stream
                self._bound = (self._bind(self.q, captions), self._bind(self.g, videos))
            if self.stream is not None:  # read in place on another stream: keep the allocator from reusing them early
                for x, b in zip((captions, videos), self._bound):
                    if torch.is_tensor(x) and b is x:
                        x.record_stream(self.stream)
            if self._bound[0] is not captions or self._bound[1] is not videos:
                self._bound = (None, None)  # copied into the session's own buffers: rebind next time
            r = self.row if self.row is not None else (None, None)
            c = self.col if self.col is not None else (None, None)
            mode = self.mode | (_lib.EVAL_PAIRED if self.paired else 0)
            self._args = (C.byref(self.q.desc), C.byref(self.g.desc), mode, _ptr(r[0]), _ptr(r[1]), _ptr(c[0]),
                          _ptr(c[1]), _ptr(self.ws), self.ws.numel(), self.cap)
        if _bind_only:
            return
        if self.stream is not None and wait_current:
            self._order_after_current()
        h = self._h if self._h is not None else handle(self.device)
        check(lib.cmve_eval_ranks(h, *self._args, _ptr(out), int(timing_slot)), "cmve_eval_ranks")

    def _order_after_current(self):
        """The session stream waits for the work enqueued so far on the caller's current stream."""
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream != self.stream.cuda_stream:
            self.stream.wait_stream(cur)

    def graph(self, captions, videos, out: Optional[torch.Tensor] = None) -> "EvalGraph":
        """One evaluation of these inputs into `out` (default self.out) captured into a HIP graph on the
        session's stream (cmve_eval_graph_create): ``launch()`` replays it with one host call, same results
        bit for bit.  Every address is baked in: the inputs must be device tensors of the session dtype read
        in place (refill them between launches), and `out` stays where it is."""
        for x in (captions, videos):
            if not (torch.is_tensor(x) and x.device == self.device and x.dtype == self.dtype):
                raise ValueError("RankSession.graph: inputs must be device tensors of the session dtype")
        self.enqueue(captions, videos, out=out, _bind_only=True)
        if self._bound[0] is not captions or self._bound[1] is not videos:
            raise ValueError("RankSession.graph: inputs must be readable in place (rows contiguous)")
        out = self.out if out is None else out
        h = self._h if self._h is not None else handle(self.device)
        gh = C.c_void_p()
        check(lib.cmve_eval_graph_create(h, *self._args, _ptr(out), C.byref(gh)), "cmve_eval_graph_create")
        return EvalGraph(gh.value, h, (captions, videos, out, self, self.ws), self, self._ws_gen)

    def timing(self, slot: int):
        """(pack+thresholds, rank GEMM, fix-up+ranks) milliseconds of the evaluation that used `slot`."""
        ms = (C.c_float * 3)()
        h = self._h if self._h is not None else handle(self.device)
        check(lib.cmve_eval_timing(h, int(slot), ms), "cmve_eval_timing")
        return list(ms)

    def kernel_timing(self, slot: int):
        """(prep, rank GEMM, fix-up, finish) kernel durations in ms of the evaluation that used `slot`, each
        from its launch's own start / stop (the durations rocprofv3 reports)."""
        ms = (C.c_float * 4)()
        h = self._h if self._h is not None else handle(self.device)
        check(lib.cmve_eval_kernel_timing(h, int(slot), ms), "cmve_eval_kernel_timing")
        return list(ms)

    def run(self, captions, videos):
        """Exact 1-based (t2v ranks, v2t ranks) of new caption / video embeddings (numpy or torch)."""
        for _attempt in range(4):
            self.enqueue(captions, videos)
            with self._ctx():
                self.host.copy_(self.out, non_blocking=True)
                torch.cuda.current_stream(self.device).synchronize()
            need = int(self.host[9])
            if int(self.host[11]):  # (the paired prep's per-caption check of CMVE_EVAL_PAIRED)
                raise _lib.CmveError("RankSession: the GT lists are not a one-to-one pairing")
            if need == 0:
                break
            self._alloc(max(need, 2 * self.cap))  # a bucket overflowed: the counts are incomplete
        else:
            raise _lib.CmveError("RankSession: undecided-pair list kept overflowing")
        h = self.host.numpy()
        nq, ng, o = self.q.n, self.g.n, _lib.EVAL_OUT_HEAD
        t2v = h[o:o + nq].copy() if self.row is not None else None
        v2t = h[o + nq:o + nq + ng].copy() if self.col is not None else None
        return t2v, v2t


class RankBatch:
    """A batch of same-shaped RankSession evaluations (cmve_eval_batch_*: one prep, one rank GEMM and one
    finish launch over all of them).  ``sessions`` share sizes, dtype, mode and GT lists (each keeps its own
    packed sets, workspace and output); ``inputs`` holds one (captions, videos) pair of device tensors of the
    session dtype per session, read in place (refill them between runs: every address is baked in, as for
    RankSession.graph); ``outs`` optionally one int64 output per session (default each session's ``out``).
    ``run()`` enqueues the batch on ``stream`` (default the current stream); the results equal each session's
    own ``enqueue`` bit for bit.  Sizes must take the G64 rank geometry (e.g. MSR-VTT-1kA's 1,000 x 1,000)."""

    def __init__(self, sessions, inputs, outs=None, stream: Optional["torch.cuda.Stream"] = None):
        sessions = list(sessions)
        if not sessions or len(inputs) != len(sessions):
            raise ValueError("RankBatch: one (captions, videos) input pair per session")
        s0 = sessions[0]
        for s in sessions[1:]:
            same_lists = all((a is None) == (b is None) and (a is None or all(torch.equal(x, y) for x, y in zip(a, b)))
                             for a, b in ((s0.row, s.row), (s0.col, s.col)))
            if (s.q.n, s.g.n, s.q.d, s.dtype, s.mode, s.paired) != (s0.q.n, s0.g.n, s0.q.d, s0.dtype, s0.mode,
                                                                   s0.paired) or not same_lists:
                raise ValueError("RankBatch: sessions must share sizes, dtype, mode and GT lists")
        # one undecided-pair capacity for the whole batch (the C table holds one cand_cap and workspace size): a
        # session whose list was grown sets it, the others are grown to it here, before any input is bound
        cap = max(s.cap for s in sessions)
        for s in sessions:
            if s.cap != cap:
                s._alloc(cap)
        outs = [s.out for s in sessions] if outs is None else list(outs)
        for s, o in zip(sessions, outs):
            if o.dtype != torch.int64 or not o.is_contiguous() or o.numel() < s.out.numel():
                raise ValueError("RankBatch: outs must be contiguous int64 tensors of EVAL_OUT_HEAD + n_q + n_g words")
        for s, (c, v) in zip(sessions, inputs):
            for x in (c, v):
                if not (torch.is_tensor(x) and x.device == s.device and x.dtype == s.dtype):
                    raise ValueError("RankBatch: inputs must be device tensors of the session dtype")
            s.enqueue(c, v, _bind_only=True)
            if s._bound[0] is not c or s._bound[1] is not v:
                raise ValueError("RankBatch: inputs must be readable in place (rows contiguous)")
        n = len(sessions)
        self._q = (C.POINTER(Rows) * n)(*[C.pointer(s.q.desc) for s in sessions])
        self._g = (C.POINTER(Rows) * n)(*[C.pointer(s.g.desc) for s in sessions])
        self._ws = (C.c_void_p * n)(*[s.ws.data_ptr() for s in sessions])
        self._out = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
        ws_bytes = sessions[0].ws.numel()
        if any(s.cap != cap or s.ws.numel() != ws_bytes for s in sessions):
            raise ValueError("RankBatch: sessions must share one undecided-pair capacity and workspace size")
        r = s0.row if s0.row is not None else (None, None)
        c = s0.col if s0.col is not None else (None, None)
        mode = s0.mode | (_lib.EVAL_PAIRED if s0.paired else 0)
        bh = C.c_void_p()
        check(lib.cmve_eval_batch_create(n, self._q, self._g, mode, _ptr(r[0]), _ptr(r[1]), _ptr(c[0]), _ptr(c[1]),
                                         self._ws, ws_bytes, cap, self._out, C.byref(bh)), "cmve_eval_batch_create")
        self._b = bh.value
        self._keep = (sessions, [tuple(x) for x in inputs], outs)  # everything the table points at stays alive
        self._ws_gens = [s._ws_gen for s in sessions]
        self.sessions, self.outs, self.stream = sessions, outs, stream
        self._h = stream_handle(s0.device, stream) if stream is not None else None

    def run(self, timing_slot: int = -1, wait_current: bool = True):
        """Enqueue the batch; ``timing_slot`` >= 0 records its launches' durations in that slot of the stream
        handle's timing ring (``kernel_timing``).  With a batch stream the run first waits for the work already
        enqueued on the caller's current stream (the producer that refilled the inputs, as RankSession.enqueue
        does); ``wait_current=False`` skips that for inputs known to be complete."""
        if not self._b:
            raise RuntimeError("RankBatch.run: the batch was closed")
        if any(s._ws_gen != g for s, g in zip(self.sessions, self._ws_gens)):
            raise RuntimeError("RankBatch.run: a session's workspace was regrown after the batch was built")
        if self.stream is not None and wait_current:
            cur = torch.cuda.current_stream(self.sessions[0].device)
            if cur.cuda_stream != self.stream.cuda_stream:
                self.stream.wait_stream(cur)
        h = self._h if self._h is not None else handle(self.sessions[0].device)
        check(lib.cmve_eval_batch_run(h, self._b, int(timing_slot)), "cmve_eval_batch_run")

    def run_chained(self, prev: Optional["RankBatch"] = None, timing_slot: int = -1, wait_current: bool = True):
        """Enqueue the batch with its finish (the words of its outputs: ranks, R@K) deferred to the next chained run on
        the same stream, whose first launch holds it beside that run's prep (``cmve_eval_batch_run_chained``); ``prev``
        is the batch chained before this one on the stream (its outputs are complete once this run's first launch
        has run), None for the first.  After a stream's last chained run call ``finish()``.  ``prev`` must share no
        session with this batch."""
        if not self._b or (prev is not None and not prev._b):
            raise RuntimeError("RankBatch.run_chained: a batch was closed")
        if any(s._ws_gen != g for s, g in zip(self.sessions, self._ws_gens)):
            raise RuntimeError("RankBatch.run_chained: a session's workspace was regrown after the batch was built")
        if self.stream is not None and wait_current:
            cur = torch.cuda.current_stream(self.sessions[0].device)
            if cur.cuda_stream != self.stream.cuda_stream:
                self.stream.wait_stream(cur)
        h = self._h if self._h is not None else handle(self.sessions[0].device)
        check(lib.cmve_eval_batch_run_chained(h, self._b, prev._b if prev is not None else None, int(timing_slot)),
              "cmve_eval_batch_run_chained")

    def finish(self):
        """The deferred finish of this batch's last chained run, alone (``cmve_eval_batch_finish``)."""
        if not self._b:
            raise RuntimeError("RankBatch.finish: the batch was closed")
        h = self._h if self._h is not None else handle(self.sessions[0].device)
        check(lib.cmve_eval_batch_finish(h, self._b), "cmve_eval_batch_finish")

    def kernel_timing(self, slot: int):
        """(prep, rank GEMM, 0, finish) durations in ms of the batch run that used `slot` (each launch's own
        start / stop: the whole batch's launches; a chained run: the prep launch holds the previous batch's finish,
        and finish is 0)."""
        ms = (C.c_float * 4)()
        h = self._h if self._h is not None else handle(self.sessions[0].device)
        check(lib.cmve_eval_kernel_timing(h, int(slot), ms), "cmve_eval_kernel_timing")
        return list(ms)

    def close(self):
        if self._b:
            if not _EXITING:  # (past interpreter exit the HIP runtime may be gone: the process releases the table)
                lib.cmve_eval_batch_destroy(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter teardown)
            pass


class EvalGraph:
    """A captured RankSession evaluation (cmve_eval_graph_*): ``launch()`` enqueues it on the session's
    stream with one host call.  Keeps its inputs, output and session alive."""

    def __init__(self, gh: int, h: int, keep, session: Optional["RankSession"] = None, ws_gen: int = 0):
        self._g, self._h, self._keep = gh, h, keep  # keep: inputs, output, session and the captured workspace
        self._session, self._ws_gen = session, ws_gen

    @property
    def stale(self) -> bool:
        """True once the session replaced its workspace (an overflow in run()): the graph's baked-in
        undecided-pair list is no longer the session's, and its capacity is the one that overflowed."""
        return self._session is not None and self._session._ws_gen != self._ws_gen

    def launch(self):
        if not self._g:
            raise RuntimeError("EvalGraph.launch: the graph was closed")
        if self.stale:
            raise RuntimeError("EvalGraph.launch: the session's workspace was regrown after this graph was "
                               "captured; capture a new graph (RankSession.graph)")
        check(lib.cmve_eval_graph_launch(self._h, self._g), "cmve_eval_graph_launch")

    def close(self):
        if self._g:
            if not _EXITING:
                lib.cmve_eval_graph_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


def rank_from_matrix(errors, gts, transposed: bool = False, device=None) -> np.ndarray:
    """1-based GT ranks from a materialised error matrix (lower = better), on device."""
    device = device or default_device()
    e = to_device(errors, device)
    n_rows, n_cols = e.shape
    n_q = n_cols if transposed else n_rows
    lists = [gts[i] if (not isinstance(gts, dict) or i in gts) else [] for i in range(n_q)]
    off, idx = csr(lists, device)
    cnt = torch.zeros(n_q, dtype=torch.int32, device=device)
    check(lib.cmve_rank_from_matrix(handle(device), _ptr(e), _dtype_code(e), n_rows, n_cols, e.stride(0),
                                    1 if transposed else 0, _ptr(off), _ptr(idx), _ptr(cnt)),
          "cmve_rank_from_matrix")
    ranks = cnt.to(torch.int64).cpu().numpy() + 1
    n_m = n_rows if transposed else n_cols
    empty = np.fromiter((len(l) == 0 for l in lists), bool, count=n_q)
    ranks[empty] = n_m + 1
    return ranks


def topk_workspace_floats(q: RowSet, g: RowSet, k: int) -> int:
    """Floats of device workspace cmve_topk needs for this query set / gallery / k."""
    n = C.c_int64()
    check(lib.cmve_topk_workspace(C.byref(q.desc), C.byref(g.desc), int(k), C.byref(n)), "cmve_topk_workspace")
    return n.value


TOPK_BATCH_MIN_Q = 512   # below this the dense score block is small: cmve_topk
TOPK_BATCH_MAX_K = 32     # cmve_topk_batch's limit (its sample is ~k/128 of the gallery)


def topk_batch_plan(q: RowSet, g: RowSet, k: int):
    """(use_batch, sample_rows, workspace_floats) of cmve_topk_batch for this problem: the fused
    path pays off when the sample it scores densely is at most a quarter of the gallery."""
    if q.n < TOPK_BATCH_MIN_Q or not 1 <= k <= TOPK_BATCH_MAX_K or g.n >= (1 << 24):
        return False, 0, 0
    ns, nf = C.c_int64(), C.c_int64()
    check(lib.cmve_topk_batch_workspace(C.byref(q.desc), C.byref(g.desc), int(k), C.byref(ns), C.byref(nf)),
          "cmve_topk_batch_workspace")
    return 4 * ns.value <= g.n, ns.value, nf.value


def topk_batch(q: RowSet, g: RowSet, k: int, mode: int = _lib.SIM_F16, ws: Optional[torch.Tensor] = None):
    """cmve_topk_batch on device: (idx int32 [n, k], fp64 scores [n, k], unresolved int32 [1]).
    Rows left unresolved hold idx -2 (topk() finishes them through cmve_topk)."""
    ok, _, need = topk_batch_plan(q, g, k)
    if not ok:
        raise ValueError("topk_batch: problem outside the batch path (see topk_batch_plan)")
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=q.device)
    idx = torch.empty((q.n, k), dtype=torch.int32, device=q.device)
    sc = torch.empty((q.n, k), dtype=torch.float64, device=q.device)
    unres = torch.zeros(1, dtype=torch.int32, device=q.device)
    check(lib.cmve_topk_batch(handle(q.device), C.byref(q.desc), C.byref(g.desc), int(mode), int(k), _ptr(ws),
                              ws.numel(), _ptr(idx), _ptr(sc), _ptr(unres)), "cmve_topk_batch")
    return idx, sc, unres


def topk(q: RowSet, g: RowSet, k: int, mode: int = _lib.SIM_F16, scores_ws: Optional[torch.Tensor] = None,
         to_host: bool = True, batch: Optional[bool] = None, out=None):
    """Exact top-k gallery indices per query (score desc, index asc) + their fp64 cosines.
    to_host=False returns the device tensors (int32 idx, fp64 scores) instead of numpy arrays.
    Large query batches go through cmve_topk_batch (no score matrix; batch=False forces the
    dense path); rows it leaves unresolved are finished by cmve_topk."""
    k = int(min(k, g.n))
    if k < 1:
        return np.zeros((q.n, 0), np.int64), np.zeros((q.n, 0))
    if k > _lib.TOPK_MAX:
        raise ValueError(f"topk: k <= {_lib.TOPK_MAX}")
    if mode == _lib.SIM_F16 and not (q.has_f16 and g.has_f16):
        mode = _lib.SIM_BF16
    use_batch = topk_batch_plan(q, g, k)[0] if batch is None else bool(batch)
    if use_batch:
        idx, sc, unres = topk_batch(q, g, k, mode, ws=scores_ws)
        if int(unres.item()):
            rows = torch.nonzero(idx[:, 0] == -2).flatten()
            sub = RowSet(q.raw.index_select(0, rows), eps=q.eps, with_lo=q.has_lo, device=q.device,
                         with_f16=q.has_f16)
            i2, s2 = topk(sub, g, k, mode, to_host=False, batch=False)
            idx[rows] = i2
            sc[rows] = s2
        if not to_host:
            return idx, sc
        return idx.to(torch.int64).cpu().numpy(), sc.cpu().numpy()
    need = topk_workspace_floats(q, g, k)
    if scores_ws is None or scores_ws.numel() < need:
        scores_ws = torch.empty(need, dtype=torch.float32, device=q.device)
    if out is not None:  # caller-held (idx int32, scores fp64 [max(n, 1), k], overflow int32 [1]) buffers
        idx, sc, ovf = out
    else:
        idx = torch.empty((max(q.n, 1), k), dtype=torch.int32, device=q.device)
        sc = torch.empty((max(q.n, 1), k), dtype=torch.float64, device=q.device)
        ovf = torch.zeros(1, dtype=torch.int32, device=q.device)
    if mode == _lib.SIM_F16 and not (q.has_f16 and g.has_f16):
        mode = _lib.SIM_BF16
    for m in ((mode, _lib.SIM_BF16X3) if (mode != _lib.SIM_BF16X3 and q.has_lo and g.has_lo) else (mode,)):
        check(lib.cmve_topk(handle(q.device), C.byref(q.desc), C.byref(g.desc), m, k, _ptr(scores_ws),
                            scores_ws.numel(), _ptr(idx), _ptr(sc), _ptr(ovf)), "cmve_topk")
        if int(ovf.item()) == 0:
            break
    else:  # a query's error band held > TOPK_CAP columns (near-duplicate gallery rows at the k-th score)
        idx, sc = _topk_dense_exact(q, g, k)
        if not to_host:
            return idx, sc
        return idx.to(torch.int64).cpu().numpy(), sc.cpu().numpy()
    if not to_host:
        return idx[:q.n], sc[:q.n]
    return idx[:q.n].to(torch.int64).cpu().numpy(), sc[:q.n].cpu().numpy()


def _topk_dense_exact(q: RowSet, g: RowSet, k: int, gallery_chunk: int = 1 << 16):
    """Exact top-k by dense fp64 scoring (the fallback of topk when an error band overflows): the
    normalised rows in fp64, gallery chunks scored by the K10 DOT kernel (a k-ordered fp64 fma chain
    per pair, so exact duplicates score identically -- a library dgemm rounds by tile position), each
    chunk merged with the running top-k by K12f (cmve_topk_dense_merge: radix select + bitonic sort on the
    device, score desc, index asc, NaN last as np.argsort of the errors)."""
    qn = q.normalized(torch.float64)
    gn_all = g.normalized(torch.float64)
    bufs = [(torch.empty((q.n, k), dtype=torch.float64, device=q.device),
             torch.empty((q.n, k), dtype=torch.int64, device=q.device)) for _ in range(2)]
    kb, cur = 0, 0
    for j0 in range(0, g.n, gallery_chunk):
        s = pairwise(qn, gn_all[j0:j0 + gallery_chunk].contiguous(), _lib.PW_DOT, 1.0, 0.0, torch.float64)
        (bs, bi), (os_, oi) = bufs[cur], bufs[1 - cur]
        check(lib.cmve_topk_dense_merge(handle(q.device), _ptr(bs), _ptr(bi), kb, _ptr(s), s.stride(0), q.n,
                                        s.shape[1], j0, k, _ptr(os_), _ptr(oi)), "cmve_topk_dense_merge")
        kb, cur = k, 1 - cur
    best_s, best_i = bufs[cur]
    return best_i.to(torch.int32), best_s


def gt_positions_fused(a: RowSet, b: RowSet, lists, mode: int = _lib.SIM_F16):
    """Exact 1-based position of EVERY GT item: for row i of `a` and k in lists[i],
    1 + #{j : cos64(a_i, b_j) > cos64(a_i, b_k)}.  Implemented as a fused rank count
    over an expanded query set (row i repeated once per GT item, GT list [k])."""
    owners = np.fromiter((i for i, l in enumerate(lists) for _ in l), dtype=np.int64)
    items = [[int(k)] for l in lists for k in l]
    out = [np.zeros(0, np.int64) for _ in lists]
    if owners.size == 0:
        return out
    sel = torch.from_numpy(owners).to(a.device)
    expanded = RowSet(a.raw.index_select(0, sel), eps=a.eps, with_lo=a.has_lo, device=a.device, with_f16=a.has_f16)
    r, _, _ = gt_rank_counts(expanded, b, row_gts=items, mode=mode)
    n_m = b.n
    p = 0
    for i, l in enumerate(lists):
        pi = r[p:p + len(l)].copy()
        # Items ranked individually: an all-NaN GT item gets n_m.  Several items at n_m are all NaN (a
        # finite item can only be last in a row without NaN), and NaN items share the row's last
        # positions n_m - n_nan + 1 .. n_m (AP depends only on the set of positions).
        last = np.flatnonzero(pi == n_m)
        if last.size > 1:
            pi[last] = n_m - last.size + 1 + np.arange(last.size)
        out[i] = pi
        p += len(l)
    return out

