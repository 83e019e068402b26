"""cmve -- MI355X-native (gfx950) text<->video retrieval hot path.

Drop-in mirrors of the reference's retrieval surface:
  cmve.linas.evaluation   (LINAS-engine/evaluation.py)
  cmve.linas.metrics      (LINAS-engine/util/metrics.py)
  cmve.linas.validate     (LINAS-engine/validate.py: cal_perf)
  cmve.linas.inference    (LINAS-engine/inference.py scorer + CLI)
All compute goes through libcmve.so (hand-written HIP); importing cmve without the
built library raises ImportError.
"""
from . import _lib  # noqa: F401  (fails loudly without libcmve.so)
from .engine import RowSet, sim_store, gt_rank_counts, rank_from_matrix, topk  # noqa: F401

__all__ = ["RowSet", "sim_store", "gt_rank_counts", "rank_from_matrix", "topk"]
