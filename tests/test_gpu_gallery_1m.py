"""The north star's 1M-video gallery on ONE GPU (bench.py's gallery_1m leg at N = 1, the base of its 1 -> 8 strong
scaling): 16,384 captions x 1,048,576 videos x 1024-d, exact t2v GT ranks through the sharded-gallery path
(LINAS-engine/inference.py:76-82 scoring, evaluation.py:17-21 + util/metrics.py:124-157 ranking).

Properties at full size (no CPU oracle can score 1.7e10 pairs in a test): every rank in [1, n_g], the recall sums
monotone, the same gallery / captions regardless of the rank count (strong_gallery_inputs), and 256 sampled captions
equal to independent fp64 torch GEMMs over the whole gallery (bit-exact ranks), 16 of them also to the CPU oracle itself
(oracle/retrieval.py exact_scores64 + rank_counts over all 1,048,576 gallery rows)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_gallery_1m_single_gpu_ranks_against_fp64():
    import torch
    import bench
    from cmve import _lib
    from cmve.dist import ShardedGallery
    dev = torch.device("cuda", 0)
    total, nq, d = 1048576, 16384, 1024
    gallery, q, gts = bench.strong_gallery_inputs(0, 1, dev, total, nq, d, 10.0)
    assert gallery.shape == (total, d) and q.shape == (nq, d)
    # the inputs do not depend on the rank count: rank 3 of 8 holds rows [3/8, 4/8) of the same gallery
    g8, q8, gts8 = bench.strong_gallery_inputs(3, 8, dev, total, nq, d, 10.0)
    assert gts8 == gts
    assert torch.equal(g8, gallery[3 * total // 8:4 * total // 8]) and torch.equal(q8, q[3 * nq // 8:4 * nq // 8])
    del g8, q8
    scorer = ShardedGallery(gallery, offset=0, n_global=total, with_lo=False, device=dev, comm=None)  # (no process group: world 1)
    ranks = scorer.rank_queries(q, scorer.local_gt_csr(gts), nq, mode=_lib.SIM_F16)
    assert ranks.min() >= 1 and ranks.max() <= total
    r1, r5, r10 = (int((ranks <= k).sum()) for k in (1, 5, 10))
    assert 0 < r1 <= r5 <= r10 <= nq
    sample = torch.arange(0, nq, nq // 256)
    exp = bench.sampled_fp64_ranks(gallery, 0, q, gts, sample, 1)
    got = ranks[sample.numpy()]
    print(f"1M gallery: R@1 {100 * r1 / nq:.2f} R@10 {100 * r10 / nq:.2f}, "
          f"{int((got != exp).sum())} of {got.size} sampled ranks differ from fp64")
    assert np.array_equal(got, exp)
    # the oracle on 16 of the sampled captions (fp64 l2norm + GEMM + rank count on the host, ~2 s)
    from oracle import retrieval as R
    sub = sample[::16]
    s64 = R.exact_scores64(q[sub.to(dev)].cpu().numpy(), gallery.cpu().numpy())
    exp_o = R.rank_counts(s64, [gts[i] for i in sub.tolist()])
    assert np.array_equal(ranks[sub.numpy()], exp_o)
