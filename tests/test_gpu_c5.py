"""C5 end to end on the GPU (BASELINE configs[4]): the MCT TSN feature-extraction
head (recognizer2d.py:76-83) on K2, the projection head on K3 / K1, the packed shard and its exact ranks /
top-k (cmve.mct.TSNGallery -> cmve.dist.ShardedGallery), against the CPU oracle.

Tolerances: the pool and the head are fp32 arithmetic against the fp64 oracle (atol 2e-6 on outputs of
magnitude <= 1, the LINAS head tolerance of tests/test_oracle_heads.py).  Ranks and top-k ids are exact:
they are checked bit for bit against the oracle's fp64 scoring of the SAME stored rows (the reference
ranks its own fp32 embeddings in fp64, LINAS-engine/evaluation.py:102), and against the oracle's own
fp64 embeddings wherever the decision is not within the head's tolerance of a tie."""
import numpy as np
import pytest

from oracle import heads as H
from oracle import retrieval as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("shape", [(3, 25, 2048, 8, 8), (2, 3, 100, 7, 7), (5, 25, 2048, 1, 1), (2, 4, 130, 11, 11),
                                   (1, 1, 64, 4, 4)])
def test_tsn_pool_matches_oracle(torch_cuda, shape):
    torch = torch_cuda
    from cmve import mct
    B, S, C, Hh, W = shape
    x = np.random.default_rng(sum(shape)).standard_normal((B * S, C, Hh, W)).astype(np.float32)
    got = mct.tsn_feature_extraction(torch.from_numpy(x).cuda(), B).cpu().numpy()
    np.testing.assert_allclose(got, H.tsn_feature_extraction(x, B), rtol=0, atol=2e-6)
    if Hh * W == 1:  # the [B, S, C] form of spatially pooled maps
        got3 = mct.tsn_feature_extraction(torch.from_numpy(x.reshape(B, S, C)).cuda(), B).cpu().numpy()
        np.testing.assert_array_equal(got3, got)


def _latent_head(torch, d_in, d_out, seed):
    from cmve.linas.model import Latent_mapping
    torch.manual_seed(seed)
    head = Latent_mapping([d_in, d_out], 0.0)
    bn = head.mapping.bn_1
    g = torch.Generator().manual_seed(seed + 1)
    bn.running_mean.copy_(0.01 * torch.randn(d_out, generator=g))
    bn.running_var.copy_(0.5 + torch.rand(d_out, generator=g))
    bn.weight.data.copy_(1.0 + 0.1 * torch.randn(d_out, generator=g))
    bn.bias.data.copy_(0.01 * torch.randn(d_out, generator=g))
    sd = {k: v.detach().cpu().numpy() for k, v in head.state_dict().items()}
    return head.cuda().eval(), sd


def test_c5_chain_matches_oracle(torch_cuda):
    """4,096 videos of TSN segment features ([N, 25, 2048], and 64 videos as [N*25, 2048, 7, 7] maps) ->
    TSNGallery (pool, Latent_mapping 2048 -> 1024 with BN running stats, l2norm) -> the packed shard:
    rows == the oracle head; exact t2v / v2t ranks and top-10 == the oracle's fp64 scoring."""
    torch = torch_cuda
    from cmve import mct
    rng = np.random.default_rng(44)
    n, S, F, D = 4096, 25, 2048, 1024
    feats = rng.standard_normal((n, S, F)).astype(np.float32)
    maps = rng.standard_normal((64 * S, F, 7, 7)).astype(np.float32)
    head, sd = _latent_head(torch, F, D, 4)
    gal = mct.TSNGallery(n + 64, head)
    for c0 in range(0, n, 1024):  # chunked ingest, as a loader would feed it
        gal.ingest(torch.from_numpy(feats[c0:c0 + 1024]).cuda(), 1024)
    gal.ingest(torch.from_numpy(maps).cuda(), 64)
    shard = gal.finalize()
    rows = gal.rows[:gal.n].double().cpu().numpy()
    exp_rows = np.concatenate([H.latent_mapping_eval(H.pool_mean(feats), sd, [F, D]),
                               H.latent_mapping_eval(H.tsn_feature_extraction(maps, 64), sd, [F, D])])
    np.testing.assert_allclose(rows, exp_rows, rtol=0, atol=2e-6)
    # captions: noisy copies of their GT video's embedding
    nq = 600
    gt = rng.integers(0, gal.n, nq)
    q = (exp_rows[gt] + 0.035 * rng.standard_normal((nq, D))).astype(np.float32)
    t2v = [[int(g)] for g in gt]
    v2t = [[] for _ in range(gal.n)]
    for i, g in enumerate(gt):
        v2t[int(g)].append(i)
    r_t, r_v = shard.evaluate(torch.from_numpy(q).cuda(), t2v, v2t)
    s = R.exact_scores64(q, rows)
    assert np.array_equal(r_t, R.rank_counts(s, t2v)) and np.array_equal(r_v, R.rank_counts(s.T, v2t))
    top, top_s = shard.topk(torch.from_numpy(q).cuda(), 10)
    assert np.array_equal(top, np.argsort(-s, axis=1, kind="stable")[:, :10])
    np.testing.assert_allclose(top_s, np.take_along_axis(s, top, 1), rtol=0, atol=1e-13)
    # against the oracle's own embeddings: every rank whose GT score is not within the head tolerance of
    # another video's score agrees
    s_o = R.exact_scores64(q, exp_rows)
    r_o = R.rank_counts(s_o, t2v)
    gts = s_o[np.arange(nq), gt]
    near = (np.abs(s_o - gts[:, None]) < 1e-5).sum(1) > 1
    assert np.array_equal(r_t[~near], r_o[~near]), int((r_t[~near] != r_o[~near]).sum())
    print(f"C5 chain: R@1 {100 * np.mean(r_t <= 1):.1f}, near-tie rows {int(near.sum())}")


def test_c5_full_shard_properties(torch_cuda):
    """The 131,072-video C5 shard (1M gallery / 8 GPUs) ingested chunk by chunk from seeded TSN features
    through an nn.Linear 2048 -> 1024 head: rows finite; 16,384 captions' exact t2v ranks; for 256 sampled
    captions the ranks and the top-10 equal an independent fp64 scoring of the whole stored shard."""
    torch = torch_cuda
    from cmve import mct
    n, S, F, D, chunk = 131072, 25, 2048, 1024, 8192
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    head = torch.nn.Linear(F, D)
    gal = mct.TSNGallery(n, head)
    gen = torch.Generator(device=dev).manual_seed(4)
    for c0 in range(0, n, chunk):
        gal.ingest(torch.randn((chunk, S, F), generator=gen, device=dev), chunk)
    shard = gal.finalize()
    rows = gal.rows
    assert bool(torch.isfinite(rows).all())
    nq = 16384
    gt = torch.randint(0, n, (nq,), generator=gen, device=dev)
    rn = rows / rows.norm(dim=1, keepdim=True)
    q = (rn[gt] + 0.03 * torch.randn((nq, D), generator=gen, device=dev)).contiguous()
    gts = [[int(g)] for g in gt.tolist()]
    ranks = shard.rank_queries(q, shard.local_gt_csr(gts), nq)
    assert ranks.min() >= 1 and ranks.max() <= n
    pick = torch.randperm(nq, generator=torch.Generator().manual_seed(1))[:256].to(dev)
    qs = q[pick].double()
    qs = qs / qs.norm(dim=1, keepdim=True)
    gd = rows.double()
    gd = gd / gd.norm(dim=1, keepdim=True)
    s64 = qs @ gd.T
    sgt = s64.gather(1, gt[pick][:, None])
    exp = (1 + (s64 > sgt).sum(1)).cpu().numpy()
    assert np.array_equal(ranks[pick.cpu().numpy()], exp)
    top, _ = shard.topk(q[pick].contiguous(), 10)
    exp_top = torch.sort(s64, dim=1, descending=True, stable=True).indices[:, :10].cpu().numpy()
    assert np.array_equal(top, exp_top)
    print(f"C5 shard: R@1 {100 * np.mean(ranks <= 1):.1f} R@10 {100 * np.mean(ranks <= 10):.1f}")
