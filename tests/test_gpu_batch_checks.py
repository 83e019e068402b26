"""GPU checks of the K14 batch's argument planning (cmve_eval_batch_create) and of the CMVE_EVAL_PAIRED safety path,
through the C ABI: inputs a batch cannot run with the first evaluation's kernels are refused, and lists that are not
the asserted one-to-one pairing are counted (out[11]) instead of writing out of range.  The ranks of the sessions
involved equal the oracle's (oracle/retrieval.py, pinned to LINAS-engine/util/metrics.py:124-157 via
retrieval_c1.npz)."""
import numpy as np
import pytest

import synth
from oracle import retrieval as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _c1_lists():
    v, c, vid, cid = synth.c1_embeddings()
    v2t_gt, t2v_gt = R.get_gt(vid, cid)
    return v, c, [t2v_gt[i] for i in range(len(cid))], v2t_gt


@pytest.mark.parametrize("paired", [True, False])
def test_rank_batch_refuses_unaligned_later_input(torch_cuda, paired):
    """cmve_eval_batch_create takes every launch's kernels from the first evaluation's plan: a later evaluation whose
    rows are not 16-B aligned (a column slice of a wider buffer) would plan without the residual plane (and, paired,
    without the paired prep), so the batch refuses it -- and that session alone still ranks as the oracle does."""
    torch = torch_cuda
    from cmve import engine
    v, c, rows, cols = _c1_lists()
    if not paired:  # multi-GT v2t lists: the general prep, which plans the residual plane from the rows' alignment
        cols = [list(l) + [(j + 1) % len(cols)] if j % 3 == 0 else list(l) for j, l in enumerate(cols)]
    n_q, n_g, d = c.shape[0], v.shape[0], c.shape[1]
    good = (torch.from_numpy(c).cuda(), torch.from_numpy(v).cuda())
    wide_c = torch.zeros((n_q, d + 2), dtype=torch.float64, device="cuda")
    wide_c[:, 1:1 + d] = good[0]
    sliced = wide_c[:, 1:1 + d]  # rows 8-B aligned only, stride(1) == 1
    assert sliced.stride(1) == 1 and (sliced.data_ptr() % 16) != 0
    sess = [engine.RankSession(n_q, n_g, d, row_gts=rows, col_gts=cols, dtype=torch.float64) for _ in range(2)]
    with pytest.raises(RuntimeError, match="another path|differs in shape / dtype / pairing"):
        engine.RankBatch(sess, [good, (sliced, good[1])])
    t2v, v2t = sess[1].run(sliced, good[1])
    s = R.exact_scores64(c, v)
    assert np.array_equal(t2v, R.rank_counts(s, rows)) and np.array_equal(v2t, R.rank_counts(s.T, cols))


def test_paired_flag_with_lists_that_are_no_pairing(torch_cuda):
    """CMVE_EVAL_PAIRED asserts a one-to-one pairing; the paired prep checks the t2v side per caption and counts the
    captions that break it in out[11] (a caption with no GT, with two GTs, with a video id past the gallery) without
    writing outside the workspace.  RankSession.run raises on it; a batch reports the same count per evaluation."""
    torch = torch_cuda
    from cmve import engine
    v, c, rows, cols = _c1_lists()
    n_q, n_g, d = c.shape[0], v.shape[0], c.shape[1]
    x = (torch.from_numpy(c).cuda(), torch.from_numpy(v).cuda())
    bad = [list(l) for l in rows]
    bad[0] = []                  # no GT
    bad[1] = [bad[1][0], 7]      # two GTs
    bad[2] = [n_g + 5]           # a video id past the gallery
    bad_csr = engine.csr(bad, torch.device("cuda", 0))

    def broken():
        s = engine.RankSession(n_q, n_g, d, row_gts=rows, col_gts=cols, dtype=torch.float64)
        assert s.paired
        s.row = bad_csr  # what a C caller passing CMVE_EVAL_PAIRED with these lists hands the library
        s._args = None
        return s

    s = broken()
    with pytest.raises(RuntimeError, match="one-to-one"):
        s.run(*x)
    assert int(s.host[11]) == 3
    sess = [broken() for _ in range(2)]
    b = engine.RankBatch(sess, [x, x])
    b.run()
    torch.cuda.synchronize()
    assert [int(t.out[11]) for t in sess] == [3, 3]
    b.close()


def _groups(torch, n_groups, per, seed=11):
    """n_groups batches of `per` C1-shaped evaluations (set 0 of group 0 is the golden C1 set, the others perturbed
    captions: the ranks differ per set)."""
    from cmve import engine
    v, c, rows, cols = _c1_lists()
    rng = np.random.default_rng(seed)
    n_q, n_g, d = c.shape[0], v.shape[0], c.shape[1]
    groups = []
    for gi in range(n_groups):
        sets, sess = [], []
        for j in range(per):
            cj = c if (gi == 0 and j == 0) else c + rng.uniform(0.05, 0.6) * rng.standard_normal(c.shape)
            sets.append((torch.from_numpy(cj).cuda(), torch.from_numpy(v).cuda()))
            sess.append(engine.RankSession(n_q, n_g, d, row_gts=rows, col_gts=cols, dtype=torch.float64))
        groups.append((sess, sets))
    return groups, n_q


@pytest.mark.parametrize("per", [8, 3])
def test_rank_batch_chained_equals_run(golden, torch_cuda, per):
    """Chained batch runs (cmve_eval_batch_run_chained: a batch's finish in the next run's prep launch) give every
    output word of the batch's own run(); a batch's outputs are complete once the next chained run is enqueued;
    the C1 set's ranks equal the reference's."""
    torch = torch_cuda
    from cmve import engine
    groups, n_q = _groups(torch, 3, per)
    batches, ref = [], []
    for sess, sets in groups:
        b = engine.RankBatch(sess, sets)
        b.run()
        torch.cuda.synchronize()
        ref.append([s.out.clone() for s in sess])
        for s in sess:  # (the chained runs must write every word an evaluation writes again; out[13:16] reserved)
            s.out[:13].fill_(-7)
            s.out[16:].fill_(-7)
        batches.append(b)
    g = golden("retrieval_c1")
    h = ref[0][0].cpu().numpy()
    assert np.array_equal(h[16:16 + n_q], g["t2v_ranks"]) and np.array_equal(h[16 + n_q:], g["v2t_ranks"])
    prev = None
    for k, bi in enumerate([0, 1, 2, 0, 1, 2, 1]):
        batches[bi].run_chained(prev, timing_slot=k % 4)
        if k == 1:
            torch.cuda.synchronize()  # batch 0's finish ran in batch 1's first launch
            for s, r in zip(groups[0][0], ref[0]):
                assert torch.equal(s.out, r)
        prev = batches[bi]
    prev.finish()
    torch.cuda.synchronize()
    for (sess, _), rs in zip(groups, ref):
        for s, r in zip(sess, rs):
            assert torch.equal(s.out, r), (s.out[:16].tolist(), r[:16].tolist())
    ms = batches[2].kernel_timing(3)
    assert ms[0] > 0 and ms[1] > 0 and ms[3] == 0.0
    twin = engine.RankBatch(groups[0][0][:per], groups[0][1][:per])
    twin.run_chained(None)
    with pytest.raises(RuntimeError, match="shares a workspace"):
        batches[0].run_chained(twin)
    twin.finish()
    torch.cuda.synchronize()
    for b in batches + [twin]:
        b.close()


def test_rank_batch_chained_general_prep(torch_cuda):
    """A batch that takes no specialised prep (multi-GT fp32 lists, split-bf16) chains through separate launches:
    the previous finish first, then the prep and the rank GEMM -- outputs equal run()'s."""
    torch = torch_cuda
    from cmve import engine, _lib
    rng = np.random.default_rng(21)
    nq, ng, d = 700, 900, 384
    rows = [[int(x) for x in rng.choice(ng, size=1 + i % 3, replace=False)] for i in range(nq)]
    cols = [[] for _ in range(ng)]
    for i, l in enumerate(rows):
        for j in l:
            cols[j].append(i)
    bats, ref = [], []
    for b in range(2):
        sets, sess = [], []
        for j in range(2):
            gal = rng.standard_normal((ng, d)).astype(np.float32)
            qs = (gal[[l[0] for l in rows]] + 0.9 * rng.standard_normal((nq, d))).astype(np.float32)
            sets.append((torch.from_numpy(qs).cuda(), torch.from_numpy(gal).cuda()))
            sess.append(engine.RankSession(nq, ng, d, row_gts=rows, col_gts=cols, dtype=torch.float32,
                                           mode=_lib.SIM_BF16X3))
        rb = engine.RankBatch(sess, sets)
        rb.run()
        torch.cuda.synchronize()
        ref.append([s.out.clone() for s in sess])
        bats.append((rb, sess))
    b0, b1 = bats[0][0], bats[1][0]
    b0.run_chained(None)
    with pytest.raises(RuntimeError, match="not finished"):
        b0.run()  # its finish is still pending
    b1.run_chained(b0)
    with pytest.raises(RuntimeError, match="no chained run awaiting"):
        b0.finish()  # (finished inside b1's first launch)
    with pytest.raises(RuntimeError, match="not finished"):
        b1.run_chained(b0)  # b1's own chained run still awaits its finish
    b1.finish()
    with pytest.raises(RuntimeError, match="no chained run awaiting"):
        b1.finish()
    torch.cuda.synchronize()
    for (rb, sess), rs in zip(bats, ref):
        for s, r in zip(sess, rs):
            assert torch.equal(s.out, r)
        rb.close()


@pytest.mark.parametrize("nq,ng", [(700, 900), (900, 600)])
def test_rank_batch_chained_f16_multi_gt(torch_cuda, nq, ng):
    """An F16 batch whose lists are no one-to-one pairing (multi-GT captions, n_q != n_g) at d = 512 takes the
    general prep in run(); its chained runs must not fuse the specialised PAIRED prep with the previous finish
    (which packs only the GT partners' gallery rows, and writes gallery rows at caption indices): every output word
    equals run()'s, and the ranks equal the oracle's exact counts."""
    torch = torch_cuda
    from cmve import engine
    rng = np.random.default_rng(31)
    d = 512
    rows = [[int(x) for x in rng.choice(ng, size=1 + i % 3, replace=False)] for i in range(nq)]
    cols = [[] for _ in range(ng)]
    for i, l in enumerate(rows):
        for j in l:
            cols[j].append(i)
    bats, ref, host = [], [], []
    for b in range(3):
        sets, sess = [], []
        for j in range(2):
            gal = rng.standard_normal((ng, d))
            qs = gal[[l[0] for l in rows]] + 0.9 * rng.standard_normal((nq, d))
            host.append((qs, gal))
            sets.append((torch.from_numpy(qs).cuda(), torch.from_numpy(gal).cuda()))
            sess.append(engine.RankSession(nq, ng, d, row_gts=rows, col_gts=cols, dtype=torch.float64))
        assert not sess[0].paired
        rb = engine.RankBatch(sess, sets)
        rb.run()
        torch.cuda.synchronize()
        ref.append([s.out.clone() for s in sess])
        for s in sess:
            s.out[:13].fill_(-7)
            s.out[16:].fill_(-7)
        bats.append((rb, sess))
    prev = None
    for bi in [0, 1, 2, 0]:
        bats[bi][0].run_chained(prev)
        prev = bats[bi][0]
    prev.finish()
    torch.cuda.synchronize()
    for (rb, sess), rs in zip(bats, ref):
        for s, r in zip(sess, rs):
            assert torch.equal(s.out, r), (s.out[:16].tolist(), r[:16].tolist())
    qs, gal = host[0]
    s = R.exact_scores64(qs, gal)
    h = bats[0][1][0].out.cpu().numpy()
    assert np.array_equal(h[16:16 + nq], R.rank_counts(s, rows)) and np.array_equal(h[16 + nq:], R.rank_counts(s.T, cols))
    for rb, _ in bats:
        rb.close()


def test_rank_batch_chained_refuses_shared_outputs(torch_cuda):
    """Two batches writing one output block: a chained run of one after the other is refused (the second's prep zeroes
    the R@K head the first's finish adds into, in the same launch); run() of either stays allowed."""
    torch = torch_cuda
    from cmve import engine
    groups, n_q = _groups(torch, 2, 2)
    n_out = groups[0][0][0].out.numel()
    shared = torch.zeros((2, n_out), dtype=torch.int64, device="cuda")
    b0 = engine.RankBatch(groups[0][0], groups[0][1], outs=list(shared))
    b1 = engine.RankBatch(groups[1][0], groups[1][1], outs=list(shared))
    b0.run()
    b1.run()
    b0.run_chained(None)
    with pytest.raises(RuntimeError, match="shares an output"):
        b1.run_chained(b0)
    b0.finish()
    torch.cuda.synchronize()
    b0.close()
    b1.close()
