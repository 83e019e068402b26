"""Benchmark of the retrieval hot path: query-video pairs/s scored + R@1/5/10 parity.

    python bench.py [--gpus N --steps K --warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Workload (one step = one pass of the hot path over one query batch):
  every rank holds a resident 131,072-video x 1024-d synthetic gallery shard (1,048,576
  videos at 8 GPUs = BASELINE north-star gallery; weak scaling); 16,384 queries per step
  (each rank contributes N_q / N, with its GT in its own shard) are all-gathered over RCCL,
  packed, GT-scored exactly (fp64 + all-reduce MAX), ranked against every shard by the
  fused bf16-MFMA rank-count kernel + fp64 fix-up, counts all-reduced (SUM), and the
  R@1/5/10 / medr / meanr computed on host.  value = N_q x N_global_gallery / step time.
Also reported: the MSR-VTT-1kA protocol (C1, 1000 x 1000 x 1024) end to end with its
R@1/5/10 checked against the reference's golden values, and the reference CPU algorithm
(oracle port: fp64 cal_error + per-row argsort eval_q2m) timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16/fp16 MFMA (MI355X_MICROARCH.md: F16 forms take the bf16 cycles)
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--shard", type=int, default=131072, help="gallery videos per GPU")
    p.add_argument("--nq", type=int, default=16384, help="queries per step (whole job)")
    p.add_argument("--dim", type=int, default=1024)
    p.add_argument("--sigma", type=float, default=10.0)
    p.add_argument("--cpu-sample-queries", type=int, default=6144, help="CPU-baseline sample (~10-15 s of host work)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip the 1kA and CPU legs (profiling runs)")
    p.add_argument("--chunks", type=int, default=1,
                   help="gallery pieces per shard: each piece's fp64 fix-up overlaps the next piece's MFMA pass")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01_traffic.json"))
    p.add_argument("--topk-leg", action="store_true",
                   help="run the sharded exact top-k leg at any N (by default only at N=1, with the extras)")
    p.add_argument("--rehearse-gloo", action="store_true",
                   help="N>1 rehearsal on a 1-GPU box: gloo instead of RCCL, ranks share the visible GPUs "
                        "(exercises every collective of the sharded path; not a measurement)")
    return p.parse_args()


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_gloo:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if args.rehearse_gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    if world > 1:
        dist.barrier()


def msrvtt1ka(steps=20):
    """C1 end to end on the GPU: fused two-direction ranks, R@K vs the reference's golden values."""
    import synth
    from cmve import engine
    from cmve.linas import metrics as M
    v, c, vid, cid = synth.c1_embeddings()
    gold = np.load(os.path.join(ROOT, "tests", "golden", "retrieval_c1.npz"))
    v2t_gt, t2v_gt = M.get_gt(vid, cid)
    t2v_lists = [t2v_gt[i] for i in range(len(cid))]
    vt = torch.from_numpy(v).cuda()
    ct = torch.from_numpy(c).cuda()

    # the evaluation as the reference's validation loop re-runs it (validate.py:61-74): resident
    # buffers, the evaluation enqueued as one sequence (pack both sets, GT thresholds, rank GEMM, fix-up)
    sess = engine.RankSession(len(cid), len(vid), v.shape[1], row_gts=t2v_lists, col_gts=v2t_gt,
                              dtype=vt.dtype, device=vt.device)

    def step():
        return sess.run(ct, vt)

    for _ in range(3):
        t2v, v2t = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t2v, v2t = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # the same evaluation without the session (fresh packing, workspace and launches per call)
    engine.gt_rank_counts(engine.RowSet(ct, with_lo=False), engine.RowSet(vt, with_lo=False),
                          row_gts=t2v_lists, col_gts=v2t_gt)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        e_t, e_v, _ = engine.gt_rank_counts(engine.RowSet(ct, with_lo=False), engine.RowSet(vt, with_lo=False),
                                            row_gts=t2v_lists, col_gts=v2t_gt)
    dt_eager = (time.perf_counter() - t1) / 5
    t2v_m = M.metrics_from_ranks(t2v)
    v2t_m = M.metrics_from_ranks(v2t)
    parity = bool(np.array_equal(t2v, gold["t2v_ranks"]) and np.array_equal(v2t, gold["v2t_ranks"])
                  and np.array_equal(e_t, t2v) and np.array_equal(e_v, v2t))
    return {"pairs_per_s": 1000 * 1000 / dt, "ms_per_eval": dt * 1e3, "ms_per_eval_eager": dt_eager * 1e3,
            "t2v_r1_r5_r10": [round(x, 3) for x in t2v_m[:3]], "v2t_r1_r5_r10": [round(x, 3) for x in v2t_m[:3]],
            "ref_t2v_r1_r5_r10": [float(x) for x in gold["t2v"][:3]], "parity_exact": parity,
            "note": "RankSession (resident buffers): device copy-in, packing of both sets, GT scoring, both directions, "
                    "D2H of ranks; eager = the same through fresh RowSets / gt_rank_counts"}


def inference_leg(n_gallery=1048576, d=1024, k=10, reps=20, cpu_rows=262144):
    """LINAS inference.py scorer (inference.py:76-82: cal_error + argsort[:topK]) at the north star's
    1M-video gallery on one GPU: exact top-k of single captions (the HBM-bound GEMV regime) and of
    16-caption batches.  The gallery is packed once (resident); a call = query pack + GEMV + top-k
    select + fp64 re-score + D2H of the ids.  CPU leg: the oracle port of the reference's per-query
    path (re-normalise the gallery, fp64 GEMV, full argsort) on a bounded sample of the gallery."""
    from cmve.linas.inference import GalleryScorer
    from oracle import retrieval as R
    dev = torch.device("cuda", torch.cuda.current_device())
    gen = torch.Generator(device=dev).manual_seed(77)
    gal = torch.randn((n_gallery, d), generator=gen, device=dev, dtype=torch.float32)
    scorer = GalleryScorer(gal)  # the inference.py mirror: gallery normalised + packed once
    g = scorer.gallery
    picks = torch.randint(0, n_gallery, (32,), generator=gen, device=dev)
    caps = (gal[picks] + 10.0 * torch.randn((32, d), generator=gen, device=dev)).contiguous()
    out = {"gallery": n_gallery, "dim": d, "k": k}
    ids1 = None
    for nq in (1, 16):
        times = []
        for r in range(reps + 3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx = scorer.topk_indices(caps[r % 16:r % 16 + nq] if nq == 1 else caps[:nq], k)
            if r >= 3:
                times.append(time.perf_counter() - t0)
            if nq == 1 and r == 3:
                ids1 = (r % 16, idx[0])
        ms = float(np.median(times)) * 1e3
        gemv_bytes = n_gallery * g.d_pad * 2  # the fp16 gallery plane, streamed once per call
        out[f"nq{nq}"] = {"ms_per_call": ms, "pairs_per_s": nq * n_gallery / (ms * 1e-3),
                          "gallery_GBps_lower_bound": gemv_bytes / (ms * 1e-3) / 1e9}
    # CPU oracle port of the reference path on a bounded sample (one caption, first cpu_rows videos)
    g_np = gal[:cpu_rows].cpu().numpy().astype(np.float64)
    c_np = caps[ids1[0]:ids1[0] + 1].cpu().numpy()
    t0 = time.perf_counter()
    top = R.inference_topk(g_np, c_np, k)
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": cpu_rows / dt, "unit": "pairs/s", "kind": "port",
                           "sample": f"1 caption x {cpu_rows} videos x {d}-d: fp64 l2norm of the gallery, GEMV, "
                                     f"full argsort (oracle/retrieval.py inference_topk), {dt:.2f} s"}
    out["gpu_over_cpu_nq1"] = out["nq1"]["pairs_per_s"] / out["cpu_baseline"]["value"]
    del g, gal, scorer
    torch.cuda.empty_cache()
    return out


def sharded_topk_leg(scorer, q_local, nq, n_global, k=10, reps=5):
    """C5 top-k regime on the bench's own resident shard: exact top-k of every gathered caption
    (all-gather Q -> K13 cmve_topk_batch on the shard, no score matrix -> all-gather + device
    merge of the per-shard top-k -> ids on host), inference.py:78-79 applied per caption."""
    scorer.topk(q_local, k)  # warm-up (sizes the batch workspace)
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ids, _ = scorer.topk(q_local, k)
        times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    return {"k": k, "queries": nq, "gallery_total": n_global, "ms_per_batch": ms,
            "pairs_per_s": nq * n_global / (ms * 1e-3), "ids_head": ids[0, :3].tolist(),
            "note": "wall clock incl. Q all-gather, sample + main MFMA passes, fp64 band re-score, merge, D2H"}


def other_configs_leg():
    """BASELINE configs C2 and C4 on this GPU (the full-size runs are tools/train_bench.py and
    tools/fusion_bench.py): the C2 training step (B 128, 1024 -> 1024 heads, InfoNCE row + col and
    TripletLoss, clip + Adam, one hipGraph replay per step) and the C4 MultiFusion composed path on
    8,192 queries x the 44,493-video gallery.  Failures are reported, never fatal to the bench line."""
    import argparse as _ap
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    out = {}
    try:
        import train_bench as TB
        dev = torch.device("cuda", torch.cuda.current_device())
        batches = TB.data(dev, 4)
        c2 = {}
        for loss_name in ("infonce", "triplet"):
            ms, _ = TB.time_leg(TB.cmve_step_fn(dev, loss_name, graph=True), batches, 10, 50, dev)
            c2[loss_name] = {"ms_per_step": ms, "samples_per_s": TB.B / ms * 1e3}
        out["c2_train_step"] = c2
    except Exception as e:  # noqa: BLE001
        out["c2_train_step"] = {"error": repr(e)}
    try:
        import fusion_bench as FB
        c4 = FB.run(_ap.Namespace(nq=8192, nv=44493, chunk=8192, loop_q=256))
        out["c4_multifusion"] = {k: c4[k] for k in ("nq", "nv", "combine_batches", "ranking", "end_to_end")}
    except Exception as e:  # noqa: BLE001
        out["c4_multifusion"] = {"error": repr(e)}
    torch.cuda.empty_cache()
    return out


def cpu_baseline(gallery_np, queries_np, gts_local, n_sample):
    """Oracle port of the reference CPU path: fp64 cal_error (evaluation.py:17-21) + per-row argsort
    eval_q2m (metrics.py:124-157) on a bounded sample of the same workload."""
    from oracle import retrieval as R
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    q = queries_np[:n_sample].astype(np.float64)
    g = gallery_np.astype(np.float64)
    lists = [[int(x)] for x in gts_local[:n_sample]]
    t0 = time.perf_counter()
    errors = R.cal_error(g, q)
    ranks = R.gt_ranks(errors, lists)
    dt = time.perf_counter() - t0
    return {"value": q.shape[0] * g.shape[0] / dt, "unit": "pairs/s", "cores": int(threads), "kind": "port",
            "sample": f"{q.shape[0]} queries x {g.shape[0]} gallery x {g.shape[1]}-d fp64 cal_error + per-row argsort "
                      f"rank (oracle/retrieval.py), {dt:.1f} s", "seconds": dt,
            "ranks_head": ranks[:8].tolist()}


def main():
    args = parse()
    rank, world, local = init_dist(args)
    from cmve import engine, _lib
    from cmve.dist import ShardedGallery, metrics_from_ranks, recall_counts_device
    dev = torch.device("cuda", local)
    shard, nq, d = args.shard, args.nq, args.dim
    assert nq % world == 0, "queries must split evenly across ranks"
    n_local = nq // world
    n_global = shard * world

    # ---- synthetic resident inputs (not timed) ----
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    gallery = torch.randn((shard, d), generator=gen, device=dev, dtype=torch.float32)
    gt_local = torch.randint(0, shard, (n_local,), generator=gen, device=dev)
    q_local = (gallery[gt_local] + args.sigma * torch.randn((n_local, d), generator=gen, device=dev)).contiguous()
    scorer = ShardedGallery(gallery, offset=rank * shard, n_global=n_global, with_lo=False, device=dev)
    gts_gathered = scorer.all_gather_rows((gt_local + rank * shard).contiguous()).cpu().numpy()
    gt_csr = scorer.local_gt_csr([[int(g)] for g in gts_gathered])
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    ranks = None
    chunks = max(1, args.chunks)
    ranks = scorer.rank_queries(q_local, gt_csr, nq, mode=_lib.SIM_F16, chunks=chunks)  # sizes the workspace
    for _ in range(args.warmup):  # the timed loop's own path (its torch ops load before timing)
        r_w, o_w = scorer.rank_queries_device(scorer.all_gather_rows(q_local), gt_csr, nq, mode=_lib.SIM_F16,
                                              chunks=chunks)
        w = torch.cat([recall_counts_device(r_w), o_w.to(torch.int64).reshape(1)]).cpu()
        assert not w[4].item(), "undecided-pair list overflowed during warm-up"
    barrier(world)
    torch.cuda.synchronize()
    # Pipelined steps: the all-gather of step s+1's queries runs on RCCL's stream while step s
    # computes (issued before step s is enqueued, so it waits only for step s-1, the last reader of
    # its buffer); each step's R@K counts and overflow flag go to pinned host memory asynchronously
    # and are read one step later, so the host never stalls the GPU inside the loop.
    import ctypes
    kms, kn = ctypes.c_float(0.0), ctypes.c_int32(0)
    mfma_launch_ms = []
    qbuf = [torch.empty((nq, d), dtype=torch.float32, device=dev) for _ in range(2 if world > 1 else 0)]
    host = [torch.empty(5, dtype=torch.int64).pin_memory() for _ in range(args.steps)]
    done = [torch.cuda.Event() for _ in range(args.steps)]
    recalls = []

    def collect(s):
        done[s].synchronize()
        if host[s][4].item():
            raise RuntimeError("undecided-pair list overflowed inside the timed loop (warm-up sizes it)")
        recalls.append(host[s][:4].tolist())
        if chunks > 1:
            _lib.check(_lib.lib.cmve_overlap_mfma_ms(engine.handle(dev), ctypes.byref(kms), ctypes.byref(kn)))
            mfma_launch_ms.append(kms.value / max(kn.value, 1))

    def gather(s):  # world 1: the local queries are all the queries (no copy)
        return scorer.gather_rows_async(q_local, qbuf[s % 2]) if world > 1 else None

    t0 = time.perf_counter()
    work = {0: gather(0)}
    for s in range(args.steps):
        if s + 1 < args.steps:
            work[s + 1] = gather(s + 1)
        if work[s] is not None:
            work[s].wait()
        q_all = qbuf[s % 2] if world > 1 else q_local
        ranks_dev, ovf = scorer.rank_queries_device(q_all, gt_csr, nq, mode=_lib.SIM_F16, events=ev[s],
                                                    chunks=chunks)
        small = torch.cat([recall_counts_device(ranks_dev), ovf.to(torch.int64).reshape(1)])
        host[s].copy_(small, non_blocking=True)
        done[s].record()
        if s > 0:
            collect(s - 1)
    collect(args.steps - 1)
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    met = metrics_from_ranks(ranks_dev.cpu().numpy())
    assert recalls[-1][0] == int(np.count_nonzero(ranks_dev.cpu().numpy() <= 1))
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if chunks > 1:
        mfma_ms = float(np.mean(mfma_launch_ms))
        fix_ms = None  # overlapped with the MFMA passes
    else:
        mfma_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
        fix_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    rank_ms = float(np.mean([e[0].elapsed_time(e[2]) for e in ev]))
    ncand = scorer.ws.ncand()

    topk_out = None
    if args.topk_leg or (world == 1 and not args.no_extras):  # collective at N > 1: every rank runs it
        topk_out = sharded_topk_leg(scorer, q_local, nq, n_global)
    if rank == 0:
        ms = dt / args.steps * 1e3
        value = nq * n_global * args.steps / dt
        launches = chunks
        flops = 2.0 * nq * (shard / launches) * d  # per MFMA-pass launch
        achieved = flops / (mfma_ms * 1e-3) / 1e12
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if (tj.get("shard") == shard and tj.get("nq") == nq and tj.get("dim") == d
                        and tj.get("chunks", 1) == chunks):
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "query-video pairs/sec scored + R@1/5/10 parity, MSR-VTT-1kA at 1/8 GPU",
            "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f16",
            "data": "synthetic (torch.randn gallery shards, queries = GT video + sigma*noise; no dataset offline)",
            "config": {"workload": f"gallery-shard retrieval scoring: {nq:,} text queries x ({shard:,} videos per "
                                   f"GPU) x {d}-d, t2v GT rank -> R@1/5/10 (fused fp16 MFMA rank count + fp64 fix-up)",
                       "queries_per_step": nq, "gallery_per_gpu": shard, "gallery_total": n_global, "dim": d,
                       "sigma": args.sigma, "parallelism": f"gallery-shard x{world} (RCCL all-gather Q, "
                                                            f"all-reduce MAX gt / SUM counts)"},
            "recall": {"r1": met[0], "r5": met[1], "r10": met[2], "medr": met[3], "meanr": met[4]},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_BF16_TFLOPS, "traffic": traffic,
                         "kernel": "cmve::sim_kernel<F16, RANK, G256 phased>", "kernel_ms": mfma_ms,
                         "flops_per_launch": flops, "launches_per_step": launches},
            "rank_count": {"ms": rank_ms, "chunks": chunks, "fixup_ms": fix_ms, "candidates_per_step": ncand,
                           "note": "MFMA passes + fp64 fix-ups of one step (fix-ups overlapped when chunks > 1)"},
        }
        if topk_out is not None:
            out["sharded_topk"] = topk_out
        if world == 1 and not args.no_extras:
            out["msrvtt1kA"] = msrvtt1ka()
            out["inference_topk"] = inference_leg()
            out.update(other_configs_leg())
            if not args.no_cpu_baseline:
                g_np = gallery.cpu().numpy()
                q_np = q_local.cpu().numpy()
                out["cpu_baseline"] = cpu_baseline(g_np, q_np, gt_local.cpu().numpy(), args.cpu_sample_queries)
                out["cpu_baseline"]["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
