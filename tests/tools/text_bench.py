"""Query-side row: caption-encoding throughput on the GPU box.  Prints one JSON line.

Workload: LINAS default text encoder (word_dim 500, biGRU 2x512, Conv2d 3 x 512 kernels of widths
2/3/4, gru_pool mean, concate full; LINAS-engine/trainer.py:41-65) + Latent_mapping [bow + 2560, 1536],
random init, a synthetic 10k-word rnn vocabulary and 7,807-word bow vocabulary (MSR-VTT scale),
59,800 synthetic captions of 4-20 words (the msrvtt10k test caption count).
  batched: QueryEncoder.encode_captions (evaluation.encode_text, evaluation.py:119-171), batch 128
  single:  process_cap + QueryEncoder on one caption (the inference.py:76-77 query path)
Legs: cmve (pools + mapping on HIP, GRU / conv PyTorch-ROCm) and the oracle restatement of the
encoder on the host cores (torch CPU GRU / conv + numpy pools; kind 'port'), on a bounded sample."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root (tests/tools/..)
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from cmve.linas import text as T
    from cmve.linas.checkpoint import QueryEncoder
    from cmve.linas.model import Latent_mapping
    rng = np.random.default_rng(0)
    words = [f"w{i}" for i in range(10000)]
    rnn = T.Vocabulary.from_words(["<pad>", "<start>", "<end>", "<unk>"] + words, "rnn")
    bow = T.Vocabulary.from_words(words[:7807], "bow")
    b2v = T.Bow2Vec(bow)
    n = int(os.environ.get("N_CAPS", 59800))
    caps = [" ".join(rng.choice(words, size=int(rng.integers(4, 21)))) for _ in range(n)]
    opt = argparse.Namespace(word_dim=500, we_parameter=None, text_rnn_size=512, dropout=0.2, concate="full",
                             gru_pool="mean", loss_fun="mrl", vocab_size=len(rnn), text_kernel_num=512,
                             text_kernel_sizes=[2, 3, 4], style="GT", teacher_model="teacher",
                             text_mapping_layers=[1024 + 1536 + len(bow), 1536], hidden_size=1024,
                             student_model="de+map", tag_vocab_size=512)
    torch.manual_seed(0)
    slots = [None] * 9
    slots[5] = T.Text_multilevel_encoding_ori(opt).state_dict()
    slots[4] = Latent_mapping(opt.text_mapping_layers, 0.2).state_dict()
    qe = QueryEncoder(opt, slots)
    qe.encode_captions(caps[:256], rnn, b2v)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    emb = qe.encode_captions(caps, rnn, b2v, batch_size=128)
    torch.cuda.synchronize()
    t_batch = time.perf_counter() - t0
    t0 = time.perf_counter()
    for s in range(0, n, 128):
        T.collate_text(caps[s:s + 128], rnn, b2v, device=qe.device)
    torch.cuda.synchronize()
    t_collate = time.perf_counter() - t0
    lat = []
    for q in caps[:200]:
        t0 = time.perf_counter()
        qe(T.process_cap(q, rnn, b2v))
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    # host baseline: the oracle restatement (torch CPU GRU/conv + numpy pools) on a bounded sample
    from oracle import text as OT
    threads = int(os.environ.get("CPU_THREADS", 16))
    torch.set_num_threads(threads)
    sd = {k: v.numpy() for k, v in slots[5].items()}
    n_cpu, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 10.0 and n_cpu < n:
        (ids, bw, lens, mask), _, _ = T.collate_text(caps[n_cpu:n_cpu + 128], rnn, b2v)
        OT.encode_text(sd, "", ids.numpy(), bw.numpy(), lens, [2, 3, 4], 512, "mean", "full")
        n_cpu += 128
    t_cpu = time.perf_counter() - t0
    print(json.dumps({
        "metric": "captions encoded per second (text encoder + mapping, LINAS defaults)",
        "config": {"workload": f"{n} synthetic captions (4-20 words), rnn vocab {len(rnn)}, bow {len(bow)}, "
                               "word_dim 500, biGRU 2x512, conv 3x512, mapping -> 1536", "batch": 128},
        "batched": {"captions_per_s": n / t_batch, "seconds": t_batch, "emb_shape": list(emb.shape),
                    "host_collate_seconds": t_collate},
        "single_query_ms": {"median": float(np.median(lat)) * 1e3, "p90": float(np.percentile(lat, 90)) * 1e3},
        "cpu_baseline": {"kind": "port", "what": "oracle encoder (torch CPU GRU/conv + numpy pools), no mapping",
                         "cores": threads, "captions_per_s": n_cpu / t_cpu, "sample": f"{n_cpu} captions"}}))


if __name__ == "__main__":
    main()
