"""Training-step row: time the C2 step (BASELINE configs[1]) on the
GPU box.  Prints one JSON line.

C2 step (B = 128, per-frame features [T in U[20, 64], 1024], synthetic):
  videos: K2 mean_valid pool -> Latent_mapping([1024, 1024], dropout 0.2, train) -> l2norm
  captions: [B, 1024] text-encoder features -> Latent_mapping([1024, 1024], 0.2, train) -> l2norm
  loss: TripletLoss(0.2, max_violation, sum, all) (LINAS) or InfoNCE(100, row + col) (C2)
  backward, clip_grad_norm_(params, 2), Adam(lr 1e-4)           = train_emb 'GT', model.py:984-1004
Legs:
  cmve:        cmve.linas.train.GTTrainer on the HIP kernels (no host sync inside the step)
  cmve_graph:  the same step captured once into a hipGraph and replayed (GTTrainer(graph=True))
  torch_eager: the same step written with torch.nn / torch.optim on the same GPU (the reference's
               module structure, loss.py TripletLoss formula restated in torch) -- a same-hardware
               comparison point, not the reference itself (which needs CUDA + a full Dual_Encoding)
  cpu:         the torch_eager step on the host cores (cpu_baseline, kind "port"), a few steps."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

B, F, D, T_MAX = 128, 1024, 1024, 64


def data(dev, n_batches, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = []
    for _ in range(n_batches):
        lengths = torch.randint(20, T_MAX + 1, (B,), generator=g)
        frames = torch.randn(B, T_MAX, F, generator=g)
        caps = torch.randn(B, F, generator=g)
        out.append((frames.to(dev), lengths.to(torch.int32).to(dev), caps.to(dev)))
    return out


# ---------------------------------------------------------------- torch restatement
class TorchHead(nn.Module):
    def __init__(self, p=0.2):
        super().__init__()
        self.fc1 = nn.Linear(F, D)
        r = (6.0 / (F + D)) ** 0.5  # xavier_init_fc, model.py:43-49 (as the cmve heads)
        nn.init.uniform_(self.fc1.weight, -r, r)
        nn.init.zeros_(self.fc1.bias)
        self.bn_1 = nn.BatchNorm1d(D)
        self.dropout = nn.Dropout(p)

    def forward(self, x):
        y = self.dropout(self.bn_1(self.fc1(x)))
        return y / y.pow(2).sum(1, keepdim=True).sqrt()


def torch_triplet(s, im, margin=0.2):
    S = im.mm(s.t())
    d = S.diag().view(-1, 1)
    cost_s = (margin + S - d.expand_as(S)).clamp(min=0)
    cost_im = (margin + S - d.t().expand_as(S)).clamp(min=0)
    I = torch.eye(S.size(0), device=S.device) > .5
    cost_s = cost_s.masked_fill_(I, 0).max(1)[0]
    cost_im = cost_im.masked_fill_(I, 0).max(0)[0]
    return cost_s.sum() + cost_im.sum()


def torch_infonce(p, t, scale=100.0):
    logits = scale * p @ t.T
    gt = torch.arange(p.shape[0], device=p.device)
    ce = nn.functional.cross_entropy
    return (ce(logits, gt) + ce(logits.T, gt)) / 2


def torch_step_fn(dev, loss_name):
    vm, tm = TorchHead().to(dev).train(), TorchHead().to(dev).train()
    params = list(vm.parameters()) + list(tm.parameters())
    opt = torch.optim.Adam(params, lr=1e-4)
    crit = torch_triplet if loss_name == "triplet" else torch_infonce

    def step(frames, lengths, caps):
        mask = (torch.arange(T_MAX, device=dev)[None, :] < lengths[:, None].long()).float()
        pooled = (frames * mask[:, :, None]).sum(1) / lengths[:, None].float()
        vid, cap = vm(pooled), tm(caps)
        opt.zero_grad()
        loss = crit(cap, vid) if loss_name == "triplet" else crit(vid, cap)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 2.0)
        opt.step()
        return loss.detach()
    return step


def cmve_step_fn(dev, loss_name, graph=False):
    from cmve.linas.model import Latent_mapping, temporal_pool
    from cmve.linas.loss import TripletLoss
    from cmve.linas.train import GTTrainer
    from cmve.multifusion.loss import InfoNCE
    vm, tm = Latent_mapping([F, D], 0.2).to(dev), Latent_mapping([F, D], 0.2).to(dev)
    crit = (TripletLoss(0.2, 'cosine', True, 'sum', 'all') if loss_name == "triplet" else
            (lambda cap, vid, _c=InfoNCE(100.0, "both"): _c(vid, cap)))
    tr = GTTrainer(vm, tm, crit, learning_rate=1e-4, grad_clip=2.0, graph=graph)
    tr.train_start()

    def step(frames, lengths, caps):
        pooled = temporal_pool(frames, "mean_valid", lengths)
        return tr.train_emb(pooled, caps, sync=False)[1]
    return step


def time_leg(step, batches, warmup, steps, dev):
    for i in range(warmup):
        step(*batches[i % len(batches)])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(*batches[i % len(batches)])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, float(loss)


def main():
    steps = int(os.environ.get("STEPS", 100))
    warmup = int(os.environ.get("WARMUP", 10))
    dev = torch.device("cuda", 0)
    batches = data(dev, 4)
    res = {}
    legs = os.environ.get("LEGS", "cmve,cmve_graph,torch_eager").split(",")
    nan = (float("nan"), float("nan"))
    for loss_name in ("triplet", "infonce"):
        ms_c, l_c = time_leg(cmve_step_fn(dev, loss_name), batches, warmup, steps, dev) if "cmve" in legs else nan
        ms_g, l_g = (time_leg(cmve_step_fn(dev, loss_name, graph=True), batches, warmup, steps, dev)
                     if "cmve_graph" in legs else nan)
        ms_t, l_t = time_leg(torch_step_fn(dev, loss_name), batches, warmup, steps, dev) if "torch_eager" in legs else nan
        res[loss_name] = {"cmve_ms_per_step": ms_c, "cmve_graph_ms_per_step": ms_g, "torch_eager_ms_per_step": ms_t,
                          "cmve_graph_samples_per_s": B / ms_g * 1e3, "speedup_vs_torch_eager": ms_t / ms_g,
                          "last_loss": {"cmve": l_c, "cmve_graph": l_g, "torch_eager": l_t}}
    cpu = torch.device("cpu")
    threads = int(os.environ.get("CPU_THREADS", 16))
    torch.set_num_threads(threads)
    cb = [(f.cpu(), l.cpu(), c.cpu()) for f, l, c in batches[:2]]
    ms_cpu, _ = time_leg(torch_step_fn(cpu, "triplet"), cb, 1, int(os.environ.get("CPU_STEPS", 5)), cpu)
    flops = 2 * (2 * B * F * D) + 2 * (2 * B * F * D)  # fwd GEMMs + dW GEMMs (inputs need no grad)
    print(json.dumps({
        "metric": "C2 training steps/s (dual-encoder heads + loss + backward + clip + Adam)",
        "config": {"workload": f"B={B}, frames T~U[20,64] x {F}, heads [{F},{D}] x2, dropout 0.2, Adam lr 1e-4, "
                               f"clip 2", "steps": steps, "warmup": warmup},
        "dtype": "f32 (GEMMs on exact-fp32 MFMA)",
        "legs": res,
        "gemm_gflop_per_step": flops / 1e9,
        "cpu_baseline": {"kind": "port", "what": "torch_eager step on the host", "cores": threads,
                         "ms_per_step": ms_cpu, "sample": f"{os.environ.get('CPU_STEPS', 5)} triplet steps"}}))


if __name__ == "__main__":
    main()
