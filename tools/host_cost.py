"""Host-side cost of one K14 evaluation enqueue and its parts (developer study)."""
import os, sys, time, json
ROOT='/root/repo' if os.path.exists('/root/repo/bench.py') else os.environ['GRAFT_REPO_ROOT']
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch, ctypes as C
import bench
from cmve import engine, _lib
dev = torch.device("cuda", 0)
sess, ct, vt, _ = bench.c1_session(dev)
sess.run(ct, vt)
st = torch.cuda.Stream(dev)
res = {}
def t(name, fn, n=2000):
    """host time of fn alone (the GPU queue is drained every 4 calls, outside the clock)"""
    torch.cuda.synchronize()
    fn()
    tot = 0.0
    for i in range(n):
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
        if i % 4 == 3:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    res[name] = tot / n * 1e6
def ctx():
    with torch.cuda.stream(st):
        pass
t("stream_ctx", ctx, 20000)
t("handle", lambda: engine.handle(dev), 20000)
t("enqueue_default_stream", lambda: sess.enqueue(ct, vt), 2000)
def enq_ctx():
    with torch.cuda.stream(st):
        sess.enqueue(ct, vt)
t("enqueue_in_stream_ctx", enq_ctx, 2000)
h = engine.handle(dev)
args = sess._args
out_p = engine._ptr(sess.out)
f = _lib.lib.cmve_eval_ranks
t("raw_ctypes_call", lambda: f(h, *args, out_p, -1), 2000)
gsess, gct, gvt, _ = bench.c1_session(dev, st)
gsess.run(gct, gvt)
gr = gsess.graph(gct, gvt)
t("graph_launch", gr.launch, 2000)
print(json.dumps({"host_us": res}))
