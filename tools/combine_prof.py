"""One combine_batches call on 8,192 composed queries (C4 shape) after a warm-up, for a
rocprofv3 kernel trace of the Combiner's kernels alone."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cross-modal-video-engine_amd"))

import torch  # noqa: E402
from cmve.multifusion.combiner import Combiner  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = Combiner(640, 2560, 5120).to(dev).eval()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
gen = torch.Generator(device=dev).manual_seed(3)
high = torch.randn((n, 8, 640), generator=gen, device=dev)
mid = torch.randn((n, 8, 16, 640), generator=gen, device=dev)
text = torch.randn((n, 640), generator=gen, device=dev)
m.combine_batches((high, mid), text)
torch.cuda.synchronize()
m.combine_batches((high, mid), text)
torch.cuda.synchronize()
print("done")
