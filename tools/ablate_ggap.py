"""Per-stage timing of the C4 genome-gap workload for one library build (diagnostics)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch  # noqa: E402
from gsnapdp import Context, ggap_op_offsets  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import GGAP_RESULT, GGAP_TRACE  # noqa: E402

prob = len(sys.argv) > 1 and sys.argv[1] == "prob"
n = 200_000
g, b = W.c4_windows(W.synthetic_genome(64_000_000, seed=1), n, seed=4, use_probabilities=prob)
ctx = Context(W.pack_genome(g), mode=0, device=0)
dev = torch.device("cuda", 0)
off = ggap_op_offsets(b.windows)
d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
d_q = torch.from_numpy(b.query.copy()).to(dev)
d_res = torch.zeros(n * GGAP_RESULT.itemsize, dtype=torch.uint8, device=dev)
d_trc = torch.zeros(n * GGAP_TRACE.itemsize, dtype=torch.uint8, device=dev)
d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
d_off = torch.from_numpy(off.copy()).to(dev)
step = lambda: ctx.ggap_run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), d_res.data_ptr(),
                                   d_trc.data_ptr(), d_ops.data_ptr(), d_off.data_ptr())
for _ in range(3):
    step()
ctx.sync()
names = ctx.profile(True)
acc = np.zeros(len(names))
K = 10
for _ in range(K):
    step()
    ctx.profile_read(acc)
print(os.path.basename(os.environ.get("GSNAPDP_LIB", "default")), "prob" if prob else "score",
      json.dumps({k: round(v / K, 4) for k, v in zip(names, acc) if v > 0}))
