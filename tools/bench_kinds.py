"""Throughput per window kind (diagnostics): single gaps vs end gaps (k_fill / k_rows)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch  # noqa: E402
from gsnapdp import Context, op_offsets  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import END3_GAP, END5_GAP, RESULT, SINGLE_GAP  # noqa: E402

g = W.synthetic_genome(16_000_000, seed=1)
ctx = Context(W.pack_genome(g), mode=0, device=0)
dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
for name, kinds in (("single", (SINGLE_GAP,)), ("ends", (END5_GAP, END3_GAP))):
    b = W.random_windows(g, n, seed=5, kinds=kinds, max_len1=100, max_len2=110, max_band=3,
                         allow_weird_chars=False)
    off = op_offsets(b.windows)
    d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(b.query.copy()).to(dev)
    d_u = torch.from_numpy(b.query_uc.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    step = lambda: ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(),
                                  d_ops.data_ptr(), d_off.data_ptr())
    for _ in range(2):
        step()
    ctx.sync()
    names = ctx.profile(True)
    acc = np.zeros(len(names))
    K = 5
    for _ in range(K):
        step()
        ctx.profile_read(acc)
    ctx.profile(False)
    ms = {k: round(v / K, 4) for k, v in zip(names, acc) if v > 0}
    print(name, n, json.dumps(ms), "windows/s %.3g" % (n / (sum(ms.values()) * 1e-3)), flush=True)
