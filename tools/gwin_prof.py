"""Diagnostics: C4 probability-mode windows through k_gwin once per size, for a
GW_PROF build (GSNAPDP_LIB=...; the library prints its per-phase cycles).
usage: python tools/gwin_prof.py [n ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch  # noqa: E402
from gsnapdp import Context, ggap_op_offsets  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import GGAP_RESULT, GGAP_TRACE  # noqa: E402

dev = torch.device("cuda", 0)
genome = W.synthetic_genome(64_000_000, seed=1)
for n in [int(a) for a in sys.argv[1:]] or [50000, 200000]:
    g, b = W.c4_windows(genome, n, seed=4, use_probabilities=True)
    ctx = Context(W.pack_genome(g), mode=0, device=0)
    off = ggap_op_offsets(b.windows)
    d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(b.query.copy()).to(dev)
    d_res = torch.zeros(n * GGAP_RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_trc = torch.zeros(n * GGAP_TRACE.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    names = ctx.profile(True)
    for _ in range(3):
        acc = np.zeros(len(names))
        ctx.ggap_run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), d_res.data_ptr(),
                            d_trc.data_ptr(), d_ops.data_ptr(), d_off.data_ptr())
        ctx.profile_read(acc)
        print(n, {k: round(v, 4) for k, v in zip(names, acc) if v > 0}, flush=True)
    ctx.close()
