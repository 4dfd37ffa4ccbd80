"""Diagnostics: does ordering a batch's windows by length2 (so each k_fill
wave-task holds windows of one length and its masked tail and traceback starts
shrink) speed up k_fill?  Times k_fill on the C3 batch (bench.py's workload) as
generated and stably sorted by (length2, length1), by HIP events, alternating.

    python tools/l2sort_probe.py [STEPS]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch  # noqa: E402

from gsnapdp import Context, op_offsets  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import RESULT  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    g, batch = W.c3_cached(1_000_000, 0)
    dev = torch.device("cuda", 0)
    ctx = Context(g.blocks, mode=0, device=0)
    w0 = np.array(batch.windows)
    order = np.lexsort((w0["length1"], w0["length2"]))
    runs = {}
    for name, w in (("as_generated", w0), ("sorted_by_length2", w0[order])):
        n = len(w)
        off = op_offsets(w)
        d_w = torch.from_numpy(w.view(np.uint8).copy()).to(dev)
        d_q = torch.from_numpy(np.array(batch.query)).to(dev)
        d_off = torch.from_numpy(off.copy()).to(dev)
        d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
        d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
        runs[name] = (n, d_w, d_q, d_off, d_res, d_ops)
    out = {k: [] for k in runs}
    for rep in range(4):
        for name, (n, d_w, d_q, d_off, d_res, d_ops) in runs.items():
            def step():
                ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), d_res.data_ptr(),
                               d_ops.data_ptr(), d_off.data_ptr())
            for _ in range(2):
                step()
            ctx.sync()
            names = ctx.profile(True)
            acc = np.zeros(len(names))
            for _ in range(steps):
                step()
                ctx.profile_read(acc)
            ctx.profile(False)
            out[name].append({k: round(v / steps, 4) for k, v in zip(names, acc) if v > 0})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
