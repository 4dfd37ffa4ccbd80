"""Diagnostics: one rank's slice of the fixed C3 batch (bench.measure_slices'
per-rank step: run_device + compact_ops_device) run K times back to back, for
a rocprofv3 --kernel-trace timeline of the per-step fixed costs.

    python tools/slice_trace.py [N] [RANK] [STEPS]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from gsnapdp import Context, gather, op_offsets  # noqa: E402
from gsnapdp import workload as W  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    r = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    dev = torch.device("cuda", 0)
    g, batch = W.c3_cached(1_000_000, 0)
    cells = bench.cells_per_window(batch.windows)
    wl, ql, sizes, lo, hi = bench.shard_slice(batch, cells, N, r)
    n = hi - lo
    ctx = Context(g.blocks, mode=0, device=0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    off = op_offsets(wl)
    d_w = torch.from_numpy(wl.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(ql.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    lay = gather.Layout(max(sizes), gather.op_budget(max(sizes)))
    payb = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
    base = payb.data_ptr()

    def step():
        ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), base + lay.res_off,
                       d_ops.data_ptr(), d_off.data_ptr(), stream=sp)
        ctx.compact_ops_device(base + lay.res_off, n, d_ops.data_ptr(), d_off.data_ptr(),
                               base + lay.ops_off, lay.budget, base, stream=sp)
    for _ in range(3):
        step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    print("N=%d rank %d: %d windows, %.4f ms per step" % (N, r, n, 1000 * (time.perf_counter() - t0) / steps))
    ctx.close()


if __name__ == "__main__":
    main()
