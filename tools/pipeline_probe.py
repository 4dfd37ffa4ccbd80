"""Diagnostics: two batches in flight.  The per-rank step (run_device +
compact_ops_device) of the C3 batch and of its N = 8 rank-0 slice, run K times
on one context / one stream, then alternating between two contexts on two
streams (each with its own scratch and output buffers), so that one batch's
k_fill tail overlaps the next batch's plan and fill.

    python tools/pipeline_probe.py [STEPS]"""
import json
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    g, batch = W.c3_cached(1_000_000, 0)
    cells = bench.cells_per_window(batch.windows)
    ctxs = [Context(g.blocks, mode=0, device=0) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    out = {}
    for N in (1, 8):
        wl, ql, sizes, lo, hi = bench.shard_slice(batch, cells, N, 0)
        n = hi - lo
        off = op_offsets(wl)
        d_w = torch.from_numpy(wl.view(np.uint8).copy()).to(dev)
        d_q = torch.from_numpy(ql.copy()).to(dev)
        d_off = torch.from_numpy(off.copy()).to(dev)
        lay = gather.Layout(max(sizes), gather.op_budget(max(sizes)))
        bufs = [(torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev),
                 torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)) for _ in range(2)]

        def step(k):
            ctx, sp = ctxs[k], streams[k].cuda_stream
            d_ops, payb = bufs[k]
            base = payb.data_ptr()
            ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), base + lay.res_off,
                           d_ops.data_ptr(), d_off.data_ptr(), stream=sp)
            ctx.compact_ops_device(base + lay.res_off, n, d_ops.data_ptr(), d_off.data_ptr(),
                                   base + lay.ops_off, lay.budget, base, stream=sp)

        def timed(ways):
            for i in range(4):
                step(i % ways)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                step(i % ways)
            torch.cuda.synchronize()
            return 1000.0 * (time.perf_counter() - t0) / steps
        res = {"reads": n}
        for rep in range(3):
            res.setdefault("one_stream_ms", []).append(round(timed(1), 4))
            res.setdefault("two_streams_ms", []).append(round(timed(2), 4))
        # the two pipelines' outputs agree with each other (same batch)
        torch.cuda.synchronize()
        a, b = bufs[0][1].cpu().numpy(), bufs[1][1].cpu().numpy()
        res["outputs_identical"] = bool(np.array_equal(a, b))
        out["N%d" % N] = res
        print(json.dumps({"N%d" % N: res}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
