"""BASELINE config 3 on the HIP path: 1M x 150 bp reads against the GRCh38-sized
synthetic genome (3.09 Gnt, 1.16 GB packed in HBM, genome positions beyond
2^31), through the device-resident entry point and the op-stream compaction
that feeds the multi-GPU gather (bench.py's step), checked against the CPU
restatement: scores and counts of every window, full pair lists of a sample
expanded from the compact op streams."""
import numpy as np
import pytest
import torch

import oracle as O
from gsnapdp import Context, gather, op_offsets
from gsnapdp import workload as W
from gsnapdp.records import RESULT

pytestmark = pytest.mark.gpu

FIELDS = ("finalscore", "nmatches", "nmismatches", "nopens", "nindels", "reserved")


def device_step(ctx, batch, dev):
    """bench.py's per-rank step: run_device into a payload, then compaction."""
    n = len(batch)
    off = op_offsets(batch.windows)
    d_w = torch.from_numpy(batch.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(batch.query.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    lay = gather.Layout(n, gather.op_budget(n))
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    base = pay.data_ptr()
    ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), base + lay.res_off, d_ops.data_ptr(),
                   d_off.data_ptr(), stream=sp)
    ctx.compact_ops_device(base + lay.res_off, n, d_ops.data_ptr(), d_off.data_ptr(), base + lay.ops_off,
                           lay.budget, base, stream=sp)
    torch.cuda.synchronize()
    res, ops, coff = gather.unpack(lay, pay.cpu().numpy(), n)
    return res, ops, coff, d_ops.cpu().numpy().view(np.uint32), off


def test_gpu_compact_ops_matches_host_mirror():
    dev = torch.device("cuda", 0)
    ctx = Context(np.zeros(64, np.uint32), device=0)
    rng = np.random.default_rng(3)
    for n in (1, 1023, 1024, 1025, 70_000, 2_500_000):  # (the last: more blocks than are resident at once)
        res = np.zeros(n, dtype=RESULT)
        cap = rng.integers(1, 40, size=n)
        off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(cap, out=off[1:])
        res["nops"] = np.where(rng.random(n) < 0.01, 10_000, rng.integers(0, 40, size=n))  # some > capacity
        ops = rng.integers(0, 1 << 32, size=int(off[-1]), dtype=np.uint32)
        want = gather.compact_ops(res, ops, off)
        d_r = torch.from_numpy(res.view(np.uint8).copy()).to(dev)
        d_o = torch.from_numpy(ops.view(np.int32).copy()).to(dev)
        d_f = torch.from_numpy(off.copy()).to(dev)
        for budget in (want.size, max(0, want.size - 1)):
            d_out = torch.zeros(max(1, want.size), dtype=torch.int32, device=dev)
            d_h = torch.zeros(2, dtype=torch.int64, device=dev)
            ctx.compact_ops_device(d_r.data_ptr(), n, d_o.data_ptr(), d_f.data_ptr(), d_out.data_ptr(), budget,
                                   d_h.data_ptr())
            torch.cuda.synchronize()
            h = d_h.cpu().numpy()
            assert int(h[0]) == want.size
            assert int(h[1]) == (1 if want.size > budget else 0)
            if budget == want.size:
                assert d_out.cpu().numpy().view(np.uint32)[:want.size].tobytes() == want.tobytes()
    ctx.close()


def test_gpu_c3_full_size_parity():
    """1M reads vs the 3.09 Gnt genome: every window's scores / counts /
    dynprogindex bit-exact, pair lists of 3000 windows bit-exact, the compact
    op streams equal to the capacity-layout ones."""
    dev = torch.device("cuda", 0)
    g = W.c3_genome(seed=3)
    batch = W.c3_windows(g, n=1_000_000, seed=33)
    absolute = batch.windows["chroffset"].astype(np.int64) + batch.windows["chrpos"]
    assert (absolute > 2**31).mean() > 0.2  # genome positions beyond int32
    ctx = Context(g.blocks, device=0)
    res, cops, coff, ops, off = device_step(ctx, batch, dev)
    assert np.all(res["status"] != 2)
    # compact stream == capacity layout, window by window
    cnt = res["nops"].astype(np.int64)
    idx = np.repeat(off[:-1], cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    assert ops[idx].tobytes() == cops.tobytes()
    O.setup(g.blocks)
    for a in range(0, len(batch), 200_000):
        ores, _, _, _ = O.run_batch(batch.windows[a:a + 200_000], batch.query, batch.query_uc, nthreads=16)
        for f in FIELDS:
            bad = np.nonzero(res[f][a:a + 200_000] != ores[f])[0]
            assert bad.size == 0, "%s differs at windows %s" % (f, (bad[:8] + a))
    rng = np.random.default_rng(1)
    samp = np.unique(np.concatenate([np.arange(1000), rng.integers(0, len(batch), size=2000),
                                     np.nonzero(absolute > 3_000_000_000)[0][:200]]))
    ores, opairs, ooff, onp = O.run_batch(batch.windows[samp], batch.query, batch.query_uc, nthreads=16)
    for j, i in enumerate(samp.tolist()):
        p, _ = ctx.pairs(batch.windows, batch.query, batch.query_uc, res, cops, coff, i)
        assert p.tobytes() == opairs[ooff[j]:ooff[j] + onp[j]].tobytes(), "pairs differ at window %d" % i
    ctx.close()
