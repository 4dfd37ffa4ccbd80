"""Diagnostics: genome-gap windows through the register-band path (k_gband) and
the row-lane path (k_ggap, GSNAPDP_GGAP_ROWLANE=1) on the same batch: per-stage
kernel times and a byte comparison of results, traces and op streams.
usage: python tools/ggap_ab.py [n_windows]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
dev = torch.device("cuda", 0)
genome = W.synthetic_genome(64_000_000, seed=1)


def run(blocks, b, rowlane, steps=10):
    os.environ["GSNAPDP_GGAP_ROWLANE"] = "1" if rowlane else "0"
    os.environ["GSNAPDP_GBAND_PROB"] = "1"  # probability mode on the band too
    ctx = Context(blocks, mode=0, device=0)
    m = len(b.windows)
    off = ggap_op_offsets(b.windows)
    d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(b.query.copy()).to(dev)
    d_u = torch.from_numpy(b.query_uc.copy()).to(dev)
    d_res = torch.zeros(m * GGAP_RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_trc = torch.zeros(m * GGAP_TRACE.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    d_off = torch.from_numpy(off.copy()).to(dev)

    def step():
        ctx.ggap_run_device(d_w.data_ptr(), m, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(),
                            d_trc.data_ptr(), d_ops.data_ptr(), d_off.data_ptr())
    step()
    ctx.sync()
    names = ctx.profile(True)
    acc = np.zeros(len(names))
    for _ in range(steps):
        step()
        ctx.profile_read(acc)
    ctx.profile(False)
    ms = {k: round(v / steps, 4) for k, v in zip(names, acc) if v > 0}
    out = (d_res.cpu().numpy(), d_trc.cpu().numpy(), d_ops.cpu().numpy())
    ctx.close()
    return ms, out


def compare(tag, a, b, windows):
    ra, ta, oa = a
    rb, tb, ob = b
    ra, rb = ra.view(GGAP_RESULT), rb.view(GGAP_RESULT)
    ta, tb = ta.view(GGAP_TRACE), tb.view(GGAP_TRACE)
    bad = {}
    for f in GGAP_RESULT.names:
        x = np.nonzero(ra[f] != rb[f])[0] if ra[f].dtype != np.float64 else \
            np.nonzero(ra[f].view(np.uint64) != rb[f].view(np.uint64))[0]
        if x.size:
            bad[f] = [int(i) for i in x[:6]] + [int(x.size)]
    for f in GGAP_TRACE.names:
        x = np.nonzero(ta[f] != tb[f])[0]
        if x.size:
            bad["trace." + f] = [int(i) for i in x[:6]] + [int(x.size)]
    ops_equal = bool(np.array_equal(oa, ob))
    print(tag, "ops identical" if ops_equal else "OPS DIFFER", json.dumps(bad), flush=True)
    return not bad and ops_equal


ok = True
for mode in ("score", "prob"):
    g, b = W.c4_windows(genome, n, seed=4, use_probabilities=(mode == "prob"))
    blocks = W.pack_genome(g)
    msb, outb = run(blocks, b, False)
    msr, outr = run(blocks, b, True)
    print("C4 %s %d windows  band %s  rowlane %s" % (mode, n, json.dumps(msb), json.dumps(msr)), flush=True)
    ok &= compare("C4 " + mode, outb, outr, b.windows)
# both tie-rule lists of the register band
g, b = W.c4_windows(genome, n, seed=5, use_probabilities=False)
b.windows["jump_late_p"][::2] = 1
blocks = W.pack_genome(g)
msb, outb = run(blocks, b, False)
msr, outr = run(blocks, b, True)
print("C4 score, jump_late_p mixed, %d windows  band %s  rowlane %s" % (n, json.dumps(msb), json.dumps(msr)), flush=True)
ok &= compare("C4 jl-mixed", outb, outr, b.windows)
for seed in (11, 12):
    g, b = W.ggap_windows(W.synthetic_genome(2_000_000, seed=seed, n_rate=0.002), 3000, seed=seed)
    blocks = W.pack_genome(g)
    _, outb = run(blocks, b, False, steps=1)
    _, outr = run(blocks, b, True, steps=1)
    ok &= compare("mix %d" % seed, outb, outr, b.windows)
print("AB", "identical" if ok else "DIFFERENT")
# ablation builds (tools/build_variant.sh -DGB_EXP_*) compute wrong results on purpose
sys.exit(0 if ok or os.environ.get("GGAP_AB_TIMING_ONLY") == "1" else 1)
