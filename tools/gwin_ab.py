"""Diagnostics: probability-mode genome-gap windows through k_gwin (one window
per lane, the default) and through k_ggap (GSNAPDP_GWIN=0) on the same batch:
per-stage kernel times and a byte comparison of results, traces and op streams.
usage: python tools/gwin_ab.py [n_windows] [out.json]"""
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

os.environ["GSNAPDP_GWIN_MIN"] = "0"  # every batch size on k_gwin (the mixed sets are 3000 windows)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
out_path = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
genome = W.synthetic_genome(64_000_000, seed=1)
report = {"windows": n, "cases": []}


def run(blocks, b, gwin, steps=10):
    os.environ["GSNAPDP_GWIN"] = "1" if gwin else "0"
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


def compare(tag, a, b, off):
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
    # the ops each traced window returns (k_ggap leaves a stale copy of the left
    # flank's ops past them, k_gwin does not: only the returned ranges compare)
    ops_equal = True
    for i in np.nonzero(ta["bridge_accepted"] != 0)[0]:
        o, m = int(off[i]), int(ta["nops_right"][i]) + int(ta["nops_left"][i])
        if not np.array_equal(oa[o:o + m], ob[o:o + m]):
            ops_equal = False
            bad.setdefault("ops", []).append(int(i))
            if len(bad["ops"]) >= 6:
                break
    print(tag, "ops identical" if ops_equal else "OPS DIFFER", json.dumps(bad), flush=True)
    return not bad and ops_equal, bad


ok = True
cases = []
g, b = W.c4_windows(genome, n, seed=4, use_probabilities=True)
cases.append(("C4 prob", g, b))
g, b = W.c4_windows(genome, n, seed=5, use_probabilities=True)
b.windows["jump_late_p"][::2] = 1
cases.append(("C4 prob jl-mixed", g, b))
g, b = W.c4_windows(genome, n // 4, seed=6, use_probabilities=True, extraband=3)
b.windows["jump_late_p"][1::3] = 1
cases.append(("C4 prob extraband 3", g, b))
for seed in (11, 12):
    g, b = W.ggap_windows(W.synthetic_genome(2_000_000, seed=seed, n_rate=0.002), 3000, seed=seed)
    cases.append(("mix %d" % seed, g, b))
for tag, g, b in cases:
    blocks = W.pack_genome(g)
    steps = 10 if len(b.windows) >= 10000 else 1
    msn, outn = run(blocks, b, True, steps)
    mso, outo = run(blocks, b, False, steps)
    same, bad = compare(tag, outn, outo, ggap_op_offsets(b.windows))
    ok &= same
    print("%s %d windows  gwin %s  old %s" % (tag, len(b.windows), json.dumps(msn), json.dumps(mso)), flush=True)
    report["cases"].append({"case": tag, "windows": int(len(b.windows)), "ms_gwin": msn, "ms_old": mso,
                            "identical": bool(same), "diff": bad})
report["identical"] = bool(ok)
print("AB", "identical" if ok else "DIFFERENT")
if out_path:
    with open(out_path, "w") as f:
        json.dump(report, f, indent=1)
sys.exit(0 if ok else 1)
