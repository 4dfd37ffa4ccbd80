"""The stage-3 intron pass on a recorded gmap run (bigdata/*_stage3.npz, made by
oracle/gen_golden.py stage3_golden from oracle/_ref/gmap_trace; not committed):
every build_pairs_introns call of the run in one gsnapdp_stage3_pass, checked
against the reference's lists, beside the reference's own time for the calls.
usage: python tools/stage3_trace_bench.py bigdata/gmap_274_stage3.npz [copies]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import Context  # noqa: E402
from gsnapdp import workload as W  # noqa: E402

z = np.load(sys.argv[1], allow_pickle=False)
copies = int(sys.argv[2]) if len(sys.argv) > 2 else 1
calls, pin, q, qu, want = W.stage3_calls(z, copies)
ctx = Context(z["blocks"])
ctx.stage3_pass(calls[:64], pin, q, qu)  # warm-up
buf = np.empty(ctx.stage3_capacity(calls), dtype=want.dtype)
best = None
for _ in range(4):  # the first run also faults the output buffer in
    t0 = time.perf_counter()
    c, got, st = ctx.stage3_pass(calls, pin, q, qu, out=buf)
    dt = time.perf_counter() - t0
    if best is None or dt < best[0]:
        best = (dt, c, got.copy(), st)
dt, c, got, st = best
ok = bool((c["status"] == 0).all()) and got.tobytes() == want.tobytes()
for f in ("out_minor", "out_major", "out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen",
          "shiftp", "incompletep", "nout"):
    ok = ok and bool(np.array_equal(c[f], calls[f]))
nwin = int(np.sum(st["windows"]))
ref = float(z["calls"]["ref_seconds"].sum()) * copies
print(json.dumps({"trace": os.path.basename(sys.argv[1]), "copies": copies, "paths": int(len(calls)),
                  "bit_exact": ok, "seconds": round(dt, 4), "rounds": int(st["rounds"]), "windows": nwin,
                  "windows_by_family": [int(x) for x in st["windows"]], "batches": [int(x) for x in st["batches"]],
                  "host_s": round(float(st["seconds"][0]), 4), "batches_s": round(float(st["seconds"][1]), 4),
                  "paths_per_s": round(len(calls) / dt, 1), "windows_per_s": round(nwin / dt, 1),
                  "reference_seconds_1thread": round(ref, 4), "speedup_vs_reference": round(ref / dt, 2)}))
