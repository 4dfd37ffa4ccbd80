"""Diagnostics: one C4 genome-gap batch (score or probability mode) through
the register band (k_gband), the row-lane kernel (k_ggap) or, probability
mode only, the window-per-lane kernel (k_gwin, the default), for counter runs.
usage: python tools/ggap_one.py score|prob band|rowlane|gwin [n] [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
mode, path = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 200_000
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
os.environ["GSNAPDP_GGAP_ROWLANE"] = "1" if path == "rowlane" else "0"
os.environ["GSNAPDP_GWIN"] = "1" if path == "gwin" else "0"
os.environ["GSNAPDP_GBAND_PROB"] = "1"  # probability mode on the band too (band runs)
from gsnapdp import Context  # noqa: E402
from gsnapdp import workload as W  # noqa: E402

genome = W.synthetic_genome(64_000_000, seed=1)
g, b = W.c4_windows(genome, n, seed=4, use_probabilities=(mode == "prob"))
ctx = Context(W.pack_genome(g))
for _ in range(steps):
    res, _, _, _ = ctx.ggap_run(b.windows, b.query, b.query_uc)
print(mode, path, n, "windows,", int((res["returned_null"] == 0).sum()), "accepted", flush=True)
ctx.close()
