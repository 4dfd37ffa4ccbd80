"""Diagnostics: C4 genome-gap windows (score and probability mode) through
k_gband once per mode, for a diagnostic build (GB_PROF prints per-phase shader
clocks summed over waves; GB_PHASES runs a subset of the phases).
usage: GSNAPDP_LIB=gpuexp/NAME/libgsnapdp.so python tools/gb_prof_c4.py [n] [steps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import Context  # noqa: E402
from gsnapdp import workload as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
os.environ.setdefault("GSNAPDP_GBAND_PROB", "1")
genome = W.synthetic_genome(64_000_000, seed=1)
for mode in ("score", "prob"):
    g, b = W.c4_windows(genome, n, seed=4, use_probabilities=(mode == "prob"))
    ctx = Context(W.pack_genome(g))
    for _ in range(steps):
        t0 = time.perf_counter()
        ctx.ggap_run(b.windows, b.query, b.query_uc)
        print(mode, "%.4f s" % (time.perf_counter() - t0), file=sys.stderr, flush=True)
    ctx.close()
