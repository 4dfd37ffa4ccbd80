"""Per-call latency of the host-buffer entry points (batches of 1 .. 4096),
the cost a per-call drop-in caller pays.  GPU box only.

usage: python tools/latency_probe.py [reps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import Context  # noqa: E402
from gsnapdp import workload as W  # noqa: E402


def timeit(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts = np.array(ts) * 1e6
    return np.median(ts), ts.mean(), ts.min()


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    g = W.synthetic_genome(2_000_000, seed=5, n_rate=0.002)
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    b = W.c2_windows(g, n=4096, seed=9)
    gg, gb = W.ggap_windows(g, 4096, seed=9, mix=False)
    ctx_g = Context(W.pack_genome(gg))
    for n in (1, 16, 256, 4096):
        w = b.windows[:n]
        med, mean, mn = timeit(lambda: ctx.run(w, b.query, b.query_uc), reps if n < 4096 else 20)
        print("gap   n=%5d  median %8.1f us  mean %8.1f  min %8.1f  per window %.2f us" % (n, med, mean, mn, med / n))
        wg = gb.windows[:n]
        med, mean, mn = timeit(lambda: ctx_g.ggap_run(wg, gb.query, gb.query_uc), reps if n < 4096 else 20)
        print("ggap  n=%5d  median %8.1f us  mean %8.1f  min %8.1f  per window %.2f us" % (n, med, mean, mn, med / n))
        rng = np.random.default_rng(1)
        model = rng.integers(0, 4, n).astype(np.uint8)
        pos = rng.integers(100, g.size - 100, n).astype(np.uint32)
        ch = np.zeros(n, np.uint32)
        med, mean, mn = timeit(lambda: ctx.maxent(model, pos, ch), reps if n < 4096 else 20)
        print("maxent n=%5d median %8.1f us  mean %8.1f  min %8.1f  per call %.2f us" % (n, med, mean, mn, med / n))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
