"""Host round trips of different families on ONE context from several threads
at once.  gsnapdp_ggap_run_host, _sj_run_host, _cgap_run_host and
_micro_run_host share the context's device staging buffer (and may grow it);
each takes the context's host lock, so concurrent callers of the public batched
API get exactly the results of serial calls."""
import threading

import numpy as np
import pytest

from gsnapdp import Context
from gsnapdp import workload as W

pytestmark = pytest.mark.gpu


def test_gpu_host_round_trips_from_threads_match_serial():
    g = W.synthetic_genome(2_000_000, seed=31, n_rate=0.002)
    _, gg = W.ggap_windows(g, 1500, seed=31)
    sj = W.sj_windows(g, 2000, seed=32)
    cg = W.cgap_windows(g, 800, seed=33)
    _, mi = W.micro_windows(g, 400, seed=34)
    ctx = Context(W.pack_genome(g))

    def run(kind):
        # results and the expanded pair lists (op slots past a window's own ops
        # are unspecified: they hold whatever the shared staging held before)
        if kind == "ggap":
            res, trc, ops, off = ctx.ggap_run(gg.windows, gg.query, gg.query_uc)
            p, k = ctx.ggap_all_pairs(gg.windows, gg.query, gg.query_uc, res, trc, ops, off)
            return res.tobytes() + trc.tobytes() + p.tobytes() + k.tobytes()
        if kind == "sj":
            res, ops, off = ctx.sj_run(sj.windows, sj.query, sj.query_uc)
            p, k = ctx.sj_all_pairs(sj.windows, sj.query, sj.query_uc, res, ops, off)
            return res.tobytes() + p.tobytes() + k.tobytes()
        if kind == "cgap":
            res, ops, off = ctx.cgap_run(cg.windows, cg.query, cg.query_uc)
            p, k = ctx.cgap_all_pairs(cg.windows, cg.query, cg.query_uc, res, ops, off)
            return res.tobytes() + p.tobytes() + k.tobytes()
        res = ctx.micro_run(mi.windows, mi.query, mi.query_uc)
        p, k = ctx.micro_all_pairs(mi.windows, mi.query, mi.query_uc, res)
        return res.tobytes() + p.tobytes() + k.tobytes()

    kinds = ["ggap", "sj", "cgap", "micro"]
    serial = {}
    for k in kinds:
        serial[k] = run(k)
        print("serial", k, len(serial[k]), flush=True)
    got, errs = {}, []

    def worker(t):
        try:
            for r in range(4):
                k = kinds[(t + r) % len(kinds)]
                got[(t, r)] = (k, run(k))
                print("thread", t, "round", r, k, flush=True)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    assert len(got) == 16
    for (t, r), (k, b) in got.items():
        assert b == serial[k], "thread %d round %d (%s) differs from the serial run" % (t, r, k)
    ctx.close()
