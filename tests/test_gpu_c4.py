"""BASELINE config 4 as stated on the GPU: synthetic 5 kbp transcripts
(workload.c4_transcripts) through the final intron pass (gsnapdp_stage3_pass,
build_pairs_introns with finalp, stage3.c:8860-8875) and score_introns
(gsnapdp_stage3_score_introns -> one k_introns launch, :9890-9941).

* the first 2000 transcripts against the reference's own build_pairs_introns /
  score_introns (tests/golden/c4_pinned.npz: counters, scores, list digests),
  through the three output forms of the pass (pairs, cells, runs with and
  without the caller's gap lists) and both score_introns entries;
* 10k transcripts against the CPU restatement of the pass (the same host code
  with the DP served by oracle/, oracle/_build/libstage3_cpu.so).  bench.py's
  c4_transcripts line checks all 50k the same way."""
import os
import sys

import numpy as np
import pytest

from gsnapdp import Context, expand_compact, expand_runs, gap_lists
from gsnapdp import workload as W
from test_c4_cpu import check_c4

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpu_c4_pinned_matches_reference(golden_dir):
    z = np.load(os.path.join(golden_dir, "c4_pinned.npz"), allow_pickle=False)
    w = W.c4_transcripts(int(z["n"]), seed=int(z["seed"]))
    ctx = Context(w.blocks)
    c, cells, new, st = ctx.stage3_pass_compact(w.calls, w.pairs_in, w.query, w.query_uc)
    lists = expand_compact(c, w.pairs_in, cells, new)
    scores = ctx.stage3_score_introns(c, lists)
    check_c4(z, c, lists, "gpu c4 (compact)", scores)
    c2, full, st2 = ctx.stage3_pass(w.calls, w.pairs_in, w.query, w.query_uc)
    assert full.tobytes() == lists.tobytes() and np.array_equal(c2["nout"], c["nout"])
    # the runs form, with the caller's gap lists and without (the pass finds them)
    gaps, gap_off = gap_lists(w.calls, w.pairs_in)
    for g, go in ((gaps, gap_off), (None, None)):
        c3, runs, new3, st3, _ = ctx.stage3_pass_runs(w.calls, w.pairs_in, w.query, w.query_uc, g, go)
        c3f, lists3 = expand_runs(c3, w.pairs_in, runs, new3)
        assert lists3.tobytes() == lists.tobytes() and np.array_equal(c3f["nout"], c["nout"])
        assert runs.size < lists.size // 50, (runs.size, lists.size)
        sc3 = ctx.stage3_score_introns_runs(c3, w.pairs_in, runs, new3, g, go)
        assert sc3.tobytes() == scores.tobytes()
    print("c4 pinned: %d transcripts, windows %s, %d new pairs, %d rounds" % (len(c), st["windows"],
                                                                             st["new_pairs"], st["rounds"]))
    ctx.close()


def test_gpu_c4_matches_cpu_restatement():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker
    w = W.c4_transcripts(10000)
    ctx = Context(w.blocks)
    c, cells, new, st = ctx.stage3_pass_compact(w.calls, w.pairs_in, w.query, w.query_uc)
    cpu = O.Stage3Cpu(w.blocks)
    rc, rcells, rnew, rst = cpu.run_compact(w.calls, w.pairs_in, w.query, w.query_uc)
    cpu.close()
    for f in ("out_minor", "out_major", "out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen",
              "shiftp", "incompletep", "nout", "first_out", "status", "ub"):
        assert np.array_equal(c[f], rc[f]), f
    assert np.array_equal(cells, rcells) and new.tobytes() == rnew.tobytes()
    assert list(st["windows"]) == list(rst["windows"])
    gaps, gap_off = gap_lists(w.calls, w.pairs_in)
    c3, runs, new3, st3, _ = ctx.stage3_pass_runs(w.calls, w.pairs_in, w.query, w.query_uc, gaps, gap_off)
    c3f, lists3 = expand_runs(c3, w.pairs_in, runs, new3)
    assert lists3.tobytes() == expand_compact(c, w.pairs_in, cells, new).tobytes()
    ctx.close()
