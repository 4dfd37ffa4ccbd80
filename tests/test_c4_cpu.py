"""BASELINE config 4 as stated: 50k synthetic 5 kbp transcripts
through GMAP's final intron pass (build_pairs_introns with finalp,
stage3.c:8860-8875) and score_introns (:9890-9941) -- the generator
(workload.c4_transcripts) and the pass's host control flow on the CPU.

tests/golden/c4_pinned.npz holds what the reference's own build_pairs_introns
and score_introns returned for the first 2000 transcripts (oracle/s3_replay.c;
oracle/gen_golden.py c4_pinned_case): counters, scores and a sha256 of every
returned list.  The generator is prefix-stable, so the tests regenerate the
inputs from the seed.  tests/test_gpu_c4.py runs the same on the GPU."""
import hashlib
import os

import numpy as np

from gsnapdp import workload as W
from test_stage3_cpu import run_stage3_cpu

COUNTERS = ["out_minor", "out_major", "out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen",
            "shiftp", "incompletep", "nout"]


def check_c4(z, calls, lists, what, scores=None):
    """counters, list digests (and score_introns) against the reference's"""
    n = len(calls)
    assert (calls["status"] == 0).all(), what
    ub = (calls["ub"] & 1) != 0
    for f in COUNTERS:
        skip = ub if f in ("out_intronlen", "out_nonintronlen") else np.zeros(n, bool)
        bad = np.nonzero((calls[f] != z["ref_" + f][:n]) & ~skip)[0]
        assert bad.size == 0, "%s: %s differs at calls %s" % (what, f, bad[:8])
    bad = [i for i in range(n) if hashlib.sha256(
        lists[int(calls["first_out"][i]):int(calls["first_out"][i]) + int(calls["nout"][i])].tobytes()).digest()
        != z["digests"][i].tobytes()]
    assert not bad, "%s: lists differ at calls %s" % (what, bad[:8])
    if scores is not None:
        si = z["si_calls"][:n]
        for f in ("avg_donor_score", "avg_acceptor_score"):
            d = np.nonzero(scores[f].view(np.uint64) != si[f].astype(np.float64).view(np.uint64))[0]
            assert d.size == 0, "%s: %s differs at calls %s" % (what, f, d[:8])
        assert np.array_equal(scores["nbadintrons"], si["nbadintrons"]), what


def test_c4_generator_shape_and_prefix():
    """transcript sizes as stated, one gapholder per intron, the path in reversed
    alignment order, and the prefix property the pinned set relies on"""
    w = W.c4_transcripts(40)
    c = w.calls
    assert (c["querylength"] >= 4500).all() and (c["querylength"] <= 5500).all()
    nex = c["npairs"] - c["querylength"] + 1
    assert (nex >= 8).all() and (nex <= 12).all()
    for i in range(len(c)):
        x = w.pairs_in[int(c["first_pair"][i]):int(c["first_pair"][i]) + int(c["npairs"][i])]
        g = (x["flags"] & 1) != 0
        assert g.sum() == nex[i] - 1
        y = x[~g]
        assert np.array_equal(y["querypos"], np.arange(c["querylength"][i])[::-1])
        assert (np.diff(y["genomepos"]) < 0).all()
        jumps = x["genomejump"][g]
        assert (jumps >= 80 - 12).all() and (jumps <= 5000 + 12).all()
    v = W.c4_transcripts(15)
    n = int(v.calls["npairs"].sum())
    assert v.pairs_in.tobytes() == w.pairs_in[:n].tobytes()
    assert np.array_equal(v.calls["chrpos"], w.calls["chrpos"][:15])


def test_c4_pass_cpu_matches_reference_prefix(golden_dir, tmp_path):
    """the first 150 pinned transcripts through the pass (ASan + UBSan, the DP
    served by the restatement) and score_introns on its lists"""
    z = np.load(os.path.join(golden_dir, "c4_pinned.npz"), allow_pickle=False)
    w = W.c4_transcripts(150, seed=int(z["seed"]))
    calls, lists, st, scores = run_stage3_cpu(str(tmp_path), {"blocks": w.blocks}, w.calls, w.pairs_in, w.query,
                                              w.query_uc, introns=True)
    check_c4(z, calls, lists, "c4 prefix", scores)
    assert st["windows"][1] > 0


def test_c4_runs_cpu_matches_reference_prefix(golden_dir):
    """the runs output (gsnapdp_stage3_pass_runs, the caller's gap lists) and
    score_introns on the runs, the DP served by the restatement
    (oracle/_build/libstage3_cpu.so): the same lists and scores as the reference's"""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle as O  # checker
    from gsnapdp import expand_runs, gap_lists
    z = np.load(os.path.join(golden_dir, "c4_pinned.npz"), allow_pickle=False)
    w = W.c4_transcripts(300, seed=int(z["seed"]))
    gaps, gap_off = gap_lists(w.calls, w.pairs_in)
    S = O.Stage3Cpu(w.blocks)
    try:
        for g, go in ((gaps, gap_off), (None, None)):
            c, runs, new, st, sc = S.run_runs(w.calls, w.pairs_in, w.query, w.query_uc, g, go, introns=True)
            cf, lists = expand_runs(c, w.pairs_in, runs, new)
            for f in ("first_out", "nout"):
                c[f] = cf[f]
            check_c4(z, c, lists, "c4 runs", sc)
            assert runs.size < lists.size // 50
    finally:
        S.close()
