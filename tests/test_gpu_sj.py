"""GPU parity of Dynprog_end5/3_splicejunction (k_sj_plan, then k_fill's END = 2
segment fills on the register band or k_rows in segment mode, through the
C-ABI) against the reference's golden vectors and the CPU restatement they pin."""
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp import Context
from gsnapdp import workload as W
from gsnapdp.records import PAIR

pytestmark = pytest.mark.gpu

FIELDS = ("finalscore", "nmatches", "nmismatches", "nopens", "nindels")


def compare(res, pairs, npairs, ref, ref_pairs, ref_npairs, what):
    assert np.all(res["status"] != 2), "%s: op overflow" % what
    assert np.all(res["status"] != 4), "%s: unsupported windows %s" % (what, np.nonzero(res["status"] == 4)[0][:8])
    for f in FIELDS:
        bad = np.nonzero(res[f] != ref[f])[0]
        assert bad.size == 0, "%s: %s differs at %s (gpu %s ref %s)" % (what, f, bad[:8], res[f][bad[:8]],
                                                                      ref[f][bad[:8]])
    bad = np.nonzero(res["reserved"] != ref["dynprogindex"])[0]
    assert bad.size == 0, "%s: dynprogindex differs at %s" % (what, bad[:8])
    bad = np.nonzero(npairs != ref_npairs)[0]
    assert bad.size == 0, "%s: list length differs at %s (gpu %s ref %s)" % (what, bad[:8], npairs[bad[:8]],
                                                                            ref_npairs[bad[:8]])
    for f in PAIR.names:
        bad = np.nonzero(pairs[f] != ref_pairs[f])[0]
        assert bad.size == 0, "%s: pair field %s differs at pair %s" % (what, f, bad[:8])


def test_gpu_sj_matches_reference_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "sj_chr17.npz"), allow_pickle=False)
    ctx = Context(np.zeros(64, np.uint32))  # use_genomicseg_p: the context genome is never read
    w = z["windows"]
    res, ops, off = ctx.sj_run(w, z["query"], z["query_uc"])
    pairs, npairs = ctx.sj_all_pairs(w, z["query"], z["query_uc"], res, ops, off)
    ref = {f: z[f] for f in FIELDS + ("dynprogindex",)}
    compare(res, pairs, npairs, ref, z["pairs"], z["npairs"], "sj_chr17")


@pytest.mark.parametrize("seed", [51, 52])
def test_gpu_sj_matches_oracle_mix(seed):
    g = W.synthetic_genome(1_000_000, seed=seed, n_rate=0.002)
    b = W.sj_windows(g, 4000, seed=seed)
    ctx = Context(np.zeros(64, np.uint32))
    res, ops, off = ctx.sj_run(b.windows, b.query, b.query_uc)
    pairs, npairs = ctx.sj_all_pairs(b.windows, b.query, b.query_uc, res, ops, off)
    O.setup(np.zeros(16, np.uint32))
    ores, opairs, ooff, onp = O.run_sj_batch(b.windows, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    ref = {f: ores[f] for f in FIELDS}
    ref["dynprogindex"] = ores["reserved"]
    compare(res, pairs, npairs, ref, oflat, onp, "sj mix %d" % seed)
    assert np.sum(b.windows["length1"] > 64) > 100  # the 64-row stripe classes run too


def test_gpu_sj_register_band_matches_rowlane(monkeypatch):
    """The same splice-junction batch on the register band (k_fill's END = 2 fill
    over the segment) and on k_rows' segment mode (GSNAPDP_ENDS_ROWLANE=1):
    identical results, endpoints and pair lists."""
    g = W.synthetic_genome(1_000_000, seed=53, n_rate=0.002)
    b = W.sj_windows(g, 6000, seed=53)
    out = []
    for rowlane in ("0", "1"):
        monkeypatch.setenv("GSNAPDP_ENDS_ROWLANE", rowlane)
        ctx = Context(np.zeros(64, np.uint32))
        res, ops, off = ctx.sj_run(b.windows, b.query, b.query_uc)
        pairs, npairs = ctx.sj_all_pairs(b.windows, b.query, b.query_uc, res, ops, off)
        out.append((res, pairs, npairs))
    (r0, p0, n0), (r1, p1, n1) = out
    for f in FIELDS + ("bestr", "bestc", "status", "reserved", "nops"):
        bad = np.nonzero(r0[f] != r1[f])[0]
        assert bad.size == 0, "%s differs at %s (band %s rowlane %s)" % (f, bad[:8], r0[f][bad[:8]], r1[f][bad[:8]])
    assert np.array_equal(n0, n1) and all(np.array_equal(p0[f], p1[f]) for f in PAIR.names)
    assert np.sum(r0["status"] == 0) > 5000
