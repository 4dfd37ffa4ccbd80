"""GPU parity of Dynprog_cdna_gap (k_cgap_plan + k_cgap, through the C-ABI)
against the reference's golden vectors and the CPU restatement they pin."""
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp import Context
from gsnapdp import workload as W
from gsnapdp.records import PAIR

pytestmark = pytest.mark.gpu

FIELDS = ("finalscore", "finalscore_set", "dynprogindex", "incompletep", "returned_null")


def compare(res, pairs, npairs, ref, ref_pairs, ref_npairs, what, ub_ok=False):
    ok = np.ones(len(res), bool) if not ub_ok else ref["status"] != 5
    assert np.all(res["status"][ok] != 2), "%s: op overflow" % what
    for f in FIELDS:
        bad = np.nonzero((res[f] != ref[f]) & ok)[0]
        assert bad.size == 0, "%s: %s differs at %s (gpu %s ref %s)" % (what, f, bad[:8], res[f][bad[:8]],
                                                                      ref[f][bad[:8]])
    bad = np.nonzero((npairs != ref_npairs) & ok)[0]
    assert bad.size == 0, "%s: list length differs at %s (gpu %s ref %s)" % (what, bad[:8], npairs[bad[:8]],
                                                                            ref_npairs[bad[:8]])
    goff = np.concatenate([[0], np.cumsum(npairs)])
    roff = np.concatenate([[0], np.cumsum(ref_npairs)])
    sel = np.nonzero(ok)[0]
    got = np.concatenate([pairs[goff[i]:goff[i + 1]] for i in sel] + [np.zeros(0, PAIR)])
    exp = np.concatenate([ref_pairs[roff[i]:roff[i + 1]] for i in sel] + [np.zeros(0, PAIR)])
    for f in PAIR.names:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, "%s: pair field %s differs at pair %s" % (what, f, bad[:8])


def test_gpu_cgap_matches_reference_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "cgap_chr17.npz"), allow_pickle=False)
    ctx = Context(z["blocks"])
    w = z["windows"]
    res, ops, off = ctx.cgap_run(w, z["query"], z["query_uc"])
    pairs, npairs = ctx.cgap_all_pairs(w, z["query"], z["query_uc"], res, ops, off, z["gseg"], z["gseg_off"])
    compare(res, pairs, npairs, z["results"], z["pairs"], z["npairs"], "cgap_chr17")
    assert res["insert_pairs"].sum() > 20


@pytest.mark.parametrize("seed,max_gap", [(41, 40), (42, 120)])
def test_gpu_cgap_matches_oracle_mix(seed, max_gap):
    g = W.synthetic_genome(2_000_000, seed=seed, n_rate=0.002)
    b = W.cgap_windows(g, 2500, seed=seed, max_gap=max_gap)
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    res, ops, off = ctx.cgap_run(b.windows, b.query, b.query_uc)
    pairs, npairs = ctx.cgap_all_pairs(b.windows, b.query, b.query_uc, res, ops, off, b.gseg, b.gseg_off)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_cgap_batch(b.windows, b.query, b.query_uc, b.gseg, b.gseg_off)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    assert np.array_equal(res["status"] == 5, ores["status"] == 5)
    compare(res, pairs, npairs, ores, oflat, onp, "cgap mix %d" % seed, ub_ok=True)
    G = b.windows["length2"]
    if max_gap > 64:  # every class: 32-row groups, 64-row stripes in LDS, global scratch
        assert np.sum(G > 70) > 50 and np.sum(G < 30) > 200
