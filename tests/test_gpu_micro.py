"""GPU parity of Dynprog_microexon_int (k_micro, through the C-ABI) against
the reference's golden vectors and the CPU restatement they pin."""
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp import Context
from gsnapdp import workload as W
from gsnapdp.records import PAIR

pytestmark = pytest.mark.gpu


def compare(res, pairs, npairs, ref, ref_pairs, ref_npairs, what):
    assert np.all(res["status"] == 0), "%s: unsupported %s" % (what, np.nonzero(res["status"])[0][:8])
    for f in ("microintrontype", "dynprogindex", "found"):
        bad = np.nonzero(res[f] != ref[f])[0]
        assert bad.size == 0, "%s: %s differs at %s (gpu %s ref %s)" % (what, f, bad[:8], res[f][bad[:8]],
                                                                      ref[f][bad[:8]])
    for f in ("bestprob2", "bestprob3"):
        bad = np.nonzero(res[f].view(np.uint64) != ref[f].view(np.uint64))[0]
        assert bad.size == 0, "%s: %s differs at %s" % (what, f, bad[:8])
    bad = np.nonzero(npairs != ref_npairs)[0]
    assert bad.size == 0, "%s: list length differs at %s" % (what, bad[:8])
    for f in PAIR.names:
        bad = np.nonzero(pairs[f] != ref_pairs[f])[0]
        assert bad.size == 0, "%s: pair field %s differs at pair %s" % (what, f, bad[:8])


def test_gpu_micro_matches_reference_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "micro_chr17.npz"), allow_pickle=False)
    ctx = Context(z["blocks"])
    res = ctx.micro_run(z["windows"], z["query"], z["query_uc"])
    pairs, npairs = ctx.micro_all_pairs(z["windows"], z["query"], z["query_uc"], res)
    compare(res, pairs, npairs, z["results"], z["pairs"], z["npairs"], "micro_chr17")
    assert res["found"].sum() > 500


@pytest.mark.parametrize("seed", [61, 62])
def test_gpu_micro_matches_oracle_mix(seed):
    g0 = W.synthetic_genome(600_000, seed=seed, n_rate=0.002)
    g, b = W.micro_windows(g0, 3000, seed=seed)
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    res = ctx.micro_run(b.windows, b.query, b.query_uc)
    pairs, npairs = ctx.micro_all_pairs(b.windows, b.query, b.query_uc, res)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_micro_batch(b.windows, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(res, pairs, npairs, ores, oflat, onp, "micro mix %d" % seed)
