"""GPU parity of Dynprog_genome_gap (k_ggap_plan + k_ggap, through the C-ABI)
against the reference's golden vectors and the CPU restatement they pin."""
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp import Context
from gsnapdp import workload as W
from gsnapdp.records import PAIR

pytestmark = pytest.mark.gpu

ALWAYS = ("finalscore", "nmatches", "nmismatches", "nopens", "nindels", "dynprogindex",
          "returned_null", "bridge_ok")
WITH_LIST = ("new_leftgenomepos", "new_rightgenomepos", "exonhead", "introntype")


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)


def unsupported_expected(w):
    """Windows outside the reference's domain: it aborts (non-positive flank)
    or its bridge reads diagonal cells past a flank's matrix rows."""
    L1, L2L, L2R = (w[f].astype(np.int64) for f in ("length1", "length2L", "length2R"))
    early = (L1 <= 1) | (L1 > w["maxlength1"]) | (L2L > w["maxlength2"]) | (L2R > w["maxlength2"])
    return ~early & ((L2L <= 0) | (L2R <= 0) | (w["extraband_paired"] < 0) | (L2L < L1 - 1) | (L2R < L1 - 1))


def compare(w, res, trc, pairs, npairs, ref, ref_pairs, ref_npairs, what):
    uns = unsupported_expected(w)
    assert np.array_equal(trc["status"] == 4, uns), "%s: unsupported set differs" % what
    assert np.all(trc["status"] != 2), "%s: op stream overflow" % what
    ok = ~uns
    for f in ALWAYS:
        bad = np.nonzero((res[f] != ref[f]) & ok)[0]
        assert bad.size == 0, "%s: %s differs at %s (gpu %s ref %s)" % (
            what, f, bad[:8], res[f][bad[:8]], ref[f][bad[:8]])
    nn = ok & (ref["returned_null"] == 0)
    for f in WITH_LIST:
        bad = np.nonzero((res[f] != ref[f]) & nn)[0]
        assert bad.size == 0, "%s: %s differs at %s" % (what, f, bad[:8])
    for f in ("left_prob", "right_prob"):
        bad = np.nonzero((res[f].view(np.uint64) != ref[f].view(np.uint64)) & ok)[0]
        assert bad.size == 0, "%s: %s differs at %s" % (what, f, bad[:8])
    bad = np.nonzero((npairs != ref_npairs) & ok)[0]
    assert bad.size == 0, "%s: list length differs at %s (gpu %s ref %s)" % (
        what, bad[:8], npairs[bad[:8]], ref_npairs[bad[:8]])
    goff = np.concatenate([[0], np.cumsum(npairs)])
    roff = np.concatenate([[0], np.cumsum(ref_npairs)])
    sel = np.nonzero(ok)[0]
    got = np.concatenate([pairs[goff[i]:goff[i + 1]] for i in sel] + [np.zeros(0, PAIR)])
    exp = np.concatenate([ref_pairs[roff[i]:roff[i + 1]] for i in sel] + [np.zeros(0, PAIR)])
    for f in PAIR.names:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, "%s: pair field %s differs at pair %s" % (what, f, bad[:8])


def run_gpu(blocks, b):
    ctx = Context(blocks)
    res, trc, ops, off = ctx.ggap_run(b.windows, b.query, b.query_uc)
    pairs, npairs = ctx.ggap_all_pairs(b.windows, b.query, b.query_uc, res, trc, ops, off)
    return res, trc, pairs, npairs


GOLDEN = ["ggap_chr17", "gmap_synth_ggap", "gmap_her2_ggap",
          # a splicing IIT (reference iit_store) given to Dynprog_setup: site-level and
          # intron-level, novel splicing on and off (dynprog.c:3375-3697, :4084-4101)
          "ggap_known_sites", "ggap_known_sites_novel", "ggap_known_introns",
          "ggap_known_introns_novel"]


@pytest.mark.parametrize("name", GOLDEN)
def test_gpu_ggap_matches_reference_golden(golden_dir, name):
    z = load(golden_dir, name)
    ctx = Context(z["blocks"])
    assert "gfx950" in ctx.arch
    w = z["windows"]
    res, trc, ops, off = ctx.ggap_run(w, z["query"], z["query_uc"])
    pairs, npairs = ctx.ggap_all_pairs(w, z["query"], z["query_uc"], res, trc, ops, off)
    compare(w, res, trc, pairs, npairs, z["results"], z["pairs"], z["npairs"], name)
    assert np.sum(z["results"]["returned_null"] == 0) > len(w) // 2 and z["pairs"].size > 1000


@pytest.mark.parametrize("name", GOLDEN)
def test_gpu_gband_matches_reference_golden(golden_dir, name, monkeypatch):
    """The goldens with every qualifying score-mode window on the register band
    (GSNAPDP_GBAND_MIN=0; by default batches under 16384 windows run on k_ggap)."""
    monkeypatch.setenv("GSNAPDP_GBAND_MIN", "0")
    z = load(golden_dir, name)
    ctx = Context(z["blocks"])
    w = z["windows"]
    res, trc, ops, off = ctx.ggap_run(w, z["query"], z["query_uc"])
    pairs, npairs = ctx.ggap_all_pairs(w, z["query"], z["query_uc"], res, trc, ops, off)
    compare(w, res, trc, pairs, npairs, z["results"], z["pairs"], z["npairs"], name + " (band)")


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_gpu_ggap_matches_oracle_mix(seed):
    """Every class (rows <= 31, <= 63, striped), both modes, odd shapes, early returns."""
    g, b = W.ggap_windows(W.synthetic_genome(2_000_000, seed=seed, n_rate=0.002), 3000, seed=seed)
    blocks = W.pack_genome(g)
    res, trc, pairs, npairs = run_gpu(blocks, b)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(b.windows, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(b.windows, res, trc, pairs, npairs, ores, oflat, onp, "mix seed %d" % seed)
    # the mix reaches every class with returned lists, in both bridge modes
    L1 = b.windows["length1"]
    listed = ores["returned_null"] == 0
    for lo, hi in ((2, 32), (32, 64), (64, 400)):
        assert np.sum(listed & (L1 >= lo) & (L1 < hi)) > 20, (lo, hi)
    assert np.sum(listed & (b.windows["use_probabilities_p"] == 1)) > 100
    assert np.sum(ores["bridge_ok"] == 0) > 0 and np.sum(trc["status"] == 1) > 0


@pytest.mark.parametrize("site_level,novel", [(True, False), (True, True), (False, False),
                                              (False, True)])
def test_gpu_ggap_known_sites_matches_oracle_mix(site_level, novel):
    """Known-site modes in every storage class (rows <= 31, <= 63, striped)."""
    g, b = W.ggap_windows(W.synthetic_genome(2_000_000, seed=21, n_rate=0.002), 1500, seed=21)
    blocks = W.pack_genome(g)
    O.setup(blocks)
    ores0, _, _, _ = O.run_ggap_batch(b.windows, b.query, b.query_uc)
    sites = W.SpliceSiteSet(W.known_site_intervals(b.windows, ores0, np.random.default_rng(5),
                                                   site_level))
    w, q, u = W.with_known_sites(b.windows, b.query, b.query_uc, sites, novel)
    ctx = Context(blocks)
    res, trc, ops, off = ctx.ggap_run(w, q, u)
    pairs, npairs = ctx.ggap_all_pairs(w, q, u, res, trc, ops, off)
    ores, opairs, ooff, onp = O.run_ggap_batch(w, q, u)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(w, res, trc, pairs, npairs, ores, oflat, onp, "known %d %d" % (site_level, novel))
    assert np.sum(ores["returned_null"] == 0) > 200
    L1 = w["length1"]
    assert np.sum((ores["returned_null"] == 0) & (L1 >= 64)) > 5


@pytest.mark.parametrize("prob", [False, True])
def test_gpu_c4_parity(prob):
    """BASELINE config 4 shape, score and probability modes."""
    g, b = W.c4_windows(W.synthetic_genome(8_000_000, seed=4), 20_000, seed=4, use_probabilities=prob)
    blocks = W.pack_genome(g)
    res, trc, pairs, npairs = run_gpu(blocks, b)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(b.windows, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(b.windows, res, trc, pairs, npairs, ores, oflat, onp, "C4 prob=%s" % prob)
    assert np.mean(ores["returned_null"] == 0) > 0.8 and oflat.size > 20 * len(b.windows)


@pytest.mark.parametrize("n", [1, 5, 17, 33])
def test_gpu_ggap_ragged_batches_with_shadow_groups(n, monkeypatch):
    """Batches that leave window groups of a register-band wave empty: the
    shadow groups replay the task's first window (here at query offset 0)
    without touching memory outside the batch (GSNAPDP_GBAND_MIN=0: batches
    this small run on the register band too)."""
    monkeypatch.setenv("GSNAPDP_GBAND_MIN", "0")
    g, b = W.c4_windows(W.synthetic_genome(2_000_000, seed=9), 64, seed=9, use_probabilities=False)
    w = b.windows[:n].copy()
    assert w["qpos"][0] == 0
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    res, trc, ops, off = ctx.ggap_run(w, b.query, b.query_uc)
    pairs, npairs = ctx.ggap_all_pairs(w, b.query, b.query_uc, res, trc, ops, off)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(w, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(w, res, trc, pairs, npairs, ores, oflat, onp, "ragged %d" % n)


@pytest.mark.parametrize("jl", ["mixed", "all"])
def test_gpu_gband_jump_late_batches(jl):
    """Round-3 regression for the k_gband fault of round 2 (DESIGN.md §4 k_gband):
    register-band genome gaps with jump_late_p = 1 in every band class, in a
    batch large enough to reuse every wave's scratch several times.  A build
    that corrupted a long-lived window field produced wrong new_leftgenomepos
    here; the kernel's invariant guard turns a bad bridge cell into an error."""
    rng = np.random.default_rng(77)
    g, b = W.c4_windows(W.synthetic_genome(16_000_000, seed=4), 100_000, seed=4)
    w = b.windows.copy()
    w["jump_late_p"] = rng.integers(0, 2, len(w)) if jl == "mixed" else 1
    # wider bands too (the S = 8 classes): extraband_paired 10 on a third of the windows
    w["extraband_paired"][::3] = 10
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    res, trc, ops, off = ctx.ggap_run(w, b.query, b.query_uc)
    pairs, npairs = ctx.ggap_all_pairs(w, b.query, b.query_uc, res, trc, ops, off)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(w, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(w, res, trc, pairs, npairs, ores, oflat, onp, "jump-late %s" % jl)


@pytest.mark.parametrize("name", ["ggap_chr17", "gmap_synth_ggap", "gmap_her2_ggap", "ggap_known_sites",
                                  "ggap_known_sites_novel"])
def test_gpu_gband_probability_mode_matches_reference_golden(golden_dir, name, monkeypatch):
    """Probability-mode windows on the register band (GSNAPDP_GBAND_PROB=1:
    the fills' cell values and the bridge sweeps of gsnapdp_gband.hip) against
    the reference's goldens."""
    monkeypatch.setenv("GSNAPDP_GBAND_PROB", "1")
    monkeypatch.setenv("GSNAPDP_GBAND_MIN", "0")
    z = load(golden_dir, name)
    ctx = Context(z["blocks"])
    w = z["windows"]
    res, trc, ops, off = ctx.ggap_run(w, z["query"], z["query_uc"])
    pairs, npairs = ctx.ggap_all_pairs(w, z["query"], z["query_uc"], res, trc, ops, off)
    compare(w, res, trc, pairs, npairs, z["results"], z["pairs"], z["npairs"], name + " (band prob)")


@pytest.mark.parametrize("jl", ["none", "mixed"])
def test_gpu_gband_probability_mode_matches_oracle(jl, monkeypatch):
    """C4-shape probability-mode windows on the register band, jump-late mixed,
    a third with extraband 10 (the S = 8 classes), against the oracle."""
    monkeypatch.setenv("GSNAPDP_GBAND_PROB", "1")
    monkeypatch.setenv("GSNAPDP_GBAND_MIN", "0")
    rng = np.random.default_rng(78)
    g, b = W.c4_windows(W.synthetic_genome(8_000_000, seed=5), 20_000, seed=5, use_probabilities=True)
    w = b.windows.copy()
    if jl == "mixed":
        w["jump_late_p"] = rng.integers(0, 2, len(w))
        w["extraband_paired"][::3] = 10
    blocks = W.pack_genome(g)
    res, trc, pairs, npairs = run_gpu(blocks, W.Batch(w, b.query, b.query_uc))
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(w, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(w, res, trc, pairs, npairs, ores, oflat, onp, "band prob %s" % jl)
    assert np.mean(ores["returned_null"] == 0) > 0.5


@pytest.mark.parametrize("jl", ["none", "mixed"])
def test_gpu_gwin_probability_mode_matches_oracle(jl):
    """Probability-mode windows on k_gwin (one window per lane, the default for
    them): both of its band shapes (extraband_paired 7 and 3), jump-late mixed,
    against the oracle; the k_gwin stage must have run."""
    rng = np.random.default_rng(79)
    g, b = W.c4_windows(W.synthetic_genome(8_000_000, seed=6), 20_000, seed=6, use_probabilities=True)
    w = b.windows.copy()
    w["extraband_paired"][1::3] = 3
    if jl == "mixed":
        w["jump_late_p"] = rng.integers(0, 2, len(w))
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    names = ctx.profile(True)
    res, trc, ops, off = ctx.ggap_run(w, b.query, b.query_uc)
    acc = np.zeros(len(names))
    ctx.profile_read(acc)
    ctx.profile(False)
    assert acc[names.index("k_gwin")] > 0, "k_gwin did not run"
    pairs, npairs = ctx.ggap_all_pairs(w, b.query, b.query_uc, res, trc, ops, off)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(w, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(w, res, trc, pairs, npairs, ores, oflat, onp, "gwin prob %s" % jl)
    assert np.mean(ores["returned_null"] == 0) > 0.5


@pytest.mark.parametrize("name", ["ggap_chr17", "gmap_synth_ggap", "gmap_her2_ggap"])
def test_gpu_gwin_matches_reference_golden(golden_dir, name, monkeypatch):
    """The goldens with every qualifying probability-mode window on k_gwin
    (GSNAPDP_GWIN_MIN=0; by default batches under 16384 windows run on k_ggap)."""
    monkeypatch.setenv("GSNAPDP_GWIN_MIN", "0")
    z = load(golden_dir, name)
    ctx = Context(z["blocks"])
    w = z["windows"]
    res, trc, ops, off = ctx.ggap_run(w, z["query"], z["query_uc"])
    pairs, npairs = ctx.ggap_all_pairs(w, z["query"], z["query_uc"], res, trc, ops, off)
    compare(w, res, trc, pairs, npairs, z["results"], z["pairs"], z["npairs"], name + " (gwin)")


@pytest.mark.parametrize("seed", [11, 12])
def test_gpu_gwin_matches_oracle_mix(seed, monkeypatch):
    """The mixed sets (every shape, both modes) with k_gwin taking what qualifies."""
    monkeypatch.setenv("GSNAPDP_GWIN_MIN", "0")
    g, b = W.ggap_windows(W.synthetic_genome(2_000_000, seed=seed, n_rate=0.002), 3000, seed=seed)
    blocks = W.pack_genome(g)
    res, trc, pairs, npairs = run_gpu(blocks, b)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(b.windows, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    compare(b.windows, res, trc, pairs, npairs, ores, oflat, onp, "gwin mix seed %d" % seed)


@pytest.mark.parametrize("length1,eb", [(2, 7), (5, 3), (13, 7), (24, 7), (24, 3), (16, 3)])
def test_gpu_gwin_shapes_match_oracle(length1, eb, monkeypatch):
    """k_gwin at the edges of its window shapes: length1 2 .. 24 (flanks of
    length1 + 8), both band shapes, jump-late mixed, a tenth of the windows at
    the genome's start (site positions below the MaxEnt margins: the per-site
    path of k_gwin_probs), against the oracle (GSNAPDP_GWIN_MIN=0)."""
    monkeypatch.setenv("GSNAPDP_GWIN_MIN", "0")
    rng = np.random.default_rng(length1 * 100 + eb)
    g, b = W.c4_windows(W.synthetic_genome(4_000_000, seed=length1), 3000, seed=length1,
                        use_probabilities=True, length1=length1, extraband=eb)
    w = b.windows.copy()
    w["jump_late_p"] = rng.integers(0, 2, len(w))
    w["chrpos"][::10] = rng.integers(0, 12, len(w[::10]))
    blocks = W.pack_genome(g)
    ctx = Context(blocks)
    names = ctx.profile(True)
    res, trc, ops, off = ctx.ggap_run(w, b.query, b.query_uc)
    acc = np.zeros(len(names))
    ctx.profile_read(acc)
    ctx.profile(False)
    assert acc[names.index("k_gwin")] > 0, "k_gwin did not run"
    pairs, npairs = ctx.ggap_all_pairs(w, b.query, b.query_uc, res, trc, ops, off)
    O.setup(blocks)
    ores, opairs, ooff, onp = O.run_ggap_batch(w, b.query, b.query_uc)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))] + [np.zeros(0, PAIR)])
    compare(w, res, trc, pairs, npairs, ores, oflat, onp, "gwin L1 %d eb %d" % (length1, eb))
