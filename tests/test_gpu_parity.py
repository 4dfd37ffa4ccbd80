"""GPU parity: the HIP path (through the C-ABI) against the reference's golden
vectors and against the CPU restatement (which the golden vectors pin)."""
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp import Context
from gsnapdp import workload as W
from gsnapdp.records import END3_GAP, END5_GAP, PAIR

pytestmark = pytest.mark.gpu

DP_CASES = ["dp_chr17_mix", "dp_synth_mix", "dp_synth_cmet", "dp_chr17_c2", "dp_synth_long",
            "gmap_synth_gap", "gmap_her2_gap"]  # the last two: windows the reference gmap issued (oracle/gmap_trace.c)


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)


def compare(res, gpu_pairs, gpu_np, ref_scores, ref_pairs, ref_np, what):
    for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels"):
        bad = np.nonzero(res[f] != ref_scores[f])[0]
        assert bad.size == 0, "%s: %s differs at windows %s (gpu %s ref %s)" % (
            what, f, bad[:8], res[f][bad[:8]], ref_scores[f][bad[:8]])
    bad = np.nonzero(res["reserved"] != ref_scores["dynprogindex"])[0]
    assert bad.size == 0, "%s: dynprogindex differs at %s" % (what, bad[:8])
    bad = np.nonzero(gpu_np != ref_np)[0]
    assert bad.size == 0, "%s: list length differs at windows %s (gpu %s ref %s)" % (
        what, bad[:8], gpu_np[bad[:8]], ref_np[bad[:8]])
    for f in PAIR.names:
        bad = np.nonzero(gpu_pairs[f] != ref_pairs[f])[0]
        assert bad.size == 0, "%s: pair field %s differs at pair %s" % (what, f, bad[:8])


@pytest.mark.parametrize("name", DP_CASES)
def test_gpu_matches_reference_golden(golden_dir, name):
    z = load(golden_dir, name)
    ctx = Context(z["blocks"], mode=int(z["mode"]))
    assert "gfx950" in ctx.arch
    res, ops, off = ctx.run(z["windows"], z["query"], z["query_uc"])
    assert np.all(res["status"] != 2), "op stream overflow"
    pairs, npairs = ctx.all_pairs(z["windows"], z["query"], z["query_uc"], res, ops, off)
    ref = {f: z[f] for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels", "dynprogindex")}
    compare(res, pairs, npairs, ref, z["pairs"], z["npairs"], name)


def run_both(blocks, batch, mode=0, threads=16):
    ctx = Context(blocks, mode=mode)
    res, ops, off = ctx.run(batch.windows, batch.query, batch.query_uc)
    pairs, npairs = ctx.all_pairs(batch.windows, batch.query, batch.query_uc, res, ops, off)
    O.setup(blocks, mode=mode)
    ores, opairs, ooff, onp = O.run_batch(batch.windows, batch.query, batch.query_uc, nthreads=threads)
    oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
    ref = {f: ores[f] for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels")}
    ref["dynprogindex"] = ores["reserved"]
    return res, pairs, npairs, ref, oflat, onp


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_matches_oracle_random(seed):
    g = W.synthetic_genome(2_000_000, seed=100 + seed, n_rate=0.002)
    blocks = W.pack_genome(g)
    batch = W.random_windows(g, 6000, seed=seed, max_len1=120, max_len2=140, max_band=20)
    res, pairs, npairs, ref, oflat, onp = run_both(blocks, batch)
    compare(res, pairs, npairs, ref, oflat, onp, "random seed %d" % seed)


def test_gpu_matches_oracle_wide_and_long():
    g = W.synthetic_genome(1_000_000, seed=7, n_rate=0.002)
    blocks = W.pack_genome(g)
    batch = W.random_windows(g, 400, seed=9, max_len1=700, max_len2=900, max_band=60)
    res, pairs, npairs, ref, oflat, onp = run_both(blocks, batch)
    compare(res, pairs, npairs, ref, oflat, onp, "wide/long")


def test_gpu_c2_full_size_parity():
    """BASELINE config 2 at full size: 100k x 150 bp, band 31, bit-exact."""
    g = W.synthetic_genome(64_000_000, seed=1)
    blocks = W.pack_genome(g)
    batch = W.c2_windows(g, n=100_000, seed=2)
    res, pairs, npairs, ref, oflat, onp = run_both(blocks, batch, threads=32)
    compare(res, pairs, npairs, ref, oflat, onp, "C2 100k")


@pytest.mark.parametrize("name", ["maxent_chr17", "maxent_synth"])
def test_gpu_maxent_matches_reference(golden_dir, name):
    z = load(golden_dir, name)
    ctx = Context(z["blocks"])
    got = ctx.maxent(z["model"], z["splice_pos"], z["chroffset"])
    ref = z["prob"]
    bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0]
    assert bad.size == 0, "maxent differs at %s" % bad[:10]


def rows_class(L1, L2, W):
    """gsnapdp_device.h rows_class: 4 tiny (LDS, 16-row groups), 0 small (LDS,
    32-row groups), 1 mid (LDS, 64-row stripes), 2 big (global scratch)."""
    stripes = (L1 + 1 + 63) // 64
    words = L1 * W + (L2 + 2 + 3) // 4 + (L1 + 1) // 2 + (3 * (L2 + 2) if stripes > 1 else 0)
    if L1 + 1 <= 16 and words <= 640:
        return 4
    if L1 + 1 <= 32 and words <= 1280:
        return 0
    return 1 if words <= 4096 else 2


@pytest.mark.parametrize("seed", [21, 22])
def test_gpu_end_gaps_every_row_class(seed):
    """End gaps (all endpoint modes, both ends) short, striped-in-LDS and global."""
    g = W.synthetic_genome(2_000_000, seed=200 + seed, n_rate=0.002)
    blocks = W.pack_genome(g)
    parts = [W.random_windows(g, 1500, seed=seed * 10 + k, kinds=(END5_GAP, END3_GAP), max_len1=m1,
                              max_len2=m1 + 20, max_band=b)
             for k, (m1, b) in enumerate(((30, 6), (250, 5), (600, 12)))]
    batch = W.concat_batches(parts)
    w = batch.windows
    L1, L2 = w["length1"].astype(np.int64), w["length2"].astype(np.int64)
    eb = w["extraband"].astype(np.int64)
    Wd = np.abs(L2 - L1) + 2 * eb + 1
    cls = np.array([rows_class(a, b, c) for a, b, c in zip(L1, L2, Wd)])
    assert all(np.sum(cls == c) > 50 for c in (0, 1, 2, 4)), np.bincount(cls)
    res, pairs, npairs, ref, oflat, onp = run_both(blocks, batch)
    compare(res, pairs, npairs, ref, oflat, onp, "end gaps seed %d" % seed)


def test_gpu_c5_gsnap_windows_parity():
    """BASELINE config 5's DP windows: 100 bp single gaps (extraband 3) and end5 / end3 gaps."""
    g = W.synthetic_genome(8_000_000, seed=5)
    blocks = W.pack_genome(g)
    batch = W.c5_windows(g, 20_000, seed=5)
    res, pairs, npairs, ref, oflat, onp = run_both(blocks, batch)
    compare(res, pairs, npairs, ref, oflat, onp, "C5 windows")
    assert np.sum(onp) > 60 * 20_000


@pytest.mark.parametrize("seed", [31, 32])
def test_gpu_end_gaps_on_register_band(seed, monkeypatch):
    """find_best_endpoint end gaps (QUERYEND_GAP, BEST_LOCAL) on k_fill's END fill:
    both ends and tie rules, extraband 0-12, L1 up to 300, and a low-complexity
    genome stretch so that many cells tie for the best score (the scan's
    row-major order decides).  The same batch through k_rows
    (GSNAPDP_ENDS_ROWLANE=1) and the restatement must agree bit for bit."""
    g = W.synthetic_genome(2_000_000, seed=300 + seed, n_rate=0.002)
    g[:400_000] = np.resize(np.frombuffer(b"AACAC", np.uint8), 400_000)  # repeats: ties
    blocks = W.pack_genome(g)
    parts = [W.random_windows(g, 2500, seed=seed * 10 + k, kinds=(END5_GAP, END3_GAP), max_len1=m1,
                              max_len2=m1 + 24, max_band=b, endaligns=(W.QUERYEND_GAP, W.BEST_LOCAL))
             for k, (m1, b) in enumerate(((30, 12), (120, 6), (300, 3)))]
    batch = W.concat_batches(parts)
    res, pairs, npairs, ref, oflat, onp = run_both(blocks, batch)
    compare(res, pairs, npairs, ref, oflat, onp, "end gaps on the band seed %d" % seed)
    monkeypatch.setenv("GSNAPDP_ENDS_ROWLANE", "1")
    ctx = Context(blocks)
    res2, ops2, off2 = ctx.run(batch.windows, batch.query, batch.query_uc)
    pairs2, np2 = ctx.all_pairs(batch.windows, batch.query, batch.query_uc, res2, ops2, off2)
    compare(res2, pairs2, np2, ref, oflat, onp, "end gaps on k_rows seed %d" % seed)
    for f in ("bestr", "bestc", "status"):
        assert np.array_equal(res[f], res2[f]), f
    assert np.sum(res["bestc"] == 0) > 0 and np.sum(res["bestr"] > 0) > 5000


def test_gpu_consecutive_batches_on_one_context():
    """One context, batches in turn whose row-lane lists are full, empty and
    full again (end gaps of every row class, then single gaps only, then wide and
    long windows): k_plan's last block resets its ticket and the histogram,
    k_rows' last block clears the class counts and END flags, so no batch sees
    another's lists.  Every batch bit-exact against the restatement."""
    g = W.synthetic_genome(2_000_000, seed=77, n_rate=0.002)
    blocks = W.pack_genome(g)
    ends = W.concat_batches([W.random_windows(g, 800, seed=700 + k, kinds=(END5_GAP, END3_GAP), max_len1=m1,
                                              max_len2=m1 + 20, max_band=b)
                             for k, (m1, b) in enumerate(((30, 6), (250, 5), (600, 12)))])
    singles = W.random_windows(g, 3000, seed=71, max_len1=120, max_len2=140, max_band=20)
    wide = W.random_windows(g, 300, seed=72, max_len1=700, max_len2=900, max_band=60)
    O.setup(blocks)
    refs = []
    for b in (ends, singles, wide):
        ores, opairs, ooff, onp = O.run_batch(b.windows, b.query, b.query_uc, nthreads=16)
        oflat = np.concatenate([opairs[ooff[i]:ooff[i] + onp[i]] for i in range(len(onp))])
        ref = {f: ores[f] for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels")}
        ref["dynprogindex"] = ores["reserved"]
        refs.append((ref, oflat, onp))
    ctx = Context(blocks)
    for k in (0, 1, 0, 2, 1, 2, 0):
        b = (ends, singles, wide)[k]
        res, ops, off = ctx.run(b.windows, b.query, b.query_uc)
        pairs, npairs = ctx.all_pairs(b.windows, b.query, b.query_uc, res, ops, off)
        compare(res, pairs, npairs, *refs[k], "batch kind %d on a shared context" % k)
    ctx.close()


def check_buckets(keys, perm, cs, cw, what):
    """k_plan's last-block scan + k_scatter: every k_fill window (key >= 0) in perm
    exactly once; each class range a whole number of wave-tasks; each wave-task
    one key, its padding (-1) at its end; each key's windows contiguous."""
    n = keys.size
    live = perm[perm >= 0]
    assert np.array_equal(np.sort(live), np.nonzero(keys >= 0)[0]), "%s: perm is not the k_fill windows" % what
    assert cs[0] == 0 and np.all(np.diff(cs) >= 0) and cs[-1] == perm.size, what
    pk = np.where(perm >= 0, keys[np.clip(perm, 0, max(n - 1, 0))], -1)
    for c in range(cw.size):
        a, b, g = int(cs[c]), int(cs[c + 1]), int(cw[c])
        assert (b - a) % g == 0, "%s: class %d range %d not a multiple of %d" % (what, c, b - a, g)
        chunks = pk[a:b].reshape(-1, g)
        if chunks.size == 0:
            continue
        first = chunks[:, 0]
        assert np.all(first >= 0), "%s: class %d has an empty wave-task" % (what, c)
        ok = (chunks == first[:, None]) | (chunks == -1)
        assert ok.all(), "%s: class %d: a wave-task mixes keys" % (what, c)
        pad = chunks == -1
        assert np.all(np.diff(pad.astype(np.int8), axis=1) >= 0), "%s: class %d: padding inside a task" % (what, c)
    # a key's wave-tasks are contiguous: keys appear as one run each in task order
    tk = pk[pk >= 0]
    if tk.size == 0:
        return
    runs = tk[np.r_[True, tk[1:] != tk[:-1]]]
    assert runs.size == np.unique(tk).size, "%s: a key's windows are split" % what


def test_gpu_bucket_scan_stress():
    """The bucketing (k_plan's histogram atomics read back by its last block's
    scan, then k_scatter) over 48 batches of 1 to 120k windows on one context,
    each batch's buckets checked against the host (check_buckets) and its
    results bit-exact against the restatement's over the same windows."""
    g = W.synthetic_genome(4_000_000, seed=91, n_rate=0.002)
    blocks = W.pack_genome(g)
    pool = W.concat_batches([W.random_windows(g, 20_000, seed=910 + k, max_len1=m1, max_len2=m1 + 20,
                                              max_band=b)
                             for k, (m1, b) in enumerate(((40, 3), (120, 10), (160, 20), (200, 40)))])
    O.setup(blocks)
    ores, _, _, _ = O.run_batch(pool.windows, pool.query, pool.query_uc, nthreads=16)
    rng = np.random.default_rng(92)
    ctx = Context(blocks)
    sizes = [1, 2, 63, 64, 65, 1000, 120_000 if len(pool) >= 120_000 else len(pool)]
    sizes += [int(x) for x in rng.integers(1, len(pool), 41)]
    for t, m in enumerate(sizes):
        idx = rng.choice(len(pool), size=m, replace=False)
        w = pool.windows[idx]
        res, _, _ = ctx.run(w, pool.query, pool.query_uc)
        keys, perm, cs, cw = ctx.debug_buckets(m)
        check_buckets(keys, perm, cs, cw, "batch %d (%d windows)" % (t, m))
        for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels", "reserved"):
            bad = np.nonzero(res[f] != ores[f][idx])[0]
            assert bad.size == 0, "batch %d (%d windows): %s differs at %s" % (t, m, f, bad[:8])
    ctx.close()
