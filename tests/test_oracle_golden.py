"""Pin the CPU restatement (oracle/) to the reference's own outputs.

The fixtures in tests/golden/ were produced by the reference compiled from
its own sources (oracle/gen_golden.py, oracle/_ref/ref_driver).  Every field
of every pair, every score / count and every maxent probability must match
bit for bit.
"""
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp.records import PAIR

DP_CASES = ["dp_chr17_mix", "dp_synth_mix", "dp_synth_cmet", "dp_chr17_c2", "dp_synth_long",
            "gmap_synth_gap", "gmap_her2_gap"]  # the last two: windows the reference gmap issued (oracle/gmap_trace.c)


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)


def split_pairs(pairs, npairs):
    off = np.zeros(len(npairs) + 1, dtype=np.int64)
    np.cumsum(npairs, out=off[1:])
    return off


@pytest.mark.parametrize("name", DP_CASES)
def test_dp_oracle_matches_reference(golden_dir, name):
    z = load(golden_dir, name)
    O.setup(z["blocks"], mode=int(z["mode"]))
    res, pairs, off, npairs = O.run_batch(z["windows"], z["query"], z["query_uc"], nthreads=4)
    for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels"):
        bad = np.nonzero(res[f] != z[f])[0]
        assert bad.size == 0, "%s differs at windows %s" % (f, bad[:10])
    assert np.array_equal(res["reserved"], z["dynprogindex"])
    assert np.array_equal(npairs, z["npairs"])
    goff = split_pairs(z["pairs"], z["npairs"])
    got = np.concatenate([pairs[off[i]:off[i] + npairs[i]] for i in range(len(npairs))])
    assert got.dtype == PAIR
    for f in PAIR.names:
        bad = np.nonzero(got[f] != z["pairs"][f])[0]
        assert bad.size == 0, "pair field %s differs (first pair %s)" % (f, bad[:5])
    assert goff[-1] == got.size


GGAP_SETS = ["ggap_chr17", "gmap_synth_ggap", "gmap_her2_ggap", "ggap_known_sites",
             "ggap_known_sites_novel", "ggap_known_introns", "ggap_known_introns_novel"]


@pytest.mark.parametrize("name", GGAP_SETS)
def test_ggap_oracle_matches_reference(golden_dir, name):
    z = load(golden_dir, name)
    O.setup(z["blocks"])
    res, pairs, off, npairs = O.run_ggap_batch(z["windows"], z["query"], z["query_uc"])
    ref = z["results"]
    assert np.all(res["bridge_ok"] == 1)
    nn = ref["returned_null"] == 0
    # out-parameters the reference always writes
    for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels", "dynprogindex",
              "returned_null"):
        bad = np.nonzero(res[f] != ref[f])[0]
        assert bad.size == 0, "%s differs at %s" % (f, bad[:10])
    # written only when a list is returned
    for f in ("new_leftgenomepos", "new_rightgenomepos", "exonhead", "introntype"):
        bad = np.nonzero((res[f] != ref[f]) & nn)[0]
        assert bad.size == 0, "%s differs at %s" % (f, bad[:10])
    for f in ("left_prob", "right_prob"):
        assert np.array_equal(res[f].view(np.uint64), ref[f].view(np.uint64)), f
    assert np.array_equal(npairs, z["npairs"])
    got = np.concatenate([pairs[off[i]:off[i] + npairs[i]] for i in range(len(npairs))])
    for f in PAIR.names:
        assert np.array_equal(got[f], z["pairs"][f]), f


@pytest.mark.parametrize("name", ["maxent_chr17", "maxent_synth"])
def test_maxent_oracle_matches_reference(golden_dir, name):
    z = load(golden_dir, name)
    O.setup(z["blocks"])
    got = O.maxent(z["model"], z["splice_pos"], z["chroffset"])
    ref = z["prob"]
    bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))[0]
    assert bad.size == 0, "maxent differs at %s (model %s shift %s)" % (
        bad[:10], z["model"][bad[:10]], z["splice_pos"][bad[:10]] % 32)


def test_pairdistance_matches_reference(golden_dir):
    z = load(golden_dir, "pairdistance_highq")
    O.setup(np.zeros(16, np.uint32))
    L = O.lib()
    got = np.array([[L.orc_pairdistance(0, a, b) for b in range(128)] for a in range(128)])
    assert np.array_equal(got, z["table"])


def test_cgap_oracle_matches_reference(golden_dir):
    """Dynprog_cdna_gap: out-parameters and the full list, including the
    INSERT_PAIRS branch (dynprog.c:4730-4752)."""
    z = load(golden_dir, "cgap_chr17")
    O.setup(z["blocks"])
    res, pairs, off, npairs = O.run_cgap_batch(z["windows"], z["query"], z["query_uc"], z["gseg"],
                                               z["gseg_off"])
    ref = z["results"]
    assert np.all(res["status"] != 5)
    for f in ("finalscore", "finalscore_set", "dynprogindex", "incompletep", "returned_null"):
        bad = np.nonzero(res[f] != ref[f])[0]
        assert bad.size == 0, "%s differs at %s (oracle %s ref %s)" % (f, bad[:10], res[f][bad[:10]], ref[f][bad[:10]])
    assert np.array_equal(npairs, z["npairs"])
    got = np.concatenate([pairs[off[i]:off[i] + npairs[i]] for i in range(len(npairs))])
    for f in PAIR.names:
        assert np.array_equal(got[f], z["pairs"][f]), f
    assert res["insert_pairs"].sum() > 20 and (res["returned_null"] == 0).sum() > 1000


def test_sj_oracle_matches_reference(golden_dir):
    """Dynprog_end5/3_splicejunction: scores recomputed from the counts, both
    traceback_local parts around the known gapholder, INDEL stripping."""
    z = load(golden_dir, "sj_chr17")
    O.setup(np.zeros(16, np.uint32))  # the genome is never read (use_genomicseg_p)
    res, pairs, off, npairs = O.run_sj_batch(z["windows"], z["query"], z["query_uc"])
    for f in ("finalscore", "nmatches", "nmismatches", "nopens", "nindels"):
        bad = np.nonzero(res[f] != z[f])[0]
        assert bad.size == 0, "%s differs at windows %s" % (f, bad[:10])
    assert np.array_equal(res["reserved"], z["dynprogindex"])
    assert np.array_equal(npairs, z["npairs"])
    got = np.concatenate([pairs[off[i]:off[i] + npairs[i]] for i in range(len(npairs))])
    for f in PAIR.names:
        assert np.array_equal(got[f], z["pairs"][f]), f
    assert (z["pairs"]["gapp"] == 3).sum() > 1500  # known gapholders


def test_micro_oracle_matches_reference(golden_dir):
    """Dynprog_microexon_int: out-parameters (f64 probabilities bit for bit) and
    the list, including the reference's last-hit offset for the middle pairs."""
    z = load(golden_dir, "micro_chr17")
    O.setup(z["blocks"])
    res, pairs, off, npairs = O.run_micro_batch(z["windows"], z["query"], z["query_uc"])
    ref = z["results"]
    for f in ("microintrontype", "dynprogindex", "found"):
        bad = np.nonzero(res[f] != ref[f])[0]
        assert bad.size == 0, "%s differs at %s" % (f, bad[:10])
    for f in ("bestprob2", "bestprob3"):
        assert np.array_equal(res[f].view(np.uint64), ref[f].view(np.uint64)), f
    assert np.array_equal(npairs, z["npairs"])
    got = np.concatenate([pairs[off[i]:off[i] + npairs[i]] for i in range(len(npairs))])
    for f in PAIR.names:
        assert np.array_equal(got[f], z["pairs"][f]), f
    assert ref["found"].sum() > 500


REF_DRIVER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref")


@pytest.mark.parametrize("amb_closest", [0, 1])
def test_splicetrie_double_matches_reference_splicetrie(golden_dir, tmp_path, amb_closest):
    """The clean-room Splicetrie_solve_end5/3 test double (tests/dropin/
    splicetrie_double.c, used by the GPU drop-in test instead of reference
    code) against the reference's splicetrie.c: ref_driver's known-site mode
    linked with each, on the known_chr17 inputs, every output byte-identical
    (and the reference build equal to the committed golden vectors)."""
    import subprocess
    ref, dbl = os.path.join(REF_DRIVER, "ref_driver"), os.path.join(REF_DRIVER, "ref_driver_dbl")
    if not (os.path.exists(ref) and os.path.exists(dbl)):
        pytest.skip("reference drivers are built only in the dev container (make -C oracle ref)")
    z = load(golden_dir, "known_chr17")
    outs = {}
    for tag, exe in (("ref", ref), ("dbl", dbl)):
        d = tmp_path / tag
        d.mkdir()
        z["windows"].tofile(str(d / "known_windows.bin"))
        z["query"].tofile(str(d / "query.bin"))
        z["query_uc"].tofile(str(d / "query_uc.bin"))
        z["blocks"].astype("<u4").tofile(str(d / "genome.u32"))
        z["sites"].tofile(str(d / "sites.u32"))
        z["types"].tofile(str(d / "types.i32"))
        for k in ("tobs", "cobs", "tmax", "cmax"):
            z[k].tofile(str(d / (k + ".u32")))
        subprocess.check_call([exe, "known", str(d), "0", str(amb_closest)])
        outs[tag] = [open(str(d / f), "rb").read() for f in ("known_results.bin", "npairs.i32", "pairs.bin")]
    assert outs["ref"] == outs["dbl"]
    if amb_closest == int(z["amb_closest"]):
        assert outs["ref"][0] == z["results"].tobytes()


def golden_intron_paths(z, path_introns):
    """The golden score_introns calls (recorded in the reference's gmap by
    oracle/gmap_trace.c) as batch records: each call's pairs -> its introns."""
    from gsnapdp.records import INTRON, INTRON_PATH, PATH_PAIR
    calls, sp = z["calls"], z["pairs"]
    paths = np.zeros(len(calls), dtype=INTRON_PATH)
    chunks = []
    n = 0
    for i, c in enumerate(calls):
        pr = np.zeros(int(c["npairs"]), dtype=PATH_PAIR)
        seg = sp[int(c["first_pair"]):int(c["first_pair"]) + int(c["npairs"])]
        for f in ("genomepos", "queryjump", "genomejump", "gapp", "knowngapp", "comp"):
            pr[f] = seg[f]
        it = path_introns(pr, int(c["nullgap"]), i)
        paths[i] = (c["chroffset"], c["chrpos"], c["genomiclength"], c["cdna_direction"], c["watsonp"], n, len(it), 0)
        chunks.append(it)
        n += len(it)
    return paths, (np.concatenate(chunks) if chunks else np.zeros(0, INTRON))


@pytest.mark.parametrize("name", ["gmap_her2_introns", "gmap_synth_introns"])
def test_score_introns_oracle_matches_reference(golden_dir, name):
    """score_introns (stage3.c:7935-8162): the restatement reproduces every
    call the reference's gmap made, its averages bit for bit."""
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    O.setup(z["blocks"])
    paths, introns = golden_intron_paths(z, O.path_introns)
    out = O.score_introns(paths, introns)
    c = z["calls"]
    assert np.array_equal(out["nbadintrons"], c["nbadintrons"])
    assert out["avg_donor_score"].tobytes() == c["avg_donor_score"].tobytes()
    assert out["avg_acceptor_score"].tobytes() == c["avg_acceptor_score"].tobytes()
    assert introns.size >= 20 and np.sum(out["nintrons"] > 0) >= 1
