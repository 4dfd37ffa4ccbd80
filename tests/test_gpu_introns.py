"""score_introns (stage3.c:7935-8162) on the GPU: the batched C-ABI
(gsnapdp_score_introns_host, one k_introns launch) and the drop-in's
Gsnapdp_score_introns (the reference's signature, List_T in, reversed list out)
against every call the reference's gmap made (gmap_trace goldens: ss.her2 and
the synthetic spliced cDNAs), and against the restatement on random paths."""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from gsnapdp import Context, path_introns
from gsnapdp import workload as W
from gsnapdp.records import INTRON, INTRON_PATH
from test_oracle_golden import golden_intron_paths

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "gmap-gsnap_amd", "lib", "libgsnapdp_dropin.so")
DOUBLE_SRC = os.path.join(ROOT, "tests", "dropin", "pairpool_double.c")
NAMES = ["gmap_her2_introns", "gmap_synth_introns"]


def check(out, calls, what):
    assert np.array_equal(out["nbadintrons"], calls["nbadintrons"]), what
    bad = np.nonzero(out["avg_donor_score"].view(np.uint64) != calls["avg_donor_score"].view(np.uint64))[0]
    assert bad.size == 0, "%s: avg_donor_score differs at %s" % (what, bad[:8])
    bad = np.nonzero(out["avg_acceptor_score"].view(np.uint64) != calls["avg_acceptor_score"].view(np.uint64))[0]
    assert bad.size == 0, "%s: avg_acceptor_score differs at %s" % (what, bad[:8])


@pytest.mark.parametrize("name", NAMES)
def test_gpu_score_introns_matches_reference_golden(golden_dir, name):
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    ctx = Context(z["blocks"])
    paths, introns = golden_intron_paths(z, path_introns)  # the product's host walk
    out = ctx.score_introns(paths, introns)
    check(out, z["calls"], name)
    ctx.close()


def test_gpu_score_introns_random_paths_match_restatement():
    """Both strands, both directions (and 0), known sites, known gaps, every
    comp kind the bad-intron rule looks at; 3000 paths in one launch."""
    rng = np.random.default_rng(41)
    glen = 3_000_000
    blocks = W.pack_genome(W.synthetic_genome(glen, seed=41, n_rate=0.002))
    n = 3000
    paths = np.zeros(n, INTRON_PATH)
    paths["chroffset"] = rng.integers(0, 1000, n)
    paths["chrpos"] = rng.integers(0, 1000, n)
    paths["genomiclength"] = rng.integers(50_000, 1_000_000, n)
    paths["cdna_direction"] = rng.choice([1, -1, 1, -1, 0], n)
    paths["watsonp"] = rng.integers(0, 2, n)
    k = rng.integers(0, 16, n)
    paths["nintrons"] = k
    paths["first_intron"] = np.concatenate([[0], np.cumsum(k)[:-1]])
    m = int(k.sum())
    it = np.zeros(m, INTRON)
    it["left_genomepos"] = rng.integers(100, 40_000, m)
    it["right_genomepos"] = it["left_genomepos"] + rng.integers(60, 8000, m)
    it["path"] = np.repeat(np.arange(n), k)
    it["comp"] = rng.choice(np.frombuffer(b"><=)(", np.uint8), m)
    it["knowngapp"] = rng.random(m) < 0.1
    it["known_donor"] = rng.random(m) < 0.1
    it["known_acceptor"] = rng.random(m) < 0.1
    ctx = Context(blocks)
    out = ctx.score_introns(paths, it)
    O.setup(blocks)
    ref = O.score_introns(paths, it)
    assert out.tobytes() == ref.tobytes()
    assert np.sum(ref["nbadintrons"] > 1) > 10 and np.sum(ref["nintrons"] == 0) > 100
    ctx.close()


def test_dropin_score_introns_matches_reference_golden(golden_dir, tmp_path):
    """Gsnapdp_score_introns as stage3.c would call it: the path as a List_T of
    the host's Pair_T cells, the three out-parameters, and the returned list
    (the path's cells, reversed)."""
    from doubles import pairpool_double
    dbl = pairpool_double()  # one copy per process (tests/doubles.py)
    dbl.dbl_list_build.restype = ctypes.c_void_p
    dbl.dbl_list_build.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dbl.dbl_list_read.restype = ctypes.c_int
    dbl.dbl_list_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    dbl.dbl_list_free.argtypes = [ctypes.c_void_p]
    L = ctypes.CDLL(DROPIN)
    L.Gsnapdp_dropin_genome.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.Gsnapdp_score_introns.restype = ctypes.c_void_p
    L.Gsnapdp_score_introns.argtypes = ([ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_ubyte, ctypes.c_int]
                                       + [ctypes.c_uint] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                                 ctypes.c_ubyte])
    z = {n: np.load(os.path.join(golden_dir, n + ".npz"), allow_pickle=False) for n in NAMES}
    # one genome per process in the drop-in: the synthetic cDNA set (the larger one)
    zz = z["gmap_synth_introns"]
    blocks = np.ascontiguousarray(zz["blocks"])
    L.Dynprog_term()  # a context an earlier test left holds another genome
    L.Gsnapdp_dropin_genome(blocks.ctypes.data, blocks.size, 0)
    from test_dropin import REC
    calls, sp = zz["calls"], np.ascontiguousarray(zz["pairs"])
    st0 = (ctypes.c_ulong * 21)()
    assert L.Gsnapdp_dropin_stats3(st0, 21) == 21
    for i, c in enumerate(calls):
        f0, npairs = int(c["first_pair"]), int(c["npairs"])
        recs = np.ascontiguousarray(sp[f0:f0 + npairs])
        lst = dbl.dbl_list_build(recs.ctypes.data, npairs)
        d, a, nb = ctypes.c_double(-1), ctypes.c_double(-1), ctypes.c_int(-7)
        out = L.Gsnapdp_score_introns(ctypes.byref(d), ctypes.byref(a), ctypes.byref(nb), lst,
                                      int(c["cdna_direction"]), int(c["watsonp"]), int(c["chrnum"]),
                                      int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]), None,
                                      int(c["genomiclength"]), int(c["nullgap"]), 0)
        assert nb.value == c["nbadintrons"], i
        assert np.float64(d.value).tobytes() == c["avg_donor_score"].tobytes(), i
        assert np.float64(a.value).tobytes() == c["avg_acceptor_score"].tobytes(), i
        back = np.zeros(npairs + 1, REC)
        k = dbl.dbl_list_read(out, back.ctypes.data, back.size)
        assert k == npairs and np.array_equal(back["querypos"][:k], recs["querypos"][::-1]), i
        dbl.dbl_list_free(out)
    st1 = (ctypes.c_ulong * 21)()
    L.Gsnapdp_dropin_stats3(st1, 21)
    assert st1[6] - st0[6] == len(calls) and st1[13] > st0[13]  # score_introns' paths and k_introns batches
    L.Dynprog_term()  # releases the device context (the genome array dies with this test)
