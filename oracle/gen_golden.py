#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

TEST INFRASTRUCTURE ONLY; runs in the development container (needs
/root/reference and oracle/_ref/ref_driver, built by `make -C oracle ref`).

Every fixture is data only: the inputs (packed genome blocks, window records,
query bytes) and the reference's outputs for them (scores, counts, the full
pair lists, maxent probabilities, the HIGHQ substitution table).  Genomes:

* ``chr17``: tests/ss.chr17test from the reference's own test suite, packed by
  gsnapdp.genome.pack (bit-identical to the reference's setup.genomecomp.ok,
  checked here and in tests/test_genome.py);
* ``synth``: 300 kb synthetic genome with N runs (seed 11).

Usage: python3 oracle/gen_golden.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import genome as G  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import (CGAP_RESULT, GGAP_RESULT, GGAP_WINDOW, MAXLENGTH1, MAXLENGTH2,  # noqa: E402
                             MICRO_RESULT, PAIR, RESULT)

REF_TESTS = "/root/reference/tests"
DRIVER = os.path.join(HERE, "_ref", "ref_driver")
OUT = os.path.join(ROOT, "tests", "golden")


def run_driver(mode: str, d: str, genome_mode: int = 0) -> None:
    subprocess.check_call([DRIVER, mode, d, str(genome_mode)])


def dp_case(name: str, blocks: np.ndarray, batch: W.Batch, mode: int = 0) -> None:
    with tempfile.TemporaryDirectory() as d:
        batch.windows.tofile(os.path.join(d, "windows.bin"))
        batch.query.tofile(os.path.join(d, "query.bin"))
        batch.query_uc.tofile(os.path.join(d, "query_uc.bin"))
        blocks.astype("<u4").tofile(os.path.join(d, "genome.u32"))
        run_driver("dp", d, mode)
        res = np.fromfile(os.path.join(d, "results.bin"), dtype=RESULT)
        npairs = np.fromfile(os.path.join(d, "npairs.i32"), dtype=np.int32)
        pairs = np.fromfile(os.path.join(d, "pairs.bin"), dtype=PAIR)
    assert pairs.size == int(npairs.sum())
    np.savez_compressed(os.path.join(OUT, name + ".npz"), blocks=blocks, windows=batch.windows,
                        query=batch.query, query_uc=batch.query_uc, mode=np.int32(mode),
                        finalscore=res["finalscore"], nmatches=res["nmatches"],
                        nmismatches=res["nmismatches"], nopens=res["nopens"], nindels=res["nindels"],
                        dynprogindex=res["reserved"], npairs=npairs, pairs=pairs)
    print("%s: %d windows, %d pairs" % (name, len(batch), pairs.size))


def ggap_windows(gseq: np.ndarray, n: int, seed: int):
    """Intron windows shaped like traverse_genome_gap's (stage3.c:5770-5809):
    length2L = length2R = length1 + extramaterial_paired (8); most carry a
    planted canonical / semi-canonical dinucleotide pair."""
    rng = np.random.default_rng(seed)
    g = gseq.copy()
    Gn = g.size
    w = np.zeros(n, dtype=GGAP_WINDOW)
    qs, us = [], []
    qpos = 0
    for i in range(n):
        L1 = int(rng.integers(2, 30)) if rng.random() < 0.8 else int(rng.integers(30, 60))
        L2 = L1 + 8
        intron = int(rng.integers(40, 400))
        glen = L1 + intron + 60
        chrpos = int(rng.integers(0, Gn - glen - 1))
        watson = int(rng.integers(0, 2))
        cdir = int(rng.choice([1, -1, 0]))
        k = int(rng.integers(0, L1 + 1))          # query bases before the splice
        offset2L = int(rng.integers(5, 25))       # genome col of query base 0
        donor = offset2L + k                      # first intron base (window coords)
        acceptor_end = donor + intron             # first base of exon 2
        revoffset2R = acceptor_end + (L1 - k) - 1
        if revoffset2R >= glen:
            revoffset2R = glen - 1

        def absolute(x):
            return chrpos + (x if watson else glen - 1 - x)

        def put(x, ch):
            c = ord(ch)
            g[absolute(x)] = c if watson else W._COMP[c]

        r = rng.random()
        if r < 0.6:
            dl, dr = ("GT", "AG") if cdir >= 0 else ("CT", "AC")
        elif r < 0.75:
            dl, dr = ("GC", "AG") if cdir >= 0 else ("CT", "GC")
        elif r < 0.85:
            dl, dr = ("AT", "AC") if cdir >= 0 else ("GT", "AT")
        else:
            dl, dr = None, None
        if dl:
            put(donor, dl[0])
            put(donor + 1, dl[1])
            put(acceptor_end - 2, dr[0])
            put(acceptor_end - 1, dr[1])
        view = np.array([g[absolute(x)] for x in range(glen)], dtype=np.uint8)
        if not watson:
            view = W._COMP[view]
        q = np.concatenate([view[offset2L:offset2L + k], view[acceptor_end:acceptor_end + (L1 - k)]])
        if q.size < L1:
            q = np.concatenate([q, W.ACGT[rng.integers(0, 4, size=L1 - q.size)]])
        q = W._mutate(rng, q, 0.04, 0.01)
        if rng.random() < 0.15 and L1 > 6:  # small indel near the junction
            p = int(rng.integers(1, L1 - 2))
            q = np.concatenate([q[:p], q[p + 1:], W.ACGT[rng.integers(0, 4, size=1)]])
        qs.append(q)
        us.append(q.copy())
        qs.append(np.full(4, ord("#"), np.uint8))
        us.append(np.full(4, ord("#"), np.uint8))
        rec = w[i]
        rec["length1"] = L1
        rec["length2L"] = L2
        rec["length2R"] = L2
        rec["offset1"] = int(rng.integers(0, 300))
        rec["offset2L"] = offset2L
        rec["revoffset2R"] = revoffset2R
        rec["chroffset"] = 0
        rec["chrhigh"] = Gn
        rec["chrpos"] = chrpos
        rec["genomiclength"] = glen
        rec["qpos"] = qpos
        rec["cdna_direction"] = cdir
        rec["extraband_paired"] = int(rng.choice([7, 3, 10]))
        rec["maxpeelback"] = int(rng.choice([11, 5]))
        rec["dynprogindex"] = int(rng.choice([-1, 2]))
        rec["maxlength1"] = MAXLENGTH1
        rec["maxlength2"] = MAXLENGTH2
        rec["defect_rate"] = float(rng.choice([0.001, 0.005, 0.02]))
        rec["watsonp"] = watson
        rec["jump_late_p"] = int(rng.integers(0, 2))
        rec["halfp"] = int(rng.random() < 0.2)
        rec["finalp"] = int(rng.random() < 0.6)
        rec["use_probabilities_p"] = int(rng.random() < 0.35)
        rec["splicingp"] = int(rng.random() < 0.9)
        rec["score_threshold"] = int(rng.integers(-20, 40)) if rec["use_probabilities_p"] else 0
        qpos += L1 + 4
    return g, w, np.concatenate(qs), np.concatenate(us)


def ggap_case(name: str, gseq: np.ndarray, n: int, seed: int) -> None:
    sys.path.insert(0, HERE)
    import oracle as O  # checker, used only to drop windows the reference cannot run (UB)
    g, w, q, u = ggap_windows(gseq, n, seed)
    blocks = G.pack(g)
    O.setup(blocks)
    ores, _, _, _ = O.run_ggap_batch(w, q, u)
    keep = ores["bridge_ok"] == 1  # dynprog.c:4055 reads uninitialised indices otherwise
    w = w[keep]
    with tempfile.TemporaryDirectory() as d:
        w.tofile(os.path.join(d, "ggap_windows.bin"))
        q.tofile(os.path.join(d, "query.bin"))
        u.tofile(os.path.join(d, "query_uc.bin"))
        blocks.astype("<u4").tofile(os.path.join(d, "genome.u32"))
        run_driver("ggap", d)
        res = np.fromfile(os.path.join(d, "ggap_results.bin"), dtype=GGAP_RESULT)
        npairs = np.fromfile(os.path.join(d, "npairs.i32"), dtype=np.int32)
        pairs = np.fromfile(os.path.join(d, "pairs.bin"), dtype=PAIR)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), blocks=blocks, windows=w, query=q,
                        query_uc=u, results=res, npairs=npairs, pairs=pairs,
                        dropped_ub=np.int32((~keep).sum()))
    print("%s: %d windows (%d dropped: probability-mode UB), %d pairs" %
          (name, len(w), int((~keep).sum()), pairs.size))


def cgap_case(name: str, gseq: np.ndarray, n: int, seed: int) -> None:
    """Dynprog_cdna_gap windows (W.cgap_windows); windows whose bridge finds no
    candidate (the reference then reads uninitialised indices) are dropped."""
    sys.path.insert(0, HERE)
    import oracle as O  # checker, used only to drop windows the reference cannot run (UB)
    b = W.cgap_windows(gseq, n, seed)
    blocks = G.pack(gseq)
    O.setup(blocks)
    ores, _, _, _ = O.run_cgap_batch(b.windows, b.query, b.query_uc, b.gseg, b.gseg_off)
    keep = ores["status"] != 5
    w, goff = b.windows[keep], b.gseg_off[keep]
    with tempfile.TemporaryDirectory() as d:
        w.tofile(os.path.join(d, "cgap_windows.bin"))
        b.query.tofile(os.path.join(d, "query.bin"))
        b.query_uc.tofile(os.path.join(d, "query_uc.bin"))
        b.gseg.tofile(os.path.join(d, "gseg.bin"))
        goff.astype("<i8").tofile(os.path.join(d, "gseg_off.i64"))
        blocks.astype("<u4").tofile(os.path.join(d, "genome.u32"))
        run_driver("cgap", d)
        res = np.fromfile(os.path.join(d, "cgap_results.bin"), dtype=CGAP_RESULT)
        npairs = np.fromfile(os.path.join(d, "npairs.i32"), dtype=np.int32)
        pairs = np.fromfile(os.path.join(d, "pairs.bin"), dtype=PAIR)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), blocks=blocks, windows=w, query=b.query,
                        query_uc=b.query_uc, gseg=b.gseg, gseg_off=goff, results=res, npairs=npairs,
                        pairs=pairs, dropped_ub=np.int32((~keep).sum()))
    print("%s: %d windows (%d dropped: no bridge candidate), %d pairs" %
          (name, len(w), int((~keep).sum()), pairs.size))


def sj_case(name: str, gseq: np.ndarray, n: int, seed: int) -> None:
    b = W.sj_windows(gseq, n, seed)
    with tempfile.TemporaryDirectory() as d:
        b.windows.tofile(os.path.join(d, "sj_windows.bin"))
        b.query.tofile(os.path.join(d, "query.bin"))
        b.query_uc.tofile(os.path.join(d, "query_uc.bin"))
        run_driver("sj", d)
        res = np.fromfile(os.path.join(d, "results.bin"), dtype=RESULT)
        npairs = np.fromfile(os.path.join(d, "npairs.i32"), dtype=np.int32)
        pairs = np.fromfile(os.path.join(d, "pairs.bin"), dtype=PAIR)
    assert pairs.size == int(npairs.sum())
    np.savez_compressed(os.path.join(OUT, name + ".npz"), windows=b.windows, query=b.query,
                        query_uc=b.query_uc, finalscore=res["finalscore"], nmatches=res["nmatches"],
                        nmismatches=res["nmismatches"], nopens=res["nopens"], nindels=res["nindels"],
                        dynprogindex=res["reserved"], npairs=npairs, pairs=pairs)
    print("%s: %d windows, %d pairs" % (name, len(b), pairs.size))


def mksj_case(name: str, gseq: np.ndarray, n: int, seed: int) -> None:
    """Dynprog_make_splicejunction_5/3 at random coordinates, every splice type, both strands."""
    rng = np.random.default_rng(seed)
    blocks = G.pack(gseq)
    rec = np.zeros(n, dtype=[("end", "<i4"), ("splicecoord", "<i4"), ("splicelength", "<i4"),
                             ("contlength", "<i4"), ("far_splicetype", "<i4"), ("watsonp", "<i4")])
    rec["end"] = rng.choice([5, 3], size=n)
    rec["splicelength"] = rng.integers(0, 120, size=n)
    rec["contlength"] = rng.integers(0, 40, size=n)
    rec["splicecoord"] = rng.integers(200, gseq.size - 200, size=n)
    rec["far_splicetype"] = rng.integers(0, 4, size=n)
    rec["watsonp"] = rng.integers(0, 2, size=n)
    with tempfile.TemporaryDirectory() as d:
        rec.tofile(os.path.join(d, "mksj_in.bin"))
        blocks.astype("<u4").tofile(os.path.join(d, "genome.u32"))
        run_driver("mksj", d)
        out = np.fromfile(os.path.join(d, "mksj_out.bin"), dtype=np.uint8)
    assert out.size == int((rec["contlength"] + rec["splicelength"]).sum())
    np.savez_compressed(os.path.join(OUT, name + ".npz"), blocks=blocks, records=rec, junctions=out)
    print("%s: %d junctions, %d bytes" % (name, n, out.size))


def micro_case(name: str, gseq: np.ndarray, n: int, seed: int) -> None:
    g, b = W.micro_windows(gseq, n, seed)
    blocks = G.pack(g)
    with tempfile.TemporaryDirectory() as d:
        b.windows.tofile(os.path.join(d, "micro_windows.bin"))
        b.query.tofile(os.path.join(d, "query.bin"))
        b.query_uc.tofile(os.path.join(d, "query_uc.bin"))
        blocks.astype("<u4").tofile(os.path.join(d, "genome.u32"))
        run_driver("micro", d)
        res = np.fromfile(os.path.join(d, "micro_results.bin"), dtype=MICRO_RESULT)
        npairs = np.fromfile(os.path.join(d, "npairs.i32"), dtype=np.int32)
        pairs = np.fromfile(os.path.join(d, "pairs.bin"), dtype=PAIR)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), blocks=blocks, windows=b.windows, query=b.query,
                        query_uc=b.query_uc, results=res, npairs=npairs, pairs=pairs)
    print("%s: %d windows (%d found), %d pairs" % (name, len(b), int(res["found"].sum()), pairs.size))


def maxent_case(name: str, blocks: np.ndarray, glen: int, n: int, seed: int) -> None:
    rng = np.random.default_rng(seed)
    model = rng.integers(0, 4, size=n).astype(np.uint32)
    pos = rng.integers(0, glen - 40, size=n).astype(np.uint32)
    # every shift of every model, plus the margin-underflow edges
    extra_m, extra_p = [], []
    for m in range(4):
        for s in range(32):
            extra_m.append(m)
            extra_p.append(1000 * 32 + s + (3, 20, 6, 3)[m])
        for p in range(0, 25):
            extra_m.append(m)
            extra_p.append(p)
    model = np.concatenate([model, np.array(extra_m, np.uint32)])
    pos = np.concatenate([pos, np.array(extra_p, np.uint32)])
    chroff = np.zeros(pos.size, np.uint32)
    chroff[:n // 10] = pos[:n // 10] - rng.integers(0, 30, size=n // 10).astype(np.uint32).clip(0, None)
    chroff = np.minimum(chroff, pos)
    rec = np.zeros(pos.size, dtype=[("model", "<u4"), ("splice_pos", "<u4"), ("chroffset", "<u4"), ("pad", "<u4")])
    rec["model"], rec["splice_pos"], rec["chroffset"] = model, pos, chroff
    with tempfile.TemporaryDirectory() as d:
        rec.tofile(os.path.join(d, "maxent_in.bin"))
        blocks.astype("<u4").tofile(os.path.join(d, "genome.u32"))
        run_driver("maxent", d)
        out = np.fromfile(os.path.join(d, "maxent_out.f64"), dtype="<f8")
    np.savez_compressed(os.path.join(OUT, name + ".npz"), blocks=blocks, model=model.astype(np.uint8),
                        splice_pos=pos, chroffset=chroff, prob=out)
    print("%s: %d positions" % (name, pos.size))


def pdist_case() -> None:
    with tempfile.TemporaryDirectory() as d:
        run_driver("pdist", d)
        t = np.fromfile(os.path.join(d, "pdist_highq.i32"), dtype=np.int32).reshape(128, 128)
    np.savez_compressed(os.path.join(OUT, "pairdistance_highq.npz"), table=t)
    print("pairdistance_highq: 128x128")


def main() -> None:
    only = set(sys.argv[1:])  # optional: names of the fixtures to (re)generate
    os.makedirs(OUT, exist_ok=True)
    subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
    chr17 = np.frombuffer(G.read_fasta(os.path.join(REF_TESTS, "ss.chr17test")), dtype=np.uint8).copy()
    b17 = G.pack(chr17)
    ok = np.fromfile(os.path.join(REF_TESTS, "setup.genomecomp.ok"), dtype="<u4")
    assert np.array_equal(b17[:ok.size], ok), "packer disagrees with setup.genomecomp.ok"
    synth = W.synthetic_genome(300_000, seed=11, n_rate=0.004)
    bsyn = G.pack(synth)

    cases = [
        ("pairdistance_highq", lambda: pdist_case()),
        ("dp_chr17_mix", lambda: dp_case("dp_chr17_mix", b17, W.random_windows(chr17, 2500, seed=101))),
        ("dp_synth_mix", lambda: dp_case("dp_synth_mix", bsyn, W.random_windows(synth, 2500, seed=102, chroms=6))),
        ("dp_synth_cmet", lambda: dp_case("dp_synth_cmet", bsyn, W.random_windows(synth, 400, seed=103), mode=1)),
        ("dp_chr17_c2", lambda: dp_case("dp_chr17_c2", b17, W.c2_windows(chr17, n=300, seed=104))),
        ("dp_synth_long", lambda: dp_case("dp_synth_long", bsyn, W.random_windows(
            synth, 150, seed=105, max_len1=640, max_len2=700, max_band=40))),
        ("ggap_chr17", lambda: ggap_case("ggap_chr17", chr17, 1500, seed=201)),
        ("cgap_chr17", lambda: cgap_case("cgap_chr17", chr17, 1500, seed=401)),
        ("sj_chr17", lambda: sj_case("sj_chr17", chr17, 2000, seed=501)),
        ("mksj_chr17", lambda: mksj_case("mksj_chr17", chr17, 2000, seed=502)),
        ("micro_chr17", lambda: micro_case("micro_chr17", chr17, 1500, seed=601)),
        ("maxent_chr17", lambda: maxent_case("maxent_chr17", b17, chr17.size, 20000, seed=301)),
        ("maxent_synth", lambda: maxent_case("maxent_synth", bsyn, synth.size, 6000, seed=302)),
    ]
    for name, fn in cases:
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main()
