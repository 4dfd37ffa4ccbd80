"""The stage-3 passes on the GPU (gsnapdp_stage3_pass: build_pairs_introns,
stage3.c:7735-7901, and build_pairs_singles, :7454-7583, for many paths at once,
every round one batch per gap family) against every recorded call of the
reference's gmap
(tests/golden/gmap_*_stage3.npz; see test_stage3_cpu.py), and at scale: the
synthetic calls replicated into one pass of thousands of paths, each copy
checked against the reference, with the pass's throughput printed beside the
reference's own time for the same calls (its build_pairs_introns wall time in
gmap_trace, DP included)."""
import os
import time

import numpy as np
import pytest

from gsnapdp import Context, SplicingIIT
from gsnapdp import workload as W
from test_stage3_cpu import (GSNAP_PIPE_NAMES, IIT_NAMES, NAMES, PIPE_NAMES, check_compute, check_pass, check_path_compute,
                             check_scores, iit_intervals, stage3_golden)

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stage2_double(ctx, z, tmp):
    """traverse_dual_break's stage-2 lists served from the golden's recording
    (tests/dropin/stage2_double.c, built here with gcc) as the context's
    stage-2 callback.  Returns (the library, its handle) or None."""
    import ctypes
    import subprocess
    if "s2_calls" not in z:
        return None
    so = os.path.join(str(tmp), "libstage2_double.so")
    subprocess.check_call(["gcc", "-O1", "-shared", "-fPIC", "-o", so,
                           os.path.join(ROOT, "tests", "dropin", "stage2_double.c")])
    d = ctypes.CDLL(so)
    d.s2dbl_new.restype = ctypes.c_void_p
    d.s2dbl_new.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    sc, sp = np.ascontiguousarray(z["s2_calls"]), np.ascontiguousarray(z["s2_pairs"])
    h = d.s2dbl_new(sc.ctypes.data, sc.size, sp.ctypes.data, sp.size)
    ctx.set_stage2(ctypes.cast(d.s2dbl_compute_one, ctypes.c_void_p).value, h)
    return d, h


@pytest.mark.parametrize("name", NAMES)
def test_gpu_stage3_pass_matches_reference(golden_dir, tmp_path, name):
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    ctx = Context(z["blocks"])
    s2 = stage2_double(ctx, z, tmp_path)
    got_calls, got, st = ctx.stage3_pass(calls, pin, q, qu)
    check_pass(got_calls, got, calls, want, name, z["ub_ref"] if "ub_ref" in z else None)
    assert st["failed"] == 0 and st["undefined"] == 0
    if name == "gmap_cins_stage3":
        assert st["windows"][2] >= 200  # traverse_cdna_gap's Dynprog_cdna_gap windows
    print("%s: %d calls, %d rounds, windows %s in batches %s, %d calls with undefined intron lengths" % (
        name, len(calls), st["rounds"], st["windows"], st["batches"], int((got_calls["ub"] & 1).sum())))
    ctx.close()


@pytest.mark.parametrize("name", IIT_NAMES)
def test_gpu_stage3_pass_with_splicing_iit(golden_dir, name):
    """known-site records on every genome-gap window (site-level and intron-level
    IITs, novel splicing on and off) and score_introns with the IIT's verdicts,
    against the reference run with the same IIT"""
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    ctx = Context(z["blocks"])
    iit = SplicingIIT(iit_intervals(z))
    got_calls, got, st = ctx.stage3_pass(calls, pin, q, qu, iit=iit)
    check_pass(got_calls, got, calls, want, name)
    assert st["failed"] == 0 and st["undefined"] == 0
    check_scores(ctx.stage3_score_introns(got_calls, got, iit=iit), got_calls, z["si_calls"], name)
    print("%s: %d calls, windows %s, %d disallowed cells" % (name, len(calls), st["windows"],
                                                            int(((got["flags"] & 4) != 0).sum())))
    iit.close()
    ctx.close()


@pytest.mark.parametrize("name", PIPE_NAMES)
def test_gpu_stage3_compute_matches_reference(golden_dir, tmp_path, name):
    """passes 2A-6 of path_compute for every recorded invocation at once
    (gsnapdp_stage3_compute), the DP passes on the GPU: the lists pass 6
    returned in gmap, bit for bit, and the same pass calls; then the
    synthetic set x8 in one call, each copy checked, timed"""
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    queries, pin, q, qu, want, final, counts = W.stage3_pipeline(z)
    ctx = Context(z["blocks"])
    s2 = stage2_double(ctx, z, tmp_path)
    got_calls, got, st = ctx.stage3_compute(queries, pin, q, qu)
    check_compute(got_calls, got, final, want, name)
    assert list(st["pass_calls"]) == list(counts.sum(axis=0))
    if name == "gmap_synth_stage3":
        copies = 8
        Q, PI, QQ, QU, WANT, FINAL, _ = W.stage3_pipeline(z, copies)
        t0 = time.perf_counter()
        got_calls, got, st = ctx.stage3_compute(Q, PI, QQ, QU)
        dt = time.perf_counter() - t0
        check_compute(got_calls, got, FINAL, WANT, "x%d" % copies)
        print("stage3 compute (passes 2A-6): %d queries in %.3f s = %.0f queries/s (%d passes, %d rounds, windows %s; "
              "host steps %.3f s, passes %.3f s)" % (len(Q), dt, len(Q) / dt, st["passes"], st["rounds"],
                                                    st["windows"], st["seconds"][0], st["seconds"][1]))
    ctx.close()


@pytest.mark.parametrize("name", PIPE_NAMES + GSNAP_PIPE_NAMES)
def test_gpu_stage3_path_compute_matches_reference(golden_dir, tmp_path, name):
    """path_compute from pass 2A to its return value for every recorded
    invocation at once (gsnapdp_stage3_path_compute: passes 2A-10, the DP
    passes and assign_gap_types' MaxEnt sites on the GPU): the lists, the
    pairs' donor / acceptor probabilities, *intronlen / *nonintronlen /
    *defect_rate and the pass calls gmap made, bit for bit; then the synthetic
    set x8 in one call, each copy checked, timed.  The *_gsnap sets run with
    gsnap = 1 against path_compute as GSNAP builds it (oracle/pc_replay.c)"""
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    gsnap = bool(int(z["gsnap"])) if "gsnap" in z else False
    queries, pin, q, qu, want, wprobs, final = W.stage3_path_pipeline(z)
    ctx = Context(z["blocks"])
    s2 = stage2_double(ctx, z, tmp_path)
    maxintron = int(final["maxintronlen_bound"][0])
    got_calls, got, probs, st = ctx.stage3_path_compute(queries, pin, q, qu, maxintronlen_bound=maxintron,
                                                        gsnap=gsnap)
    check_path_compute(got_calls, got, probs, want, wprobs, final, name)
    assert list(st["pass_calls"]) == list(final["passes"].sum(axis=0))
    assert st["sites"] > 0
    if name == "gmap_synth_stage3":
        copies = 8
        Q, PI, QQ, QU, WANT, WP, FINAL = W.stage3_path_pipeline(z, copies)
        t0 = time.perf_counter()
        got_calls, got, probs, st = ctx.stage3_path_compute(Q, PI, QQ, QU, maxintronlen_bound=maxintron)
        dt = time.perf_counter() - t0
        check_path_compute(got_calls, got, probs, WANT, WP, FINAL, "x%d" % copies)
        print("stage3 path_compute (passes 2A-10): %d queries in %.3f s = %.0f queries/s (%d passes, %d rounds, "
              "windows %s, %d MaxEnt sites; host steps %.3f s, GPU %.3f s)" % (
                  len(Q), dt, len(Q) / dt, st["passes"], st["rounds"], st["windows"], st["sites"],
                  st["seconds"][0], st["seconds"][1]))
    ctx.close()


def test_gpu_stage3_pass_at_scale(golden_dir, tmp_path):
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    ctx = Context(z["blocks"])
    s2 = stage2_double(ctx, z, tmp_path)
    ctx.stage3_pass(calls[:8], pin, q, qu)  # warm-up (first launches, staging)
    copies = 16  # 7,424 paths
    C, PI, Q, QU, WANT = W.stage3_calls(z, copies)
    t0 = time.perf_counter()
    got_calls, got, st = ctx.stage3_pass(C, PI, Q, QU)
    dt = time.perf_counter() - t0
    check_pass(got_calls, got, C, WANT, "replicated x%d" % copies)
    nwin = int(np.sum(st["windows"]))
    ref = float(calls["ref_seconds"].sum()) * copies
    print("stage3 pass: %d paths in %.3f s (%d rounds; %d windows: %s; %d batches; host %.3f s, batches %.3f s) "
          "= %.0f paths/s, %.0f windows/s; reference build_pairs_introns (1 CPU thread) %.3f s = %.0f paths/s" %
          (len(C), dt, st["rounds"], nwin, st["windows"], int(np.sum(st["batches"])), st["seconds"][0],
           st["seconds"][1], len(C) / dt, nwin / dt, ref, len(C) / ref))
    ctx.close()


@pytest.mark.parametrize("name", ["gmap_synth_stage3", "gmap_cins_stage3", "gmap_dual_stage3"] + IIT_NAMES)
def test_dropin_build_pairs_introns_matches_reference(golden_dir, tmp_path, name):
    """Gsnapdp_build_pairs_introns, _singles, _end5, _dualintrons and
    Gsnapdp_build_path_end3 as stage3.c would call them (the reference's
    signature): the path as a List_T of the host's Pair_T cells, the counters
    as in/out arguments, the returned list (kept cells and pushed pairs, with
    disallowedp).  The IIT sets give Dynprog_setup a splicing IIT (the IIT test
    double over the golden's intervals, as test_dropin's genome-gap test does)."""
    import ctypes

    from gsnapdp.records import S3_DUALBREAKS, S3_DUALINTRONS, S3_END3, S3_END5, S3_PAIR, S3_SINGLES
    from test_dropin import SETUP_ARGS, load_iit_double

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    from doubles import pairpool_double
    dbl = pairpool_double()  # one copy per process: the drop-in binds Stage2_compute_one from the first one
    vp, i32, u8, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_ubyte, ctypes.c_uint
    dbl.dbl_s3_build.restype = vp
    dbl.dbl_s3_build.argtypes = [vp, i32]
    dbl.dbl_s3_read.restype = i32
    dbl.dbl_s3_read.argtypes = [vp, vp, i32]
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    L = ctypes.CDLL(os.path.join(root, "gmap-gsnap_amd", "lib", "libgsnapdp_dropin.so"))
    L.Gsnapdp_dropin_genome.argtypes = [vp, ctypes.c_size_t, i32]
    L.Dynprog_new.restype = vp
    L.Dynprog_new.argtypes = [i32] * 5
    L.Gsnapdp_build_pairs_singles.restype = vp
    L.Gsnapdp_build_pairs_singles.argtypes = [vp, vp, u32, u32, u32, u32, vp, vp, vp, vp, i32, u8, u8, i32, i32,
                                              i32, ctypes.c_double, i32, vp, vp]
    dbl_ = ctypes.c_double
    L.Gsnapdp_build_pairs_end5.restype = vp
    L.Gsnapdp_build_pairs_end5.argtypes = ([vp] * 5 + [vp, u32, u32, u32, i32, u32, u32, vp, vp, vp, vp, i32, u8, u8] +
                                           [i32] * 5 + [dbl_, vp, vp, u8, i32])
    L.Gsnapdp_build_path_end3.restype = vp
    L.Gsnapdp_build_path_end3.argtypes = ([vp] * 5 + [vp, u32, u32, u32, i32, i32, u32, u32, vp, vp, vp, vp, i32, u8,
                                                      u8] + [i32] * 5 + [dbl_, vp, vp, u8, i32])
    L.Gsnapdp_build_pairs_dualintrons.restype = vp
    L.Gsnapdp_build_pairs_dualintrons.argtypes = ([vp, vp, i32, u32, u32, u32, i32, vp, vp, vp, vp, u8, i32, u8, u8] +
                                                  [i32] * 4 + [dbl_, vp, vp, vp])
    L.Gsnapdp_build_dual_breaks.restype = vp
    L.Gsnapdp_build_dual_breaks.argtypes = ([vp, vp, vp, u32, u32, u32, u32, vp, vp, vp, vp, i32, u8, i32, u8, vp, vp,
                                             i32, vp, i32, vp, i32, i32, i32, i32, dbl_, i32])
    if "s2_calls" in z:  # traverse_dual_break's stage 2: the host's Stage2_compute_one, served by the double
        s2c, s2p = np.ascontiguousarray(z["s2_calls"]), np.ascontiguousarray(z["s2_pairs"])
        dbl.dbl_stage2_load(ctypes.c_void_p(s2c.ctypes.data), s2c.size, ctypes.c_void_p(s2p.ctypes.data))
    L.Gsnapdp_build_pairs_introns.restype = vp
    L.Gsnapdp_build_pairs_introns.argtypes = (
        [vp] * 8 + [vp, i32, u32, u32, u32, vp, i32, i32, vp, vp, vp, vp, u8, i32, u8, u8] + [i32] * 5 +
        [ctypes.c_double, i32, vp, vp, vp, vp, u8])
    calls, pin, q, qu, want = stage3_golden(z)
    assert (calls["maxlength1"] == 611).all() and (calls["maxlength2"] == 2000).all()
    blocks = np.ascontiguousarray(z["blocks"])
    L.Dynprog_term()  # a context an earlier test left holds another genome
    L.Dynprog_setup.argtypes = SETUP_ARGS
    iit = None
    if "intervals" in z:
        iv = iit_intervals(z)  # as the ggap_known_* sets store them: start, end, 0 none / 1 donor / 2 acceptor
        dz = {"intervals": np.stack([iv["start"].astype(np.int64), iv["end"].astype(np.int64),
                                     iv["type"].astype(np.int64) + 1], axis=1)}
        iitlib, iit, (dtype, atype) = load_iit_double(tmp_path, dz)
        crosstable = (ctypes.c_int * 2)(0, 0)  # the calls' chrnum 0 -> the IIT's one division
        L.Dynprog_setup(int(z["novelsplicingp"]), iit, ctypes.addressof(crosstable), dtype, atype,
                        None, None, None, 0, None, None, None, None, None)
    else:
        L.Dynprog_setup(1, None, None, -1, -1, None, None, None, 0, None, None, None, None, None)
    L.Gsnapdp_dropin_genome(blocks.ctypes.data, blocks.size, 0)
    dp = L.Dynprog_new(600, 10, 11, 10, 8)  # gmap.c's dynprogL / M / R: 611 x 2000
    qb = np.ascontiguousarray(q)
    qub = np.ascontiguousarray(qu)
    # which calls' intron lengths the reference took from uninitialised locals: the pass says
    ctx = Context(z["blocks"])
    siit = SplicingIIT(iit_intervals(z)) if iit is not None else None
    s2 = stage2_double(ctx, z, tmp_path)
    ub = (ctx.stage3_pass(calls, pin, q, qu, iit=siit)[0]["ub"] & 1) != 0
    ctx.close()
    nsingles = nother = 0
    for i, c in enumerate(calls):
        f0, n = int(c["first_pair"]), int(c["npairs"])
        recs = np.ascontiguousarray(pin[f0:f0 + n])
        lst = dbl.dbl_s3_build(recs.ctypes.data, n)
        shift, inc = ctypes.c_ubyte(7), ctypes.c_ubyte(7)
        ctr = [ctypes.c_int(int(c[f])) for f in ("in_nintrons", "in_nnonintrons", "in_intronlen",
                                                 "in_nonintronlen", "in_minor", "in_major")]
        qp = qb.ctypes.data + int(c["qpos"])
        qup = qub.ctypes.data + int(c["qpos"])
        exp = want[int(c["first_out"]):int(c["first_out"]) + int(c["nout"])]
        got = np.zeros(len(exp) + 1, S3_PAIR)
        if c["pass"] == S3_SINGLES:  # the golden's query is NUL-padded, as Sequence_fullpointer's
            ctr[4] = ctypes.c_int(int(c["in_minor"]))
            out = L.Gsnapdp_build_pairs_singles(
                ctypes.byref(ctr[4]), lst, int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]),
                int(c["genomiclength"]), qp, qup, None, None, int(c["cdna_direction"]), int(c["watsonp"]),
                int(c["jump_late_p"]), int(c["maxpeelback"]), int(c["nullgap"]), int(c["extraband_single"]),
                float(c["defect_rate"]), int(c["close_indels_mode"]), None, dp)
            k = dbl.dbl_s3_read(out, got.ctypes.data, got.size)
            assert k == len(exp) and got[:k].tobytes() == exp.tobytes(), i
            assert ctr[4].value == int(c["out_minor"]), i
            nsingles += 1
            continue
        if c["pass"] in (S3_END5, S3_END3):
            ks, ch = ctypes.c_ubyte(7), ctypes.c_ubyte(7)
            amb, ambt = ctypes.c_int(7), ctypes.c_int(0)
            minor = ctypes.c_int(int(c["in_minor"]))
            common = (int(c["cdna_direction"]), int(c["watsonp"]), int(c["jump_late_p"]), int(c["maxpeelback"]),
                      int(c["maxpeelback"]), int(c["nullgap"]), int(c["extramaterial_end"]), int(c["extraband_end"]),
                      float(c["defect_rate"]), None, dp, 1, int(c["endalign"]))
            head = (ctypes.byref(ks), ctypes.byref(amb), ctypes.byref(ambt), ctypes.byref(ch), ctypes.byref(minor), lst,
                    int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]))
            if c["pass"] == S3_END5:
                out = L.Gsnapdp_build_pairs_end5(*head, int(c["genomiclength"]), 0, 0, qp, qup, None, None, *common)
            else:
                out = L.Gsnapdp_build_path_end3(*head, int(c["querylength"]), int(c["genomiclength"]), 0, 0, qp, qup,
                                                None, None, *common)
            k = dbl.dbl_s3_read(out, got.ctypes.data, got.size)
            assert k == len(exp) and got[:k].tobytes() == exp.tobytes(), i
            assert minor.value == int(c["out_minor"]) and amb.value == 0, i
            if len(exp):  # extend_ending ran: no known splice, no chopped exon
                assert (ks.value, ch.value) == (0, 0), i
            nother += 1
            continue
        if c["pass"] == S3_DUALBREAKS:
            minor, dbp = ctypes.c_int(int(c["in_minor"])), ctypes.c_ubyte(7)
            out = L.Gsnapdp_build_dual_breaks(
                ctypes.byref(dbp), ctypes.byref(minor), lst, int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]),
                int(c["genomiclength"]), qp, qup, None, None, int(c["cdna_direction"]), int(c["watsonp"]), 0,
                int(c["jump_late_p"]), None, dp, int(c["maxpeelback"]), None, 0, None, 0, 0, 0,
                int(c["extraband_single"]), float(c["defect_rate"]), int(c["close_indels_mode"]))
            k = dbl.dbl_s3_read(out, got.ctypes.data, got.size)
            assert k == len(exp) and got[:k].tobytes() == exp.tobytes(), i
            assert minor.value == int(c["out_minor"]) and dbp.value == int(c["shiftp"]), i
            nother += 1
            continue
        if c["pass"] == S3_DUALINTRONS:
            major = ctypes.c_int(int(c["in_major"]))
            out = L.Gsnapdp_build_pairs_dualintrons(
                ctypes.byref(major), lst, int(c["chrnum"]), int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]),
                int(c["genomiclength"]), qp, qup, None, None, 0, int(c["cdna_direction"]), int(c["watsonp"]),
                int(c["jump_late_p"]), int(c["maxpeelback"]), int(c["nullgap"]), int(c["extramaterial_paired"]),
                int(c["extraband_paired"]), float(c["defect_rate"]), None, dp, dp)
            k = dbl.dbl_s3_read(out, got.ctypes.data, got.size)
            assert k == len(exp) and got[:k].tobytes() == exp.tobytes(), i
            assert major.value == int(c["out_major"]), i
            nother += 1
            continue
        out = L.Gsnapdp_build_pairs_introns(
            ctypes.byref(shift), ctypes.byref(inc), *[ctypes.byref(x) for x in ctr], lst, int(c["chrnum"]),
            int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]), None, int(c["querylength"]),
            int(c["genomiclength"]), qp, qup, None, None, 0, int(c["cdna_direction"]), int(c["watsonp"]),
            int(c["jump_late_p"]), int(c["maxpeelback"]), int(c["nullgap"]), int(c["extramaterial_paired"]),
            int(c["extraband_single"]), int(c["extraband_paired"]), float(c["defect_rate"]),
            int(c["close_indels_mode"]), None, dp, dp, dp, int(c["finalp"]))
        k = dbl.dbl_s3_read(out, got.ctypes.data, got.size)
        assert k == len(exp), (i, k, len(exp))
        assert got[:k].tobytes() == exp.tobytes(), i
        assert (shift.value, inc.value) == (int(c["shiftp"]), int(c["incompletep"])), i
        fields = ("out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen", "out_minor", "out_major")
        skip = ub[i] if ub is not None else False  # the reference's own intron lengths are garbage there
        assert [x.value for j, x in enumerate(ctr) if not (skip and j in (2, 3))] == [
            int(c[f]) for j, f in enumerate(fields) if not (skip and j in (2, 3))], i
    assert nsingles == int((calls["pass"] == S3_SINGLES).sum())
    assert nother == int(np.isin(calls["pass"], (S3_END5, S3_END3, S3_DUALINTRONS, S3_DUALBREAKS)).sum())
    if iit is not None:  # back to no IIT for the other tests of this process
        L.Dynprog_setup(1, None, None, -1, -1, None, None, None, 0, None, None, None, None, None)
    L.Dynprog_term()  # releases the device context (the genome array dies with this test)


def test_gpu_stage3_concurrent_passes_on_one_context(golden_dir, tmp_path):
    """Three host threads running whole passes (and a 2A-6 pipeline) on ONE
    context at once: each pass takes its own executor (staging, launcher
    thread) from the context's pool, the rounds of all passes share the context
    stream in submission order, and every result equals the serial run's."""
    import threading
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    Q, PI, QQ, QU, WANT, FINAL, counts = W.stage3_pipeline(z)
    ctx = Context(z["blocks"])
    s2 = stage2_double(ctx, z, tmp_path)
    c0, g0, _ = ctx.stage3_pass(calls, pin, q, qu)
    check_pass(c0, g0, calls, want, "serial", z["ub_ref"] if "ub_ref" in z else None)
    k0, l0, _ = ctx.stage3_compute(Q, PI, QQ, QU)
    out, errs = {}, []

    def worker(t):
        try:
            for r in range(3):
                if t == 2:
                    k, l, _ = ctx.stage3_compute(Q, PI, QQ, QU)
                    out[(t, r)] = (k.tobytes() == k0.tobytes(), l.tobytes() == l0.tobytes())
                else:
                    c, g, _ = ctx.stage3_pass(calls, pin, q, qu)
                    out[(t, r)] = (c.tobytes() == c0.tobytes(), g.tobytes() == g0.tobytes())
        except Exception as e:  # reported below
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errs, errs
    assert len(out) == 9 and all(a and b for a, b in out.values()), out
    ctx.close()
