"""The stage-3 intron pass on the GPU (gsnapdp_stage3_pass: build_pairs_introns,
stage3.c:7735-7901, for many paths at once, every round one batch per gap
family) against every recorded build_pairs_introns call of the reference's gmap
(tests/golden/gmap_*_stage3.npz; see test_stage3_cpu.py), and at scale: the
synthetic calls replicated into one pass of thousands of paths, each copy
checked against the reference, with the pass's throughput printed beside the
reference's own time for the same calls (its build_pairs_introns wall time in
gmap_trace, DP included)."""
import os
import time

import numpy as np
import pytest

from gsnapdp import Context
from gsnapdp import workload as W
from test_stage3_cpu import NAMES, check_pass, stage3_golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", NAMES)
def test_gpu_stage3_pass_matches_reference(golden_dir, name):
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    ctx = Context(z["blocks"])
    got_calls, got, st = ctx.stage3_pass(calls, pin, q, qu)
    check_pass(got_calls, got, calls, want, name)
    assert st["failed"] == 0 and st["undefined"] == 0
    print("%s: %d calls, %d rounds, windows %s in batches %s" % (name, len(calls), st["rounds"], st["windows"],
                                                                st["batches"]))
    ctx.close()


def test_gpu_stage3_pass_at_scale(golden_dir):
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    ctx = Context(z["blocks"])
    ctx.stage3_pass(calls[:8], pin, q, qu)  # warm-up (first launches, staging)
    copies = 64
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


def test_dropin_build_pairs_introns_matches_reference(golden_dir, tmp_path):
    """Gsnapdp_build_pairs_introns as stage3.c would call it (the reference's
    signature): the path as a List_T of the host's Pair_T cells, the counters
    as in/out arguments, the returned list (kept cells and pushed pairs)."""
    import ctypes
    import subprocess

    from gsnapdp.records import S3_PAIR

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(str(tmp_path), "libpairpool_double.so")
    subprocess.check_call(["gcc", "-O1", "-shared", "-fPIC", "-o", so,
                           os.path.join(root, "tests", "dropin", "pairpool_double.c")])
    dbl = ctypes.CDLL(so, mode=ctypes.RTLD_GLOBAL)
    vp, i32, u8, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_ubyte, ctypes.c_uint
    dbl.dbl_s3_build.restype = vp
    dbl.dbl_s3_build.argtypes = [vp, i32]
    dbl.dbl_s3_read.restype = i32
    dbl.dbl_s3_read.argtypes = [vp, vp, i32]
    L = ctypes.CDLL(os.path.join(root, "gmap-gsnap_amd", "lib", "libgsnapdp_dropin.so"))
    L.Gsnapdp_dropin_genome.argtypes = [vp, ctypes.c_size_t, i32]
    L.Dynprog_new.restype = vp
    L.Dynprog_new.argtypes = [i32] * 5
    L.Gsnapdp_build_pairs_introns.restype = vp
    L.Gsnapdp_build_pairs_introns.argtypes = (
        [vp] * 8 + [vp, i32, u32, u32, u32, vp, i32, i32, vp, vp, vp, vp, u8, i32, u8, u8] + [i32] * 5 +
        [ctypes.c_double, i32, vp, vp, vp, vp, u8])
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    assert (calls["maxlength1"] == 611).all() and (calls["maxlength2"] == 2000).all()
    blocks = np.ascontiguousarray(z["blocks"])
    L.Dynprog_term()  # a context an earlier test left holds another genome
    L.Gsnapdp_dropin_genome(blocks.ctypes.data, blocks.size, 0)
    dp = L.Dynprog_new(600, 10, 11, 10, 8)  # gmap.c's dynprogL / M / R: 611 x 2000
    qb = np.ascontiguousarray(q)
    qub = np.ascontiguousarray(qu)
    for i, c in enumerate(calls):
        f0, n = int(c["first_pair"]), int(c["npairs"])
        recs = np.ascontiguousarray(pin[f0:f0 + n])
        lst = dbl.dbl_s3_build(recs.ctypes.data, n)
        shift, inc = ctypes.c_ubyte(7), ctypes.c_ubyte(7)
        ctr = [ctypes.c_int(int(c[f])) for f in ("in_nintrons", "in_nnonintrons", "in_intronlen",
                                                 "in_nonintronlen", "in_minor", "in_major")]
        qp = qb.ctypes.data + int(c["qpos"])
        qup = qub.ctypes.data + int(c["qpos"])
        out = L.Gsnapdp_build_pairs_introns(
            ctypes.byref(shift), ctypes.byref(inc), *[ctypes.byref(x) for x in ctr], lst, int(c["chrnum"]),
            int(c["chroffset"]), int(c["chrhigh"]), int(c["chrpos"]), None, int(c["querylength"]),
            int(c["genomiclength"]), qp, qup, None, None, 0, int(c["cdna_direction"]), int(c["watsonp"]),
            int(c["jump_late_p"]), int(c["maxpeelback"]), int(c["nullgap"]), int(c["extramaterial_paired"]),
            int(c["extraband_single"]), int(c["extraband_paired"]), float(c["defect_rate"]),
            int(c["close_indels_mode"]), None, dp, dp, dp, int(c["finalp"]))
        exp = want[int(c["first_out"]):int(c["first_out"]) + int(c["nout"])]
        got = np.zeros(len(exp) + 1, S3_PAIR)
        k = dbl.dbl_s3_read(out, got.ctypes.data, got.size)
        assert k == len(exp), (i, k, len(exp))
        assert got[:k].tobytes() == exp.tobytes(), i
        assert (shift.value, inc.value) == (int(c["shiftp"]), int(c["incompletep"])), i
        assert [x.value for x in ctr] == [int(c[f]) for f in ("out_nintrons", "out_nnonintrons", "out_intronlen",
                                                              "out_nonintronlen", "out_minor", "out_major")], i
    L.Dynprog_term()  # releases the device context (the genome array dies with this test)
