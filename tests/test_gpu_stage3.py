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


def replicate(calls, pin, q, qu, want, copies):
    """`copies` copies of every call, in one set of buffers"""
    n = len(calls)
    C = np.tile(calls, copies)
    k = np.repeat(np.arange(copies), n)
    C["first_pair"] += (k * pin.size).astype(np.int32)
    C["qpos"] += (k * q.size).astype(np.int32)
    C["first_out"] += (k * want.size).astype(np.int32)
    return C, np.tile(pin, copies), np.tile(q, copies), np.tile(qu, copies), np.tile(want, copies)


def test_gpu_stage3_pass_at_scale(golden_dir):
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    ctx = Context(z["blocks"])
    ctx.stage3_pass(calls[:8], pin, q, qu)  # warm-up (first launches, staging)
    copies = 64
    C, PI, Q, QU, WANT = replicate(calls, pin, q, qu, want, copies)
    t0 = time.perf_counter()
    got_calls, got, st = ctx.stage3_pass(C, PI, Q, QU)
    dt = time.perf_counter() - t0
    check_pass(got_calls, got, C, WANT, "replicated x%d" % copies)
    nwin = int(np.sum(st["windows"]))
    ref = float(calls["ref_seconds"].sum()) * copies
    print("stage3 pass: %d paths in %.3f s (%d rounds; %d windows: %s; %d batches) = %.0f paths/s, %.0f windows/s; "
          "reference build_pairs_introns (1 CPU thread) %.3f s = %.0f paths/s" %
          (len(C), dt, st["rounds"], nwin, st["windows"], int(np.sum(st["batches"])), len(C) / dt, nwin / dt, ref,
           len(C) / ref))
    ctx.close()
