"""The stage-3 passes (gsnapdp_stage3_pass: build_pairs_introns
stage3.c:7735-7901 and build_pairs_singles :7454-7583 over many paths) on the
CPU, against the reference.

gmap_trace recorded every build_pairs_introns and build_pairs_singles call the
reference's gmap made
(ss.her2 against ss.chr17test, and the synthetic spliced cDNAs): the path it was
given, its arguments and counters, and the list it returned
(tests/golden/gmap_*_stage3.npz, oracle/gen_golden.py stage3_golden).  Here the
pass's host control flow (gmap-gsnap_amd/csrc/gsnapdp_stage3.cpp) runs with its
gap families served by the oracle's restatement (tests/dropin/gsnapdp_oracle_abi.c),
built under AddressSanitizer + UBSan (oracle/Makefile `stage3_cpu`), and must
return the reference's lists cell for cell.  tests/test_gpu_stage3.py runs the
same calls with the gap families on the GPU."""
import os
import subprocess

import numpy as np
import pytest

from gsnapdp import workload as W
from gsnapdp.records import S3_CALL, S3_PAIR, S3_SINGLES, S3_STATS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["gmap_her2_stage3", "gmap_synth_stage3", "gmap_cins_stage3", "gmap_dual_stage3"]
# the cDNA-insertion calls replayed through the reference with a splicing IIT
# (oracle/gen_golden.py gmap_cins_case): site-level with and without novel
# splicing, intron-level without
IIT_NAMES = ["gmap_cins_iit_sites_novel", "gmap_cins_iit_sites", "gmap_cins_iit_introns"]
UB_COUNTERS = ("out_intronlen", "out_nonintronlen")
COUNTERS = ["out_minor", "out_major", "out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen",
            "shiftp", "incompletep", "nout"]


def stage3_golden(z):
    """(calls, pairs_in, query, query_uc, the expected returned lists concatenated)."""
    return W.stage3_calls(z)


def check_pass(calls, out, want_calls, want_out, what, ub_ref=None):
    """the pass's counters and lists against the reference's, call by call.
    The intron-length counters are skipped where the pass reports that the
    reference read traverse_genome_gap's uninitialised locals (calls["ub"]);
    `ub_ref` marks the calls where two runs of the reference itself disagree
    there, and the pass must report every one of them."""
    assert (calls["status"] == 0).all(), "%s: failed calls %s" % (what, np.nonzero(calls["status"])[0][:8])
    ub = (calls["ub"] & 1) != 0
    if ub_ref is not None:
        miss = np.nonzero((np.asarray(ub_ref) != 0) & ~ub)[0]
        assert miss.size == 0, "%s: reference garbage not flagged at calls %s" % (what, miss[:8])
    for f in COUNTERS:
        bad = np.nonzero((calls[f] != want_calls[f]) & ~(ub if f in UB_COUNTERS else False))[0]
        assert bad.size == 0, "%s: %s differs at calls %s (got %s want %s)" % (
            what, f, bad[:8], calls[f][bad[:8]], want_calls[f][bad[:8]])
    for i, (c, w) in enumerate(zip(calls, want_calls)):
        got = out[int(c["first_out"]):int(c["first_out"]) + int(c["nout"])]
        exp = want_out[int(w["first_out"]):int(w["first_out"]) + int(w["nout"])]
        if got.tobytes() != exp.tobytes():
            k = int(np.nonzero(got != exp)[0][0])
            raise AssertionError("%s: call %d, cell %d of %d: got %s want %s" % (what, i, k, len(exp), got[k], exp[k]))


def write_stage2(d, z):
    """traverse_dual_break's recorded stage-2 lists, for the driver's stage-2 callback"""
    if "s2_calls" in z:
        z["s2_calls"].tofile(os.path.join(d, "stage2_calls.bin"))
        z["s2_pairs"].tofile(os.path.join(d, "stage2_pairs.bin"))


def run_stage3_cpu(d, z, calls, pin, q, qu, intervals=None, introns=False):
    """stage3_cpu (ASan + UBSan) on the calls; returns (calls, lists, stats[, scores])"""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu"])
    calls.tofile(os.path.join(d, "calls.bin"))
    pin.tofile(os.path.join(d, "pairs_in.bin"))
    q.tofile(os.path.join(d, "query.bin"))
    qu.tofile(os.path.join(d, "query_uc.bin"))
    z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
    write_stage2(d, z)
    if intervals is not None:
        intervals.tofile(os.path.join(d, "intervals.bin"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu"), d] + (["--introns"] if introns else []),
                       env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, "stage3_cpu failed (%d):\n%s" % (p.returncode, p.stderr[-6000:])
    assert "runtime error" not in p.stderr, p.stderr[-6000:]
    got_calls = np.fromfile(os.path.join(d, "pass_calls.bin"), dtype=S3_CALL)
    got = np.fromfile(os.path.join(d, "pass_pairs.bin"), dtype=S3_PAIR)
    st = np.fromfile(os.path.join(d, "pass_stats.bin"), dtype=S3_STATS)[0]
    if introns:
        from gsnapdp.records import INTRON_SCORES
        return got_calls, got, st, np.fromfile(os.path.join(d, "pass_scores.bin"), dtype=INTRON_SCORES)
    return got_calls, got, st


def test_stage3_pass_cpu_two_cohorts(golden_dir, tmp_path):
    """enough paths (the synthetic calls x3) for the pass's two cohorts in flight"""
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = W.stage3_calls(z, 3)
    assert len(calls) >= 256
    got_calls, got, st = run_stage3_cpu(str(tmp_path), z, calls, pin, q, qu)
    check_pass(got_calls, got, calls, want, "x3")
    assert st["failed"] == 0 and st["undefined"] == 0


@pytest.mark.parametrize("name", NAMES)
def test_stage3_pass_cpu_matches_reference(golden_dir, tmp_path, name):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu"])
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    d = str(tmp_path)
    calls.tofile(os.path.join(d, "calls.bin"))
    pin.tofile(os.path.join(d, "pairs_in.bin"))
    q.tofile(os.path.join(d, "query.bin"))
    qu.tofile(os.path.join(d, "query_uc.bin"))
    z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
    write_stage2(d, z)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu"), d], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, "stage3_cpu failed (%d):\n%s" % (p.returncode, p.stderr[-6000:])
    assert "runtime error" not in p.stderr, p.stderr[-6000:]
    got_calls = np.fromfile(os.path.join(d, "pass_calls.bin"), dtype=S3_CALL)
    got = np.fromfile(os.path.join(d, "pass_pairs.bin"), dtype=S3_PAIR)
    st = np.fromfile(os.path.join(d, "pass_stats.bin"), dtype=S3_STATS)[0]
    check_pass(got_calls, got, calls, want, name, z["ub_ref"] if "ub_ref" in z else None)
    assert st["failed"] == 0 and st["undefined"] == 0
    assert st["windows"][1] > 0  # genome gaps were exercised
    if name != "gmap_dual_stage3":
        assert st["windows"][3] > 0  # and microexons
    else:  # traverse_dual_genome_gap's windows, the reference's dynprogindex_major steps
        assert st["windows"][1] == int((calls["in_major"] - calls["out_major"]).sum()) >= 300
    if name == "gmap_cins_stage3":
        assert st["windows"][2] >= 200  # traverse_cdna_gap's Dynprog_cdna_gap windows


def test_stage3_golden_covers_the_branches(golden_dir):
    """what the recorded calls exercise: final and non-final passes, filled
    genome gaps (new gapholders), shifted introns, both cDNA directions"""
    z = np.load(os.path.join(golden_dir, "gmap_synth_stage3.npz"), allow_pickle=False)
    c = z["calls"]
    assert (c["finalp"] == 1).any() and (c["finalp"] == 0).any()
    assert (c["shiftp"] == 1).any()
    assert set(np.unique(c["cdna_direction"])) == {-1, 1}
    new = z["out_new"]
    assert ((new["flags"] & 1) == 1).any()  # gapholders made by the genome-gap fills
    assert (c["out_nintrons"] > c["in_nintrons"]).any()
    # build_pairs_singles calls (passes 2A / 2C / 7C of path_compute) among them,
    # some of whose single gaps were filled by traverse_single_gap
    singles = c["pass"] == S3_SINGLES
    assert singles.sum() >= 100 and (c["out_minor"][singles] > c["in_minor"][singles]).any()


def iit_intervals(z):
    from gsnapdp.records import IIT_INTERVAL
    return np.ascontiguousarray(z["intervals"], dtype=IIT_INTERVAL)


def check_scores(scores, calls, si_calls, what):
    """score_introns on every returned list against the reference's (s3_replay --si)"""
    assert len(scores) == len(si_calls)
    for f in ("avg_donor_score", "avg_acceptor_score"):
        bad = np.nonzero(scores[f].view(np.uint64) != si_calls[f].astype(np.float64).view(np.uint64))[0]
        assert bad.size == 0, "%s: %s differs at calls %s" % (what, f, bad[:8])
    bad = np.nonzero(scores["nbadintrons"] != si_calls["nbadintrons"])[0]
    assert bad.size == 0, "%s: nbadintrons differs at calls %s" % (what, bad[:8])


@pytest.mark.parametrize("name", IIT_NAMES)
def test_stage3_pass_cpu_with_splicing_iit(golden_dir, tmp_path, name):
    """the pass with a splicing IIT (every genome-gap window's known-site record,
    gsnapdp_known_site_record) and score_introns on its lists with the IIT's
    verdicts, against the reference's build_pairs_introns / score_introns run
    with the same IIT (oracle/s3_replay.c)"""
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    calls, pin, q, qu, want = stage3_golden(z)
    got_calls, got, st, scores = run_stage3_cpu(str(tmp_path), z, calls, pin, q, qu, iit_intervals(z), introns=True)
    check_pass(got_calls, got, calls, want, name)
    assert st["failed"] == 0 and st["undefined"] == 0
    check_scores(scores, got_calls, z["si_calls"], name)


PIPE_NAMES = ["gmap_her2_stage3", "gmap_synth_stage3"]
# the same invocations through path_compute as GSNAP builds it (-DGSNAP; oracle/pc_replay.c)
GSNAP_PIPE_NAMES = ["gmap_her2_stage3_gsnap", "gmap_synth_stage3_gsnap"]


def check_compute(got_calls, got, final, want, what):
    """gsnapdp_stage3_compute's lists and counters against the pass-6 calls gmap made"""
    assert (got_calls["status"] == 0).all(), "%s: failed queries %s" % (what, np.nonzero(got_calls["status"])[0][:8])
    ub = (got_calls["ub"] & 1) != 0
    for f in COUNTERS:
        bad = np.nonzero((got_calls[f] != final[f]) & ~(ub if f in UB_COUNTERS else False))[0]
        assert bad.size == 0, "%s: %s differs at queries %s (got %s want %s)" % (
            what, f, bad[:8], got_calls[f][bad[:8]], final[f][bad[:8]])
    bad = np.nonzero(got_calls["defect_rate"].view(np.uint64) != final["defect_rate"].view(np.uint64))[0]
    assert bad.size == 0, "%s: defect_rate differs at queries %s" % (what, bad[:8])
    for i, (c, w) in enumerate(zip(got_calls, final)):
        g = got[int(c["first_out"]):int(c["first_out"]) + int(c["nout"])].copy()
        e = want[int(w["first_out"]):int(w["first_out"]) + int(w["nout"])].copy()
        g["src"] = e["src"] = -1  # the pipeline's cells are its own
        if g.tobytes() != e.tobytes():
            k = int(np.nonzero(g != e)[0][0]) if len(g) == len(e) else min(len(g), len(e))
            raise AssertionError("%s: query %d (invocation %d): %d cells, want %d; first difference at %d: "
                                 "got %s want %s" % (what, i, int(c["invocation"]), len(g), len(e), k,
                                                     g[k] if k < len(g) else None, e[k] if k < len(e) else None))


@pytest.mark.parametrize("name", PIPE_NAMES)
def test_stage3_compute_cpu_matches_reference(golden_dir, tmp_path, name):
    """passes 2A-6 of path_compute (gsnapdp_stage3_compute: the host steps
    restated, the DP passes batched across queries) from each recorded
    invocation's pass-2A path to the list its pass 6 returned, bit for bit, with
    the DP families served by the oracle and traverse_dual_break's stage 2 by
    the recording"""
    from gsnapdp.records import S3_CALL, S3_PAIR
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    queries, pin, q, qu, want, final, counts = W.stage3_pipeline(z)
    assert len(queries) >= (2 if name == "gmap_her2_stage3" else 150)
    d = str(tmp_path)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu"])
    queries.tofile(os.path.join(d, "calls.bin"))
    pin.tofile(os.path.join(d, "pairs_in.bin"))
    q.tofile(os.path.join(d, "query.bin"))
    qu.tofile(os.path.join(d, "query_uc.bin"))
    z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
    write_stage2(d, z)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu"), d, "--compute", "9"], env=env,
                       capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, "stage3_cpu --compute failed (%d):\n%s" % (p.returncode, p.stderr[-6000:])
    assert "runtime error" not in p.stderr, p.stderr[-6000:]
    got_calls = np.fromfile(os.path.join(d, "pass_calls.bin"), dtype=S3_CALL)
    got = np.fromfile(os.path.join(d, "pass_pairs.bin"), dtype=S3_PAIR)
    check_compute(got_calls, got, final, want, name)
    from gsnapdp.records import S3_COMPUTE_STATS
    cs = np.fromfile(os.path.join(d, "compute_stats.bin"), dtype=S3_COMPUTE_STATS)[0]
    # the same pass calls as gmap made up to pass 6: 2A / 2C singles, dual introns, introns, dual breaks
    assert list(cs["pass_calls"]) == list(counts.sum(axis=0)), (cs["pass_calls"], counts.sum(axis=0))


def check_path_compute(got_calls, got, probs, want, want_probs, final, what):
    """gsnapdp_stage3_path_compute's lists, pair probabilities and outputs
    against what path_compute returned in gmap (tests/golden pc_*)"""
    assert (got_calls["status"] == 0).all(), "%s: failed queries %s" % (what, np.nonzero(got_calls["status"])[0][:8])
    ub = (got_calls["ub"] & 1) != 0
    for f, g in (("intronlen", "out_intronlen"), ("nonintronlen", "out_nonintronlen")):
        bad = np.nonzero((got_calls[g] != final[f]) & ~ub)[0]
        assert bad.size == 0, "%s: %s differs at queries %s" % (what, f, bad[:8])
    bad = np.nonzero(got_calls["defect_rate"].view(np.uint64) != final["defect_rate"].view(np.uint64))[0]
    assert bad.size == 0, "%s: defect_rate differs at queries %s" % (what, bad[:8])
    for i, (c, w) in enumerate(zip(got_calls, final)):
        a, n = int(c["first_out"]), int(c["nout"])
        b, m = int(w["first_out"]), int(w["nout"])
        g, e = got[a:a + n].copy(), want[b:b + m].copy()
        g["src"] = e["src"] = -1
        if g.tobytes() != e.tobytes():
            k = int(np.nonzero(g != e)[0][0]) if n == m else min(n, m)
            raise AssertionError("%s: query %d (invocation %d): %d cells, want %d; first difference at %d: "
                                 "got %s want %s" % (what, i, int(c["invocation"]), n, m, k,
                                                     g[k] if k < n else None, e[k] if k < m else None))
        gp, ep = probs[a:a + n], want_probs[b:b + m]
        if gp.tobytes() != ep.tobytes():
            k = int(np.nonzero((gp != ep).any(axis=1))[0][0])
            raise AssertionError("%s: query %d pair %d: probabilities %s, want %s" % (what, i, k, gp[k], ep[k]))


@pytest.mark.parametrize("name", PIPE_NAMES + GSNAP_PIPE_NAMES)
def test_stage3_path_compute_cpu_matches_reference(golden_dir, tmp_path, name):
    """path_compute from pass 2A to its return value (passes 2A-10: the dual
    breaks at the ends, the adjacent indels, the end extensions,
    assign_gap_types with its MaxEnt probabilities and the noncanonical
    end-exon trims; gsnapdp_stage3_path_compute) for every recorded
    invocation, bit for bit: the returned list, every pair's
    donor_prob / acceptor_prob, *intronlen, *nonintronlen, *defect_rate and
    the pass calls made, with the DP families and MaxEnt served by the oracle
    under ASan + UBSan.  The *_gsnap sets hold what the reference's path_compute
    returns when built as GSNAP builds it (-DGSNAP, oracle/pc_replay.c) on the
    same invocations, and run with gsnap = 1"""
    from gsnapdp.records import S3_COMPUTE_STATS, S3_CALL, S3_PAIR
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    gsnap = int(z["gsnap"]) if "gsnap" in z else 0
    queries, pin, q, qu, want, want_probs, final = W.stage3_path_pipeline(z)
    assert len(queries) == len(z["pc_calls"])
    d = str(tmp_path)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu"])
    queries.tofile(os.path.join(d, "calls.bin"))
    pin.tofile(os.path.join(d, "pairs_in.bin"))
    q.tofile(os.path.join(d, "query.bin"))
    qu.tofile(os.path.join(d, "query_uc.bin"))
    z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
    write_stage2(d, z)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
    maxintron = int(final["maxintronlen_bound"][0])
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu"), d, "--path-compute", "9",
                        str(maxintron), str(gsnap)], env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, "stage3_cpu --path-compute failed (%d):\n%s" % (p.returncode, p.stderr[-6000:])
    assert "runtime error" not in p.stderr, p.stderr[-6000:]
    got_calls = np.fromfile(os.path.join(d, "pass_calls.bin"), dtype=S3_CALL)
    got = np.fromfile(os.path.join(d, "pass_pairs.bin"), dtype=S3_PAIR)
    probs = np.fromfile(os.path.join(d, "pass_probs.bin"), dtype=np.float64).reshape(-1, 2)
    check_path_compute(got_calls, got, probs, want, want_probs, final, name)
    cs = np.fromfile(os.path.join(d, "compute_stats.bin"), dtype=S3_COMPUTE_STATS)[0]
    assert list(cs["pass_calls"]) == list(final["passes"].sum(axis=0)), (cs["pass_calls"], final["passes"].sum(0))
    assert cs["sites"] > 0
