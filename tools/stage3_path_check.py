"""Every path_compute call of a recorded gmap run (TRACE.npz, tools/make_stage3_trace.py)
from its pass-2A path to its return value through gsnapdp_stage3_path_compute on
the CPU under ASan + UBSan (oracle/_build/stage3_cpu: the DP families and MaxEnt
served by the oracle/ restatement), checked against what path_compute returned in
gmap: lists, pair probabilities, *intronlen / *nonintronlen / *defect_rate, pass
calls.  Dev container (no GPU).

    python tools/stage3_path_check.py TRACE.npz"""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import S3_CALL, S3_COMPUTE_STATS, S3_PAIR  # noqa: E402
from test_stage3_cpu import check_path_compute  # noqa: E402


def main():
    z = np.load(sys.argv[1], allow_pickle=False)
    queries, pin, q, qu, want, wprobs, final = W.stage3_path_pipeline(z)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu"])
    with tempfile.TemporaryDirectory() as d:
        queries.tofile(os.path.join(d, "calls.bin"))
        pin.tofile(os.path.join(d, "pairs_in.bin"))
        q.tofile(os.path.join(d, "query.bin"))
        qu.tofile(os.path.join(d, "query_uc.bin"))
        z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
        z["s2_calls"].tofile(os.path.join(d, "stage2_calls.bin"))
        z["s2_pairs"].tofile(os.path.join(d, "stage2_pairs.bin"))
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
                   GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
        t0 = time.time()
        p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu"), d, "--path-compute", "9",
                            str(int(final["maxintronlen_bound"][0]))], env=env, capture_output=True, text=True)
        assert p.returncode == 0 and "runtime error" not in p.stderr, p.stderr[-4000:]
        got_calls = np.fromfile(os.path.join(d, "pass_calls.bin"), dtype=S3_CALL)
        got = np.fromfile(os.path.join(d, "pass_pairs.bin"), dtype=S3_PAIR)
        probs = np.fromfile(os.path.join(d, "pass_probs.bin"), dtype=np.float64).reshape(-1, 2)
        cs = np.fromfile(os.path.join(d, "compute_stats.bin"), dtype=S3_COMPUTE_STATS)[0]
    check_path_compute(got_calls, got, probs, want, wprobs, final, os.path.basename(sys.argv[1]))
    assert list(cs["pass_calls"]) == list(final["passes"].sum(axis=0))
    print("%s: %d path_compute calls bit-exact from pass 2A to the returned list (%d pairs, %d with probabilities), "
          "pass calls %s, %d MaxEnt sites, %d rounds; CPU under ASan + UBSan, %.1f s" %
          (os.path.basename(sys.argv[1]), len(queries), got.size, int((probs != 0).any(axis=1).sum()),
           list(cs["pass_calls"]), cs["sites"], cs["rounds"], time.time() - t0))


if __name__ == "__main__":
    main()
