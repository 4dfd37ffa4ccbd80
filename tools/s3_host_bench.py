"""Times the stage-3 pass's own host work on the CPU (no GPU): the recorded
build_pairs_introns calls replicated COPIES times, run through
oracle/_build/stage3_cpu_fast (gsnapdp_stage3.cpp with its batches served by
the oracle's restatement, tests/dropin/stage3_exec_host.cpp).  The pass's host
work is its wall time minus the time the oracle spent serving the batches.

    python tools/s3_host_bench.py [COPIES] [THREADS] [golden name]"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import workload as W  # noqa: E402


def main():
    copies = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    threads = sys.argv[2] if len(sys.argv) > 2 else str(os.cpu_count())
    name = sys.argv[3] if len(sys.argv) > 3 else "gmap_synth_stage3"
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu_fast"])
    z = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    calls, pin, q, qu, want = W.stage3_calls(z, copies)
    with tempfile.TemporaryDirectory() as d:
        calls.tofile(os.path.join(d, "calls.bin"))
        pin.tofile(os.path.join(d, "pairs_in.bin"))
        q.tofile(os.path.join(d, "query.bin"))
        qu.tofile(os.path.join(d, "query_uc.bin"))
        z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
        if "s2_calls" in z:  # build_dual_breaks' stage 2, from the recording
            z["s2_calls"].tofile(os.path.join(d, "stage2_calls.bin"))
            z["s2_pairs"].tofile(os.path.join(d, "stage2_pairs.bin"))
        env = dict(os.environ, GSNAPDP_S3_THREADS=threads,
                   GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
        p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu_fast"), d], env=env,
                           capture_output=True, text=True, check=True)
    print("%d paths, %s threads: %s" % (len(calls), threads, p.stderr.strip()))


if __name__ == "__main__":
    main()
