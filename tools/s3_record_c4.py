"""PROFILING INFRASTRUCTURE ONLY: records the C4 transcript pass
(gsnapdp_stage3_pass_runs, bench.measure_c4_transcripts' call) on the GPU with
GSNAPDP_S3_RECORD set, so that its host work can be replayed and profiled on
a machine without a GPU (oracle/_build/stage3_host_replay DIR).

    GPU box:  GSNAPDP_S3_RECORD=DIR python tools/s3_record_c4.py DIR N --gpu
              (the rounds, plus the pass's runs / new pairs as the GPU made them)
    here:     python tools/s3_record_c4.py DIR N --inputs
              (the same deterministic workload's inputs beside them)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))


def main():
    d = sys.argv[1]
    n = int(sys.argv[2])
    os.makedirs(d, exist_ok=True)
    from gsnapdp import gap_lists
    from gsnapdp import workload as W
    w = W.c4_transcripts(n)
    gaps, gap_off = gap_lists(w.calls, w.pairs_in)
    if "--inputs" in sys.argv:
        w.calls.tofile(os.path.join(d, "calls.bin"))
        w.pairs_in.tofile(os.path.join(d, "pairs_in.bin"))
        w.query.tofile(os.path.join(d, "query.bin"))
        w.query_uc.tofile(os.path.join(d, "query_uc.bin"))
        np.asarray(w.blocks, dtype="<u4").tofile(os.path.join(d, "genome.u32"))
        np.asarray(gaps, dtype="<i4").tofile(os.path.join(d, "gaps.bin"))
        np.asarray(gap_off, dtype="<i8").tofile(os.path.join(d, "gap_off.bin"))
        open(os.path.join(d, "pairs_out.bin"), "wb").close()
        return
    from gsnapdp import Context
    assert os.environ.get("GSNAPDP_S3_RECORD") == d, "set GSNAPDP_S3_RECORD=DIR"
    ctx = Context(w.blocks)
    c, runs, new, st, _ = ctx.stage3_pass_runs(w.calls, w.pairs_in, w.query, w.query_uc, gaps, gap_off)
    runs.tofile(os.path.join(d, "runs_out.bin"))
    new.tofile(os.path.join(d, "new_out.bin"))
    ctx.close()
    print("recorded %d paths, %d rounds, %d runs, %d new pairs" % (n, int(st["rounds"]), runs.size, new.size))


if __name__ == "__main__":
    main()
