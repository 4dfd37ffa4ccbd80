"""Records one stage-3 pass on the GPU for host profiling on a machine without
one: the 7,424-path pass of bench.measure_stage3 with GSNAPDP_S3_RECORD set
(every round's layout and GPU outputs, gsnapdp_stage3_exec.cpp) into DIR.
`python tools/s3_record.py DIR PATHS --inputs` (no GPU) then writes the same
pass's inputs and the reference's lists beside them, and
oracle/_build/stage3_host_replay DIR replays it.

    python tools/s3_record.py DIR [PATHS] [--inputs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))


def main():
    d = sys.argv[1]
    paths = int(sys.argv[2]) if len(sys.argv) > 2 else 7424
    os.makedirs(d, exist_ok=True)
    import numpy as np
    from gsnapdp import workload as W
    z = np.load(os.path.join(ROOT, "tests", "golden", "gmap_synth_stage3.npz"), allow_pickle=False)
    calls, pin, q, qu, want = W.stage3_calls(z, max(1, paths // len(z["calls"])))
    if "--inputs" in sys.argv:
        calls.tofile(os.path.join(d, "calls.bin"))
        pin.tofile(os.path.join(d, "pairs_in.bin"))
        q.tofile(os.path.join(d, "query.bin"))
        qu.tofile(os.path.join(d, "query_uc.bin"))
        want.tofile(os.path.join(d, "pairs_out.bin"))
        z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
        return
    os.environ["GSNAPDP_S3_RECORD"] = d  # read once, when the first pass runs
    from gsnapdp import Context
    ctx = Context(z["blocks"])
    sys.path.insert(0, ROOT)
    import bench
    bench.stage2_double(ctx, z)  # build_dual_breaks' stage 2, from the recording
    c, got, st = ctx.stage3_pass(calls, pin, q, qu)
    assert got.tobytes() == want.tobytes()
    print("recorded %d paths, %d rounds into %s" % (len(calls), st["rounds"], d))
    ctx.close()


if __name__ == "__main__":
    main()
