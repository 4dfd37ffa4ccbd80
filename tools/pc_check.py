"""path_compute from pass 2A to its return value on every invocation of a recorded
gmap run (tools/make_stage3_trace.py: bigdata/gmap_267_stage3.npz, 892 calls), in
both flavours of stage3.c: gmap's (the recording itself) and GSNAP's (the
reference's own path_compute built with -DGSNAP and replayed from each call's
pass-2A path, oracle/pc_replay.c).  Each query's returned list, every pair's
donor / acceptor probability, *intronlen / *nonintronlen / *defect_rate and the
pass calls must be bit-exact.

    python tools/pc_check.py prep TRACE.npz OUT.npz   (dev container: replays the reference)
    python tools/pc_check.py cpu OUT.npz [JSON]       (gsnapdp_stage3_path_compute on the CPU under ASan +
                                                       UBSan, DP served by the restatement)
    python tools/pc_check.py gpu OUT.npz [JSON]       (gsnapdp_stage3_path_compute on the GPU, timed)"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def prep(trace, out):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import gen_golden as G
    z = np.load(trace, allow_pickle=False)
    (queries, pin, q, qu), (want, wprobs, final), (gpc, gpp, gpr), differ = G.pc_replay(z)
    # keep only the pass-2A paths and query bytes the queries use
    pin = np.concatenate([pin[int(c["first_pair"]):int(c["first_pair"]) + int(c["npairs"])] for c in queries])
    queries = queries.copy()
    queries["first_pair"] = np.concatenate([[0], np.cumsum(queries["npairs"])[:-1]]).astype(np.int32)
    np.savez_compressed(out, blocks=z["blocks"], queries=queries, pin=pin, q=q, qu=qu, want=want, wprobs=wprobs,
                        final=final, gsnap_final=gpc, gsnap_want=gpp, gsnap_wprobs=gpr, s2_calls=z["s2_calls"],
                        s2_pairs=z["s2_pairs"])
    print("%s: %d path_compute calls (gmap's build of the replay reproduces all); GSNAP's build: %d differ from "
          "gmap's, %d with a stage-2 request the recording lacks" % (out, len(final), differ,
                                                                     int((gpc["pad"] != 0).sum())))


def flavours(z):
    yield "gmap", 0, z["want"], z["wprobs"], z["final"]
    yield "gsnap", 1, z["gsnap_want"], z["gsnap_wprobs"], z["gsnap_final"]


def cpu(path, js):
    from gsnapdp.records import S3_CALL, S3_COMPUTE_STATS, S3_PAIR
    from test_stage3_cpu import check_path_compute
    z = np.load(path, allow_pickle=False)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "stage3_cpu"])
    rep = {}
    for name, gs, want, wprobs, final in flavours(z):
        ok = final["pad"] == 0
        with tempfile.TemporaryDirectory() as d:
            z["queries"].tofile(os.path.join(d, "calls.bin"))
            z["pin"].tofile(os.path.join(d, "pairs_in.bin"))
            z["q"].tofile(os.path.join(d, "query.bin"))
            z["qu"].tofile(os.path.join(d, "query_uc.bin"))
            z["blocks"].astype("<u4").tofile(os.path.join(d, "genome.u32"))
            z["s2_calls"].tofile(os.path.join(d, "stage2_calls.bin"))
            z["s2_pairs"].tofile(os.path.join(d, "stage2_pairs.bin"))
            env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
                       UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
                       GSNAPDP_MAXENT_TABLES=os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin"))
            t0 = time.perf_counter()
            p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "stage3_cpu"), d, "--path-compute", "9",
                                str(int(final["maxintronlen_bound"][0])), str(gs)], env=env, capture_output=True,
                               text=True, timeout=3000)
            dt = time.perf_counter() - t0
            assert p.returncode == 0, p.stderr[-4000:]
            assert "runtime error" not in p.stderr, p.stderr[-4000:]
            got_calls = np.fromfile(os.path.join(d, "pass_calls.bin"), dtype=S3_CALL)
            got = np.fromfile(os.path.join(d, "pass_pairs.bin"), dtype=S3_PAIR)
            probs = np.fromfile(os.path.join(d, "pass_probs.bin"), dtype=np.float64).reshape(-1, 2)
            cs = np.fromfile(os.path.join(d, "compute_stats.bin"), dtype=S3_COMPUTE_STATS)[0]
        n = check_all(got_calls, got, probs, want, wprobs, final, ok, name, check_path_compute)
        assert list(cs["pass_calls"]) == list(final["passes"].sum(axis=0)), name
        rep[name] = {"queries": int(len(final)), "bit_exact": n, "checked": int(ok.sum()), "asan_ubsan": True,
                     "seconds": round(dt, 3), "pass_calls": [int(x) for x in cs["pass_calls"]]}
        print(name, rep[name], flush=True)
    if js:
        json.dump({"what": "path_compute 2A-return, every invocation of the 267-cDNA gmap run, CPU under ASan+UBSan "
                           "(DP served by the restatement)", **rep}, open(js, "w"), indent=1)


def check_all(got_calls, got, probs, want, wprobs, final, ok, name, check):
    """check_path_compute over the invocations whose outputs the reference fixed (ok)"""
    if ok.all():
        check(got_calls, got, probs, want, wprobs, final, name)
        return int(len(final))
    keep = np.nonzero(ok)[0]
    gl, gp, wl, wp = [], [], [], []
    for i in keep:
        a, n = int(got_calls["first_out"][i]), int(got_calls["nout"][i])
        b, m = int(final["first_out"][i]), int(final["nout"][i])
        gl.append(got[a:a + n]), gp.append(probs[a:a + n]), wl.append(want[b:b + m]), wp.append(wprobs[b:b + m])
    gc, fc = got_calls[keep].copy(), final[keep].copy()
    gc["first_out"] = np.concatenate([[0], np.cumsum(gc["nout"])[:-1]])
    fc["first_out"] = np.concatenate([[0], np.cumsum(fc["nout"])[:-1]])
    check(gc, np.concatenate(gl), np.concatenate(gp), np.concatenate(wl), np.concatenate(wp), fc, name)
    return int(keep.size)


def gpu(path, js):
    from gsnapdp import Context
    from test_stage3_cpu import check_path_compute
    from test_gpu_stage3 import stage2_double
    z = np.load(path, allow_pickle=False)
    ctx = Context(z["blocks"])
    rep = {}
    with tempfile.TemporaryDirectory() as tmp:
        s2 = stage2_double(ctx, z, tmp)  # noqa: F841 (kept alive while the context uses it)
        for name, gs, want, wprobs, final in flavours(z):
            ok = final["pad"] == 0
            maxintron = int(final["maxintronlen_bound"][0])
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                got_calls, got, probs, st = ctx.stage3_path_compute(z["queries"], z["pin"], z["q"], z["qu"],
                                                                    maxintronlen_bound=maxintron, gsnap=bool(gs))
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            n = check_all(got_calls, got, probs, want, wprobs, final, ok, name, check_path_compute)
            assert list(st["pass_calls"]) == list(final["passes"].sum(axis=0)), name
            rep[name] = {"queries": int(len(final)), "bit_exact": n, "checked": int(ok.sum()),
                         "seconds_best_of_3": round(best, 4), "queries_per_s": round(len(final) / best, 1),
                         "rounds": int(st["rounds"]), "passes": int(st["passes"]), "sites": int(st["sites"]),
                         "host_s": round(float(st["seconds"][0]), 4), "gpu_s": round(float(st["seconds"][1]), 4),
                         "pass_calls": [int(x) for x in st["pass_calls"]]}
            print(name, rep[name], flush=True)
    ctx.close()
    if js:
        json.dump({"what": "path_compute 2A-return on MI355X, every invocation of the 267-cDNA gmap run", **rep},
                  open(js, "w"), indent=1)


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "prep":
        prep(sys.argv[2], sys.argv[3])
    elif mode == "cpu":
        cpu(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        gpu(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
