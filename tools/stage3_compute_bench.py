"""Every stage-3 pass of a recorded gmap run on the GPU, beside the same-box CPU
restatement: (1) all its pass calls (build_pairs_introns / _singles / _end5 /
_end3 / _dualintrons / build_dual_breaks) in one gsnapdp_stage3_pass, and (2)
passes 2A-6 of every path_compute call in one gsnapdp_stage3_compute; both
checked cell for cell against the reference's lists.  traverse_dual_break's
stage 2 is served from the recording (tests/dropin/stage2_double.c).  The CPU
leg is the same host code with every DP window served by the oracle/
restatement on the pass's 16 threads (oracle/_build/libstage3_cpu.so).

    python tools/stage3_compute_bench.py TRACE.npz [COPIES] [--no-cpu]"""
import ctypes
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
from gsnapdp import Context  # noqa: E402
from gsnapdp import workload as W  # noqa: E402


def stage2_lib(tmp):
    so = os.path.join(tmp, "libstage2_double.so")
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                           os.path.join(ROOT, "tests", "dropin", "stage2_double.c")])
    d = ctypes.CDLL(so)
    d.s2dbl_new.restype = ctypes.c_void_p
    d.s2dbl_new.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    return d


def best_of(n, fn):
    best = None
    for _ in range(n):
        t0 = time.perf_counter()
        r = fn()
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, r)
    return best


def main():
    from test_stage3_cpu import check_compute
    z = np.load(sys.argv[1], allow_pickle=False)
    copies = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 1
    cpu = "--no-cpu" not in sys.argv
    calls, pin, q, qu, want = W.stage3_calls(z, copies)
    Q, PI, QQ, QU, WANT, FINAL, counts = W.stage3_pipeline(z, copies)
    out = {"trace": os.path.basename(sys.argv[1]), "copies": copies}
    with tempfile.TemporaryDirectory() as tmp:
        d = stage2_lib(tmp)
        sc, sp = np.ascontiguousarray(z["s2_calls"]), np.ascontiguousarray(z["s2_pairs"])
        h = d.s2dbl_new(sc.ctypes.data, sc.size, sp.ctypes.data, sp.size)
        ctx = Context(z["blocks"])
        ctx.set_stage2(ctypes.cast(d.s2dbl_compute_one, ctypes.c_void_p).value, h)
        ctx.stage3_pass(calls[:64], pin, q, qu)  # warm-up
        buf = np.empty(ctx.stage3_capacity(calls), dtype=want.dtype)
        dt, (c, got, st) = best_of(4, lambda: ctx.stage3_pass(calls, pin, q, qu, out=buf))
        ok = bool((c["status"] == 0).all()) and got.tobytes() == want.tobytes()
        out["all_passes"] = {"paths": int(len(calls)), "by_pass": np.bincount(calls["pass"], minlength=6).tolist(),
                             "bit_exact_vs_reference": ok, "seconds": round(dt, 4), "rounds": int(st["rounds"]),
                             "windows": [int(x) for x in st["windows"]], "paths_per_s": round(len(calls) / dt, 1),
                             "host_s": round(float(st["seconds"][0]), 4),
                             "reference_1thread_s_cross_machine": round(float(calls["ref_seconds"].sum()), 4)}
        dt, (c, got, st) = best_of(3, lambda: ctx.stage3_compute(Q, PI, QQ, QU))
        check_compute(c, got, FINAL, WANT, "compute")
        out["passes_2A_6"] = {"queries": int(len(Q)), "bit_exact_vs_reference": True, "seconds": round(dt, 4),
                              "queries_per_s": round(len(Q) / dt, 1), "passes": int(st["passes"]),
                              "rounds": int(st["rounds"]), "pass_calls": [int(x) for x in st["pass_calls"]],
                              "host_steps_s": round(float(st["seconds"][0]), 4),
                              "passes_s": round(float(st["seconds"][1]), 4)}
        ctx.close()
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg
        S = O.Stage3Cpu(z["blocks"])
        S.set_stage2_recording(z["s2_calls"], z["s2_pairs"])
        threads = int(os.environ.get("GSNAPDP_S3_THREADS", min(16, os.cpu_count() or 1)))
        dt, (c, got, st) = best_of(2, lambda: S.run(calls, pin, q, qu))
        out["all_passes"]["cpu_restatement"] = {"seconds": round(dt, 4), "paths_per_s": round(len(calls) / dt, 1),
                                                "cores": threads, "lists_equal": got.tobytes() == want.tobytes()}
        dt, (c, got, st) = best_of(2, lambda: S.compute(Q, PI, QQ, QU))
        check_compute(c, got, FINAL, WANT, "cpu compute")
        out["passes_2A_6"]["cpu_restatement"] = {"seconds": round(dt, 4), "queries_per_s": round(len(Q) / dt, 1),
                                                 "cores": threads}
        S.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
