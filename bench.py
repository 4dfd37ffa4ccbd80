#!/usr/bin/env python3
"""Benchmark: GMAP/GSNAP stage-3 single-gap DP on MI355X (BASELINE config 3).

One step = one pass of the hot path over ONE read batch: 1,000,000 synthetic
150 bp reads (2 % substitutions, 30 % with a 1-3 bp indel, band 31) against a
GRCh38-sized synthetic genome (24 chromosomes with the GRCh38 lengths, 3.09
Gnt, 1.16 GB packed, resident in HBM), each read one Dynprog_single_gap window
(fill + endpoint + traceback through gsnapdp_run_device), plus the op-stream
compaction, and -- for N GPUs -- the RCCL gather of every rank's result
records and compact op streams to rank 0.  The batch is FIXED: N GPUs split it
per read into slices balanced by in-band cells (strong scaling, SURVEY.md
8(e)).  Side lines at N=1: C2 (100k reads, 64 Mbp genome), C4, C5 (DP part),
splice-junction ends, microexons, the PCIe-inclusive host-buffer rate.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       --gpus N > 1 without a launcher re-runs itself under
       torch.distributed.run (one process per GPU) before touching the GPU.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))

import torch  # noqa: E402

from gsnapdp import Context, gather, op_offsets, shard  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import RESULT  # noqa: E402

HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# int32 VALU: measured 4 cycles per wave64 instruction on gfx950 (v_max_i32,
# v_add_u32, v_alignbit_b32; tools/ubench/valu_rate.hip), i.e. 16 lanes/clk per
# SIMD (fp32 FMA issues at 2 cycles): 256 CU x 4 SIMD x 16 lanes x 2.4 GHz
VALU_INT32_PEAK = 256 * 4 * 16 * 2.4e9
OPS_PER_CELL = 14             # gap1 4 + gap2 4 + nogap 6 int32 ops
XGMI_LINK_GBS = 153.0         # one xGMI link per peer (7 links x ~153 GB/s per GPU, nominal)
C3_READS = 1_000_000          # BASELINE config 3: one fixed batch, split across the GPUs
C2_READS = 100_000            # side line: BASELINE config 2
GENOME_NT = 64_000_000        # side-line genome (C2, C4, C5, ...)
MIN_STEADY_S = 1.0            # steady-state figure: at least this many seconds of steps
DOMINANT = "k_fill"           # every C2 window is a register-band (k_fill) window
C4_WINDOWS = 200_000          # intron windows per config-4 step
C4_TRANSCRIPTS = 50_000       # config 4 as stated: transcripts through the final intron pass
C5_READS = 100_000            # reads per config-5 step (3 DP windows each)


def window_bytes(w: np.ndarray, nops: np.ndarray, uc_aliased: bool = False) -> np.ndarray:
    """Algorithmic HBM bytes of one window (DESIGN.md "Roofline"): query and
    uppercase query (L1 each; L1 once when the caller passes one buffer for
    both, as this bench does), the packed genome blocks its columns touch
    (12 B per 32 nt), the 68 B descriptor, the 48 B result and 4 B per op."""
    span_blocks = (w["length2"].astype(np.int64) + 31) // 32 + 1
    qb = (1 if uc_aliased else 2) * w["length1"].astype(np.int64)
    return qb + 12 * span_blocks + 68 + 48 + 4 * nops.astype(np.int64)


def profile_order(path: str):
    """Sort key of a committed profile file: its round and version (r2v10 after
    r2v9, r3v1 after both; r1_v1 / r2c3a style tags too), then the name."""
    import re
    m = re.match(r"r(\d+)_?[a-z]*?v?(\d*)", os.path.basename(path))
    if not m:
        return (-1, -1, os.path.basename(path))
    return (int(m.group(1)), int(m.group(2) or 0), os.path.basename(path))


def band_cells(w: np.ndarray) -> int:
    """Exact in-band cell count of the widened band (dynprog.c:1442-1516)."""
    L1 = w["length1"].astype(np.int64)
    L2 = w["length2"].astype(np.int64)
    eb = w["extraband"].astype(np.int64)
    rband = np.where(L2 >= L1, L2 - L1 + eb, eb)
    lband = np.where(L2 >= L1, eb, L1 - L2 + eb)
    total = 0
    for c in range(1, int(L2.max()) + 1):
        lo = np.maximum(1, c - rband)
        hi = np.minimum(L1, c + lband)
        total += int(np.where(c <= L2, np.clip(hi - lo + 1, 0, None), 0).sum())
    return total


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` on `workload` from the committed
    rocprofv3 PMC passes (profiles/*_traffic.json, written by
    tools/pmc_traffic.py), or None.  The newest round/version wins (profile_order)."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), key=profile_order):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("kernel") == kernel and d.get("workload", "C2") == workload:
            best = (d["traffic_bytes"], os.path.basename(f), d.get("dispatches"))
    return best


def rocprof_kernel_ms(kernel: str, workload: str):
    """Average duration (ms) of `kernel` in the committed rocprofv3
    --kernel-trace --stats summary of this bench on `workload`
    (profiles/*_<workload>_kernel_stats.csv), or None."""
    import csv
    import glob
    best = None
    pat = os.path.join(ROOT, "profiles", "*_%s_kernel_stats.csv" % workload.lower())
    for f in sorted(glob.glob(pat), key=profile_order):
        try:
            for row in csv.DictReader(open(f)):
                name = row.get("Name", "").replace("(anonymous namespace)::", "")
                if name.split("(")[0].strip().endswith(kernel):
                    best = (float(row["AverageNs"]) / 1e6, os.path.basename(f))
        except (OSError, ValueError, KeyError):
            continue
    return best


def cells_per_window(w: np.ndarray) -> np.ndarray:
    """In-band cells of every window (band_cells per distinct shape)."""
    key = np.stack([w["length1"], w["length2"], w["extraband"]], axis=1).astype(np.int64)
    shapes, inv = np.unique(key, axis=0, return_inverse=True)
    per = np.array([band_cells(w[np.flatnonzero(inv.reshape(-1) == k)[:1]]) for k in range(len(shapes))],
                   dtype=np.int64)
    return per[inv.reshape(-1)]


def cpu_info():
    """(allotted threads, host CPU count, CPU model string)."""
    threads = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, os.cpu_count(), model


def measure_c4(genome, n, steps, warmup, dev, with_cpu):
    """Side measurement, BASELINE config 4: Dynprog_genome_gap on intron windows
    (length1 22, length2 30, extraband_paired 7), score and probability modes,
    device-resident, timed like the main line; CPU restatement (1 core) beside it."""
    from gsnapdp import ggap_op_offsets
    from gsnapdp.records import GGAP_RESULT, GGAP_TRACE
    out = {"workload": "C4: Dynprog_genome_gap, %d intron windows per step, length1 22, "
                       "length2L/R 30, extraband_paired 7, finalp" % n, "unit": "windows/s"}
    for mode in ("score", "prob"):
        g, b = W.c4_windows(genome, n, seed=4, use_probabilities=(mode == "prob"))
        blocks = W.pack_genome(g)
        ctx = Context(blocks, mode=0, device=dev.index)
        off = ggap_op_offsets(b.windows)
        d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
        d_q = torch.from_numpy(b.query.copy()).to(dev)
        d_res = torch.zeros(n * GGAP_RESULT.itemsize, dtype=torch.uint8, device=dev)
        d_trc = torch.zeros(n * GGAP_TRACE.itemsize, dtype=torch.uint8, device=dev)
        d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
        d_off = torch.from_numpy(off.copy()).to(dev)

        def step():
            ctx.ggap_run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), d_res.data_ptr(),
                                d_trc.data_ptr(), d_ops.data_ptr(), d_off.data_ptr())
        for _ in range(warmup):
            step()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.sync()
        el = time.perf_counter() - t0
        names = ctx.profile(True)
        acc = np.zeros(len(names))
        for _ in range(steps):
            step()
            ctx.profile_read(acc)
        ctx.profile(False)
        rec = {"value": round(n * steps / el, 1), "ms_per_step": round(1000 * el / steps, 4),
               "kernel_ms_per_step": {nm: round(acc[i] / steps, 4) for i, nm in enumerate(names) if acc[i] > 0}}
        if with_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            O.setup(blocks)
            sample = min(n, 40_000)
            t1 = time.perf_counter()
            ores, _, _, _ = O.run_ggap_batch(b.windows[:sample], b.query, b.query)
            cpu = sample / (time.perf_counter() - t1)
            res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=GGAP_RESULT)[:sample]
            rec["cpu_baseline"] = {"value": round(cpu, 1), "unit": "windows/s", "cores": 1, "kind": "port",
                                   "sample": "%d C4 windows, oracle/ restatement, 1 thread" % sample}
            rec["parity_bit_exact"] = bool(all(np.array_equal(res[f], ores[f]) for f in
                                               ("finalscore", "nmatches", "nmismatches", "nopens", "nindels",
                                                "returned_null", "dynprogindex")))
        out[mode] = rec
        ctx.close()
    return out


def measure_c5(genome, nreads, steps, warmup, dev, with_cpu):
    """Side measurement, BASELINE config 5 reduced to its DP windows (SURVEY
    8(d)): per 100 bp read one single gap (extraband 3) and an end5 + end3 gap
    (length1 1-30, length2 +10, extraband_end 3); whole-batch windows/s."""
    b = W.c5_windows(genome, nreads, seed=5)
    n = len(b)
    ctx = Context(W.pack_genome(genome), mode=0, device=dev.index)
    off = op_offsets(b.windows)
    d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(b.query.copy()).to(dev)
    d_u = torch.from_numpy(b.query_uc.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)

    def step():
        ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(),
                       d_ops.data_ptr(), d_off.data_ptr())
    for _ in range(warmup):
        step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    el = time.perf_counter() - t0
    names = ctx.profile(True)
    acc = np.zeros(len(names))
    for _ in range(steps):
        step()
        ctx.profile_read(acc)
    ctx.profile(False)
    out = {"workload": "C5 (DP part): %d reads x (single gap 100 bp, extraband 3 + end5 + end3 gaps, "
                       "extraband_end 3, QUERYEND_GAP) = %d windows per step" % (nreads, n),
           "value": round(n * steps / el, 1), "unit": "windows/s", "reads_per_s": round(nreads * steps / el, 1),
           "ms_per_step": round(1000 * el / steps, 4),
           "kernel_ms_per_step": {nm: round(acc[i] / steps, 4) for i, nm in enumerate(names) if acc[i] > 0}}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        O.setup(W.pack_genome(genome))
        t1 = time.perf_counter()
        ores, _, _, _ = O.run_batch(b.windows, b.query, b.query_uc, nthreads=16)
        cpu = n / (time.perf_counter() - t1)
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=RESULT)
        out["cpu_baseline"] = {"value": round(cpu, 1), "unit": "windows/s", "cores": 16, "kind": "port",
                               "sample": "the whole %d-window batch once, oracle/ restatement, pthreads" % n}
        out["parity_bit_exact"] = bool(all(np.array_equal(res[f], ores[f]) for f in
                                           ("finalscore", "nmatches", "nmismatches", "nopens", "nindels")))
    ctx.close()
    return out


def timed(step, sync, steps, warmup):
    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    return time.perf_counter() - t0


def measure_sj(genome, n, steps, warmup, dev, with_cpu):
    """Side measurement: Dynprog_end5/3_splicejunction (the known-splice end
    candidates Splicetrie_solve_end5/3 issue), device-resident; CPU restatement
    (1 core) on a sample beside it."""
    b = W.sj_windows(genome, n, seed=9, mix=False)
    ctx = Context(np.zeros(64, np.uint32), mode=0, device=dev.index)
    off = op_offsets(b.windows)
    d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(b.query.copy()).to(dev)
    d_u = torch.from_numpy(b.query_uc.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    el = timed(lambda: ctx.sj_run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(),
                                         d_ops.data_ptr(), d_off.data_ptr()), ctx.sync, steps, warmup)
    out = {"workload": "Dynprog_end5/3_splicejunction: %d junction end gaps per step (length1 1-160, "
                       "length2 = length1 + 10..40, extraband_end 3)" % n,
           "value": round(n * steps / el, 1), "unit": "windows/s", "ms_per_step": round(1000 * el / steps, 4)}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        O.setup(np.zeros(16, np.uint32))
        sample = min(n, 20_000)
        t1 = time.perf_counter()
        ores, _, _, _ = O.run_sj_batch(b.windows[:sample], b.query, b.query_uc)
        cpu = sample / (time.perf_counter() - t1)
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=RESULT)[:sample]
        out["cpu_baseline"] = {"value": round(cpu, 1), "unit": "windows/s", "cores": 1, "kind": "port",
                               "sample": "%d windows, oracle/ restatement, 1 thread" % sample}
        out["parity_bit_exact"] = bool(all(np.array_equal(res[f], ores[f]) for f in
                                           ("finalscore", "nmatches", "nmismatches", "nopens", "nindels")))
    ctx.close()
    return out


def measure_micro(genome, n, steps, warmup, dev, with_cpu):
    """Side measurement: Dynprog_microexon_int (intron gaps of 40-800 nt with a
    planted 3-12 nt microexon), device-resident; CPU restatement (1 core) on a
    sample beside it."""
    from gsnapdp.records import MICRO_RESULT
    g, b = W.micro_windows(genome[:8_000_000], n, seed=10, mix=False)
    blocks = W.pack_genome(g)
    ctx = Context(blocks, mode=0, device=dev.index)
    d_w = torch.from_numpy(b.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(b.query.copy()).to(dev)
    d_u = torch.from_numpy(b.query_uc.copy()).to(dev)
    d_res = torch.zeros(n * MICRO_RESULT.itemsize, dtype=torch.uint8, device=dev)
    el = timed(lambda: ctx.micro_run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr()),
               ctx.sync, steps, warmup)
    out = {"workload": "Dynprog_microexon_int: %d intron gaps per step (span 40-800 nt, planted microexon)" % n,
           "value": round(n * steps / el, 1), "unit": "windows/s", "ms_per_step": round(1000 * el / steps, 4)}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        O.setup(blocks)
        sample = min(n, 5_000)
        t1 = time.perf_counter()
        ores, _, _, _ = O.run_micro_batch(b.windows[:sample], b.query, b.query_uc)
        cpu = sample / (time.perf_counter() - t1)
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=MICRO_RESULT)[:sample]
        out["cpu_baseline"] = {"value": round(cpu, 1), "unit": "windows/s", "cores": 1, "kind": "port",
                               "sample": "%d windows, oracle/ restatement, 1 thread" % sample}
        out["parity_bit_exact"] = bool(all(np.array_equal(res[f], ores[f]) for f in
                                           ("found", "microintrontype", "dynprogindex", "bestcL", "bestcR")) and
                                       np.array_equal(res["bestprob2"].view(np.uint64),
                                                      ores["bestprob2"].view(np.uint64)))
    ctx.close()
    return out


_S2 = []  # the stage-2 doubles the contexts use (kept alive)


def stage2_double(ctx, z):
    """traverse_dual_break's stage 2 served from the golden's recording
    (tests/dropin/stage2_double.c, built here with gcc) as ctx's stage-2 callback"""
    import ctypes
    import subprocess
    import tempfile
    tmp = tempfile.mkdtemp(prefix="gsnapdp_s2_")
    so = os.path.join(tmp, "libstage2_double.so")
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                           os.path.join(ROOT, "tests", "dropin", "stage2_double.c")])
    d = ctypes.CDLL(so)
    d.s2dbl_new.restype = ctypes.c_void_p
    d.s2dbl_new.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    sc, sp = np.ascontiguousarray(z["s2_calls"]), np.ascontiguousarray(z["s2_pairs"])
    h = d.s2dbl_new(sc.ctypes.data, sc.size, sp.ctypes.data, sp.size)
    _S2.append((d, sc, sp))
    ctx.set_stage2(ctypes.cast(d.s2dbl_compute_one, ctypes.c_void_p).value, h)


def measure_stage3(paths=7424, reps=6):
    """Side line: the stage-3 passes (gsnapdp_stage3_pass: path_compute's
    build_pairs_introns, build_pairs_singles, build_pairs_end5 / build_path_end3
    and build_pairs_dualintrons, mixed in one pass) on the recorded calls of the
    reference's gmap (tests/golden/gmap_synth_stage3.npz: 464 introns, 336
    singles, 160 end5, 152 end3 and 96 dual-intron calls) replicated `copies`
    times into one pass;
    every copy is checked against the reference's lists.  `reference_s` is the
    reference's own time for the same calls (its build_pairs_introns wall time,
    DP included, one thread; recorded by oracle/gmap_trace in the dev container,
    not on this host)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "gmap_synth_stage3.npz"), allow_pickle=False)
    copies = max(1, paths // len(z["calls"]))
    calls, pin, q, qu, want = W.stage3_calls(z, copies)
    ctx = Context(z["blocks"])
    stage2_double(ctx, z)  # build_dual_breaks' stage-2 dual breaks, from the recording
    from gsnapdp import expand_compact
    ctx.stage3_pass(calls[:64], pin, q, qu)  # warm-up
    # the full-pair output (every returned cell as a whole pair record) ...
    buf = np.empty(ctx.stage3_capacity(calls), dtype=want.dtype)
    full_s = None
    for _ in range(reps + 1):  # the first run also faults the output buffer in
        t0 = time.perf_counter()
        c, got, st = ctx.stage3_pass(calls, pin, q, qu, out=buf)
        dt = time.perf_counter() - t0
        full_s = dt if full_s is None else min(full_s, dt)
    ok_full = bool((c["status"] == 0).all()) and got.tobytes() == want.tobytes()
    # ... and the timed form, the compact output a caller that owns the input
    # cells takes (gsnapdp_stage3_pass_compact: each returned cell as the index
    # of its input pair, new pairs apart; what the drop-in relinks)
    bufs = None
    best = None
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        c, cells, new, st = ctx.stage3_pass_compact(calls, pin, q, qu, bufs=bufs)
        dt = time.perf_counter() - t0
        if bufs is None:
            bufs = (cells.base, new.base)
        if best is None or dt < best[0]:
            best = (dt, c, cells.copy(), new.copy(), st)
    dt, c, cells, new, st = best
    got = expand_compact(c, pin, cells, new)
    ok = ok_full and bool((c["status"] == 0).all()) and got.tobytes() == want.tobytes()
    for f in ("out_minor", "out_major", "out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen",
              "shiftp", "incompletep", "nout"):
        ok = ok and bool(np.array_equal(c[f], calls[f]))
    nwin = int(np.sum(st["windows"]))
    ref = float(z["calls"]["ref_seconds"].sum()) * copies
    ctx.close()
    cpu, (_, rcells, rnew, _) = stage3_cpu_baseline(z["blocks"], calls, pin, q, qu, z=z, compact=True)
    cpu["cells_equal_gpu"] = bool(np.array_equal(rcells, cells) and rnew.tobytes() == new.tobytes())
    return {"metric": "stage-3 passes (path_compute's DP passes), paths/s",
            "output": "compact (gsnapdp_stage3_pass_compact); full-pair output %.4f s" % full_s,
            "value": round(len(calls) / dt, 1), "unit": "paths/s", "paths": int(len(calls)),
            "paths_by_pass": {n: int((calls["pass"] == i).sum())
                              for i, n in enumerate(("introns", "singles", "end5", "end3", "dualintrons"))},
            "seconds": round(dt, 4), "rounds": int(st["rounds"]),
            "windows": nwin, "windows_per_s": round(nwin / dt, 1),
            "windows_by_family": {"single": int(st["windows"][0]), "genome_gap": int(st["windows"][1]),
                                  "cdna_gap": int(st["windows"][2]), "microexon": int(st["windows"][3])},
            "host_s": round(float(st["seconds"][0]), 4), "batches_s": round(float(st["seconds"][1]), 4),
            "bit_exact_vs_reference": ok,
            "cpu_baseline": cpu,
            "reference_cross_machine": {
                "value": round(len(calls) / ref, 1), "unit": "paths/s", "seconds": round(ref, 4), "cores": 1,
                "kind": "reference",
                "note": "the reference's own pass functions on the same calls, timed by gmap_trace in the "
                        "development container (a different machine), DP included"}}


def stage3_cpu_baseline(blocks, calls, pin, q, qu, want=None, compact=False, z=None):
    """The same pass on this host's CPU: the pass's host code with every DP
    window served by the oracle/ restatement on the pass's 16 threads
    (oracle/_build/libstage3_cpu.so) -- best of two runs after a warm-up on a
    slice.  Its lists are compared with the GPU pass's (`want`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # CPU baseline leg
    S = O.Stage3Cpu(blocks)
    if z is not None and "s2_calls" in z:
        S.set_stage2_recording(z["s2_calls"], z["s2_pairs"])
    S.run_compact(calls[:min(len(calls), 256)], pin, q, qu)
    best = None
    for _ in range(2):
        t0 = time.perf_counter()
        res = S.run_compact(calls, pin, q, qu) if compact else S.run(calls, pin, q, qu)
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, res)
    S.close()
    dt, res = best
    out = {"value": round(len(calls) / dt, 1), "unit": "paths/s", "seconds": round(dt, 4),
           "cores": int(os.environ.get("GSNAPDP_S3_THREADS", min(16, os.cpu_count() or 1))), "kind": "port",
           "sample": "the same %d paths, oracle/ restatement of every DP window under the pass's host code "
                     "(oracle/_build/libstage3_cpu.so)" % len(calls)}
    if want is not None and not compact:
        out["lists_equal_gpu"] = bool(res[1].tobytes() == want.tobytes())
    return out if not compact else (out, res)


def measure_stage3_compute(copies=64, reps=5, cpu=True, small=8):
    """Side line: path_compute from pass 2A to its return value
    (gsnapdp_stage3_path_compute: passes 2A-10, the host steps restated, every
    round of DP passes one gsnapdp_stage3_pass across the queries, each
    assign_gap_types' MaxEnt sites one k_maxent batch) for every path_compute
    call the reference's gmap made on the synthetic cDNAs
    (tests/golden/gmap_synth_stage3.npz, 168 calls) x `copies` in one batch,
    each copy checked against the list path_compute returned in gmap (pairs and
    their donor / acceptor probabilities); `by_batch` gives the same at `small`
    copies.  traverse_dual_break's stage 2 is served from the recording
    (tests/dropin/stage2_double.c, built here).  The CPU leg runs the same host
    code with every DP window and MaxEnt site served by the oracle/ restatement,
    16 threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_stage3_cpu import check_path_compute  # list-by-list comparison with the recording
    z = np.load(os.path.join(ROOT, "tests", "golden", "gmap_synth_stage3.npz"), allow_pickle=False)
    ctx = Context(z["blocks"])
    stage2_double(ctx, z)

    def gpu(k):
        Q, PI, QQ, QU, WANT, WP, FINAL = W.stage3_path_pipeline(z, k)
        maxintron = int(FINAL["maxintronlen_bound"][0])
        ctx.stage3_path_compute(Q[:8], PI, QQ, QU, maxintronlen_bound=maxintron)  # warm-up
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            res = ctx.stage3_path_compute(Q, PI, QQ, QU, maxintronlen_bound=maxintron)
            dt = time.perf_counter() - t0
            if best is None or dt < best[0]:
                best = (dt, res)
        dt, (c, got, probs, st) = best
        check_path_compute(c, got, probs, WANT, WP, FINAL, "stage3 path_compute x%d" % k)
        r = {"queries": int(len(Q)), "value": round(len(Q) / dt, 1), "seconds": round(dt, 4),
             "bit_exact_vs_reference": True, "passes": int(st["passes"]), "rounds": int(st["rounds"]),
             "maxent_sites": int(st["sites"]), "pass_calls": [int(x) for x in st["pass_calls"]],
             "windows": [int(x) for x in st["windows"]], "host_steps_s": round(float(st["seconds"][0]), 4),
             "gpu_wait_s": round(float(st["seconds"][1]), 4),
             "host_frac": round(float(st["seconds"][0]) / dt, 3)}
        return r, (Q, PI, QQ, QU, WANT, WP, FINAL, maxintron)

    out = {"metric": "stage-3 path_compute (passes 2A-10), queries/s", "unit": "queries/s"}
    r, data = gpu(copies)
    out.update(r)
    out["by_batch"] = {str(small): gpu(small)[0]}
    ctx.close()
    if cpu:
        Q, PI, QQ, QU, WANT, WP, FINAL, maxintron = data
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg
        S = O.Stage3Cpu(z["blocks"])
        S.set_stage2_recording(z["s2_calls"], z["s2_pairs"])
        S.path_compute(Q[:8], PI, QQ, QU, maxintronlen_bound=maxintron)
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            res = S.path_compute(Q, PI, QQ, QU, maxintronlen_bound=maxintron)
            dt = time.perf_counter() - t0
            if best is None or dt < best[0]:
                best = (dt, res)
        dt, (c, got, probs, st) = best
        check_path_compute(c, got, probs, WANT, WP, FINAL, "stage3 path_compute, CPU")
        S.close()
        out["cpu_baseline"] = {"value": round(len(Q) / dt, 1), "unit": "queries/s", "seconds": round(dt, 4),
                               "cores": int(os.environ.get("GSNAPDP_S3_THREADS", min(16, os.cpu_count() or 1))),
                               "kind": "port",
                               "sample": "the same %d queries, the host steps and passes with every DP window and "
                                         "MaxEnt site served by the oracle/ restatement "
                                         "(oracle/_build/libstage3_cpu.so)" % len(Q)}
    return out


def measure_c4_transcripts(n=C4_TRANSCRIPTS, cpu=True, pinned=2000):
    """Side line, BASELINE config 4 as stated: `n` synthetic 5 kbp transcripts
    (workload.c4_transcripts: 8-12 exons, GT-AG introns of 80-5000 nt, 1 % subs,
    30 % of the boundaries stage 2 misplaces by 1-6 nt) through GMAP's final
    intron pass (gsnapdp_stage3_pass_runs: build_pairs_introns with finalp,
    stage3.c:8860-8875, each path's gap pairs named by the caller as
    insert_gapholders placed them, the lists returned as runs) and score_introns
    on every returned list (gsnapdp_stage3_score_introns_runs: one k_introns
    launch, :9890-9941).  The timed region is the pass plus score_introns over
    all paths, inputs in host memory (the pass is host-driven).  Parity: the
    lists expanded from the runs -- the first `pinned` against the reference's
    own results (tests/golden/c4_pinned.npz), all against the CPU restatement
    run in the same process, which times the same two calls."""
    import hashlib
    from gsnapdp import expand_runs, gap_lists
    t0 = time.perf_counter()
    w = W.c4_transcripts(n)
    gen_s = time.perf_counter() - t0
    gaps, gap_off = gap_lists(w.calls, w.pairs_in)  # the caller's own bookkeeping (insert_gapholders)
    ctx = Context(w.blocks)
    ctx.stage3_pass_compact(w.calls[:256], w.pairs_in, w.query, w.query_uc)  # launches, staging
    bufs = None
    best = None
    for _ in range(3):  # the first run also faults the output buffers in
        t0 = time.perf_counter()
        c, runs, new, st, bufs = ctx.stage3_pass_runs(w.calls, w.pairs_in, w.query, w.query_uc, gaps, gap_off,
                                                      bufs=bufs)
        t1 = time.perf_counter()
        sc = ctx.stage3_score_introns_runs(c, w.pairs_in, runs, new, gaps, gap_off)
        t2 = time.perf_counter()
        if best is None or t2 - t0 < best[0]:
            best = (t2 - t0, t1 - t0, t2 - t1, c, runs.copy(), new.copy(), st, sc)
    total, dt, si_s, c, runs, new, st, sc = best
    c_full, lists = expand_runs(c, w.pairs_in, runs, new)
    introns = int(sc["nintrons"].sum())
    ctx.close()
    z = np.load(os.path.join(ROOT, "tests", "golden", "c4_pinned.npz"), allow_pickle=False)
    m = min(pinned, n, int(z["n"]))
    fo, no = c_full["first_out"], c_full["nout"]
    ok_ref = all(hashlib.sha256(lists[int(fo[i]):int(fo[i]) + int(no[i])].tobytes()).digest() ==
                 z["digests"][i].tobytes() for i in range(m))
    for f in ("out_minor", "out_major", "out_nintrons", "out_nnonintrons", "shiftp", "incompletep"):
        ok_ref = ok_ref and bool(np.array_equal(c[f][:m], z["ref_" + f][:m]))
    ok_ref = ok_ref and bool(np.array_equal(no[:m], z["ref_nout"][:m]))
    ok_ref = ok_ref and bool(np.array_equal(sc["avg_donor_score"][:m].view(np.uint64),
                                            z["si_calls"]["avg_donor_score"][:m].astype(np.float64).view(np.uint64)))
    nwin = int(np.sum(st["windows"]))
    out = {"workload": "C4 as stated: %d synthetic transcripts of 4.5-5.5 kbp (8-12 exons, GT-AG introns of "
                       "80-5000 nt, 1%% substitutions), each GMAP's final intron pass (build_pairs_introns, "
                       "finalp) + score_introns; %d path pairs, %d gap pairs, %d introns; generated in %.1f s"
                       % (n, w.pairs_in.size, gaps.size, w.nintrons, gen_s),
           "metric": "C4 transcripts (final intron pass + score_introns), paths/s",
           "value": round(n / total, 1), "unit": "paths/s", "seconds": round(total, 4),
           "pass_s": round(dt, 4), "score_introns_s": round(si_s, 4),
           "output": "runs (gsnapdp_stage3_pass_runs: %d runs for %d returned pairs)" % (runs.size, lists.size),
           "windows": nwin, "windows_per_s": round(nwin / dt, 1),
           "windows_by_family": {"single": int(st["windows"][0]), "genome_gap": int(st["windows"][1]),
                                 "cdna_gap": int(st["windows"][2]), "microexon": int(st["windows"][3])},
           "introns_scored": introns, "introns_per_s": round(introns / si_s, 1),
           "rounds": int(st["rounds"]), "host_s": round(float(st["seconds"][0]), 4),
           "wait_s": round(float(st["seconds"][1]), 4),
           "host_frac": round((float(st["seconds"][0]) + si_s) / total, 3),
           "bit_exact_vs_reference": {"paths": m, "ok": bool(ok_ref)}}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg
        S = O.Stage3Cpu(w.blocks)
        S.run_compact(w.calls[:256], w.pairs_in, w.query, w.query_uc)
        cb = None
        for _ in range(2):
            t0 = time.perf_counter()
            rc, rruns, rnew, rst, rsc = S.run_runs(w.calls, w.pairs_in, w.query, w.query_uc, gaps, gap_off,
                                                   introns=True)
            dt_c = time.perf_counter() - t0
            if cb is None or dt_c < cb[0]:
                cb = (dt_c, rc, rruns, rnew, rsc)
        S.close()
        dt_c, rc, rruns, rnew, rsc = cb
        same = bool(np.array_equal(rruns, runs) and rnew.tobytes() == new.tobytes() and
                    rsc.tobytes() == sc.tobytes())
        for f in ("out_minor", "out_major", "out_nintrons", "out_nnonintrons", "out_intronlen", "out_nonintronlen",
                  "shiftp", "incompletep", "nout"):
            same = same and bool(np.array_equal(rc[f], c[f]))
        out["cpu_baseline"] = {
            "value": round(n / dt_c, 1), "unit": "paths/s", "seconds": round(dt_c, 4),
            "cores": int(os.environ.get("GSNAPDP_S3_THREADS", min(16, os.cpu_count() or 1))), "kind": "port",
            "sample": "the same %d paths: the pass's host code with every DP window served by the oracle/ "
                      "restatement, then score_introns on the same runs (oracle/_build/libstage3_cpu.so)" % n}
        out["bit_exact_vs_cpu_restatement"] = {"paths": n, "ok": same}
    return out


def measure_c2(genome, n, steps, warmup, dev):
    """Side line, BASELINE config 2 (round-1 headline): 100k reads on the 64 Mbp
    genome, one GPU, device-resident; per-kernel event times."""
    batch = W.c2_windows(genome, n=n, seed=2)
    ctx = Context(W.pack_genome(genome), mode=0, device=dev.index)
    off = op_offsets(batch.windows)
    d_w = torch.from_numpy(batch.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(batch.query.copy()).to(dev)
    d_u = torch.from_numpy(batch.query_uc.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)

    def step():
        ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(),
                       d_ops.data_ptr(), d_off.data_ptr())
    el = timed(step, ctx.sync, steps, warmup)
    names = ctx.profile(True)
    acc = np.zeros(len(names))
    for _ in range(steps):
        step()
        ctx.profile_read(acc)
    ctx.profile(False)
    ctx.close()
    return {"workload": "C2: Dynprog_single_gap, %d x 150 bp reads, 64 Mbp genome, extraband 15" % n,
            "value": round(n * steps / el, 1), "unit": "reads/s", "ms_per_step": round(1000 * el / steps, 4),
            "kernel_ms_per_step": {nm: round(acc[i] / steps, 4) for i, nm in enumerate(names) if acc[i] > 0}}


def shard_slice(batch, cells: np.ndarray, world: int, rank: int):
    """This rank's contiguous slice of the fixed batch, balanced by in-band
    cells (shard.balanced_ranges), with query positions rebased to its own
    query bytes.  Returns (windows, query, sizes of every rank, lo, hi)."""
    spans = shard.balanced_ranges(cells, world)
    lo, hi = spans[rank]
    sizes = [b - a for a, b in spans]
    stride = int(batch.windows["qpos"][1] - batch.windows["qpos"][0]) if len(batch) > 1 else 158
    wl = np.array(batch.windows[lo:hi])
    wl["qpos"] -= np.uint32(lo * stride)
    ql = np.array(batch.query[lo * stride:hi * stride])
    return wl, ql, sizes, lo, hi


def payload_budget(ranks, payload_header: np.ndarray, layout) -> int:
    """The op words every rank's payload must reserve: the largest total any
    rank's step emitted (its payload header, all-reduced MAX over ranks),
    with 25 % headroom when the current budget is short; 0 if it fits.  Every
    rank gets the same answer, so the payloads stay equal-sized for the one
    gather."""
    need = shard.max_over_ranks(ranks, float(int(payload_header.view(np.int64)[0])))
    return 0 if need <= layout.budget else int(need * 1.25) + 1024


def measure_slices(ctx, batch, cells, dev, sp, t1_ms, steps=20, warmup=3, xgmi_gbs=XGMI_LINK_GBS):
    """The N = 2, 4, 8 step of the fixed batch, projected from one GPU: every
    rank's slice (shard.balanced_ranges, as bench.py --gpus N cuts it) run
    through the per-rank step itself -- k_plan / k_scan / k_scatter, k_fill,
    k_rows, and the op-stream compaction into the payload -- timed like the
    bench's step (K steps between two synchronisations), k_fill by HIP events.  A step of N ranks takes its slowest slice;
    the RCCL gather of the N - 1 remote payloads into rank 0 (bytes measured
    here) is asynchronous in the step and overlaps the next one, and is
    bounded below at one xGMI link per peer.  projected = T(1) / T(N)."""
    out = {"method": "per-rank step on each slice of the fixed batch, one GPU, K steps between synchronisations; "
                     "gather overlapped (payload bytes and their one-link time reported beside)",
           "t1_ms": round(t1_ms, 4), "slices": {}}
    for N in (2, 4, 8):
        worst, fill_worst, pay_bytes = 0.0, 0.0, 0
        per = []
        for r in range(N):
            wl, ql, sizes, lo, hi = shard_slice(batch, cells, N, r)
            n = hi - lo
            off = op_offsets(wl)
            d_w = torch.from_numpy(wl.view(np.uint8).copy()).to(dev)
            d_q = torch.from_numpy(ql.copy()).to(dev)
            d_off = torch.from_numpy(off.copy()).to(dev)
            d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
            lay = gather.Layout(max(sizes), gather.op_budget(max(sizes)))
            payb = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
            base = payb.data_ptr()

            def step():
                ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), base + lay.res_off,
                               d_ops.data_ptr(), d_off.data_ptr(), stream=sp)
                ctx.compact_ops_device(base + lay.res_off, n, d_ops.data_ptr(), d_off.data_ptr(),
                                       base + lay.ops_off, lay.budget, base, stream=sp)
            ms = 1000.0 * timed(step, ctx.sync, steps, warmup) / steps
            names = ctx.profile(True)
            acc = np.zeros(len(names))
            for _ in range(steps):
                step()
                ctx.profile_read(acc)
            ctx.profile(False)
            fill = float(sum(acc[i] for i, nm in enumerate(names) if nm.startswith("k_fill"))) / steps
            nops = int(payb[:gather.HEADER].cpu().numpy().view(np.int64)[0])
            pay_bytes = max(pay_bytes, gather.HEADER + n * RESULT.itemsize + 4 * nops)
            per.append(round(ms, 4))
            if ms > worst:
                worst, fill_worst = ms, fill
        gather_ms = pay_bytes / (xgmi_gbs * 1e9) * 1e3
        out["slices"][str(N)] = {"reads_per_rank": int(len(batch) // N), "slice_ms": per,
                                 "step_ms": round(worst, 4), "k_fill_ms": round(fill_worst, 4),
                                 "fixed_ms": round(worst - fill_worst, 4),
                                 "fixed_frac": round((worst - fill_worst) / worst, 4),
                                 "payload_bytes_per_rank": pay_bytes,
                                 "gather_one_link_ms": round(gather_ms, 4),
                                 "projected_scaling": round(t1_ms / worst, 3),
                                 "projected_scaling_gather_unoverlapped": round(t1_ms / (worst + gather_ms), 3)}
    return out


def relaunch_if_needed(args) -> None:
    """--gpus N > 1 without a launcher: run this script under
    torch.distributed.run as a child (before anything touches the GPU) and
    exit with its status.  Under a launcher, WORLD_SIZE must equal N."""
    world = os.environ.get("WORLD_SIZE")
    if world is None and args.gpus > 1:
        import socket
        import subprocess
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if int(world or "1") != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%s\n" % (args.gpus, world))
        sys.exit(2)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=C3_READS, help="reads in the (fixed) batch")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline / parity leg")
    ap.add_argument("--no-side", action="store_true", help="skip every side line (C2, C4, C5, sj, micro, PCIe)")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the splice-junction / microexon side lines")
    ap.add_argument("--c4-windows", type=int, default=C4_WINDOWS)
    ap.add_argument("--c4-transcripts", type=int, default=C4_TRANSCRIPTS,
                    help="transcripts in the C4 final-pass line (BASELINE: 50k)")
    ap.add_argument("--no-c4t", action="store_true", help="skip the C4 transcript line")
    ap.add_argument("--no-steady", action="store_true", help="skip the >= 1 s steady-state figure (profiling runs)")
    ap.add_argument("--no-slices", action="store_true", help="skip the N = 2/4/8 slice projection")
    args = ap.parse_args()
    relaunch_if_needed(args)

    ranks = shard.init_from_env("nccl")
    world, rank, local = ranks.world, ranks.rank, ranks.local
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    # ---- workload: the same fixed batch on every rank, sliced per read (balanced by in-band
    # cells); generated once per node and mapped read-only by every rank (W.c3_cached)
    g, batch = W.c3_cached(args.reads, local)
    cells = cells_per_window(batch.windows)
    wl, ql, sizes, lo, hi = shard_slice(batch, cells, world, rank)
    n = hi - lo
    stride = int(batch.windows["qpos"][1] - batch.windows["qpos"][0]) if len(batch) > 1 else 158
    off = op_offsets(wl)
    ctx = Context(g.blocks, mode=0, device=local)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    d_w = torch.from_numpy(wl.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(ql.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    lay = gather.Layout(max(sizes), gather.op_budget(max(sizes)))
    pay, recv = [], []

    def alloc_payloads():
        pay[:] = [torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
        recv[:] = [[torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev) for _ in range(world)]
                   if (rank == 0 and world > 1) else None for _ in range(2)]
    alloc_payloads()
    pending = [None, None]
    nstep = [0]
    torch.cuda.synchronize()

    def step():
        b = nstep[0] & 1
        nstep[0] += 1
        if pending[b] is not None:  # the gather that last read this payload (stream-ordered wait)
            pending[b].wait()
            pending[b] = None
        base = pay[b].data_ptr()
        ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), base + lay.res_off,
                       d_ops.data_ptr(), d_off.data_ptr(), stream=sp)
        ctx.compact_ops_device(base + lay.res_off, n, d_ops.data_ptr(), d_off.data_ptr(), base + lay.ops_off,
                               lay.budget, base, stream=sp)
        if world > 1:
            pending[b] = shard.gather_to_root(ranks, pay[b], recv[b], async_op=True)

    def sync():
        for b in (0, 1):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None
        torch.cuda.synchronize()

    for _ in range(max(1, args.warmup)):
        step()
    sync()
    # an indel-heavier batch than the default budget allows: resize every rank's
    # payload (the header's op total, all-reduced) and warm up again
    grow = payload_budget(ranks, pay[(nstep[0] - 1) & 1][:gather.HEADER].cpu().numpy(), lay)
    if grow:
        lay = gather.Layout(max(sizes), grow)
        alloc_payloads()
        for _ in range(max(1, args.warmup)):
            step()
        sync()

    # ---- timed region: exactly K steps, barrier + sync on both sides, max over ranks
    elapsed = shard.timed_steps(ranks, step, args.steps, sync)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = args.reads * args.steps / elapsed  # the whole fixed batch per step, all ranks together
    steady = None
    if elapsed < MIN_STEADY_S and not args.no_steady:
        k2 = int(np.ceil(MIN_STEADY_S / (elapsed / args.steps)))
        el2 = shard.timed_steps(ranks, step, k2, sync)
        steady = {"steps": k2, "seconds": round(el2, 4), "value": round(args.reads * k2 / el2, 1),
                  "ms_per_step": round(1000.0 * el2 / k2, 4)}

    # ---- per-kernel durations (HIP events on the launch stream), same K steps
    names = ctx.profile(True)
    acc = np.zeros(len(names), dtype=np.float64)
    for _ in range(args.steps):
        step()
        ctx.profile_read(acc)
    ctx.profile(False)
    sync()
    kernel_ms = {nm: acc[i] / args.steps for i, nm in enumerate(names) if acc[i] > 0}
    last = (nstep[0] - 1) & 1

    # ---- this rank's results (last step): sanity + algorithmic bytes of the dominant kernel
    res_l = np.frombuffer(pay[last][lay.res_off:lay.res_off + n * RESULT.itemsize].cpu().numpy().tobytes(),
                          dtype=RESULT)
    Wd = (wl["extraband"].astype(np.int64) * 2 + 1 + np.abs(wl["length2"].astype(np.int64) - wl["length1"]))
    dom = (Wd <= 48) & (wl["length2"] <= 640)  # k_fill's windows (FAST_WMAX, FAST_L2MAX)
    # d_q is passed as both query and query_uc: its bytes count once
    dom_bytes = float(window_bytes(wl[dom], res_l["nops"][dom], uc_aliased=True).sum())
    dom_ms = kernel_ms.get(DOMINANT, float("nan"))
    achieved_gbs = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms == dom_ms else None
    fill_ms = sum(v for k, v in kernel_ms.items() if k.startswith("k_fill"))
    cells_local = int(cells[lo:hi].sum())
    traffic = pmc_traffic(DOMINANT, "C3")
    rp = rocprof_kernel_ms(DOMINANT, "C3")

    out = None
    if rank == 0:
        # ---- the gathered batch (every rank's payload of the last step) on the root
        bufs = ([t.cpu().numpy() for t in recv[last]] if world > 1 else [pay[last].cpu().numpy()])
        res, cops, coff = gather.reassemble(lay, bufs, sizes)
        threads, host_cpus, cpu_model = cpu_info()
        cpu = parity = None
        if not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O  # CPU restatement: baseline + checker only
            O.setup(g.blocks)
            fields = ("finalscore", "nmatches", "nmismatches", "nopens", "nindels", "reserved")
            same = True
            t_cpu = 0.0
            chunk = 125_000
            for a in range(0, args.reads, chunk):
                ws = batch.windows[a:a + chunk]
                t1 = time.perf_counter()
                ores, _, _, _ = O.run_batch(ws, batch.query, batch.query_uc, nthreads=threads)
                t_cpu += time.perf_counter() - t1
                same = same and all(np.array_equal(res[f][a:a + chunk], ores[f]) for f in fields)
            t2 = time.perf_counter()
            one = min(args.reads, 20_000)
            O.run_batch(batch.windows[:one], batch.query, batch.query_uc, nthreads=1)
            cpu1 = one / (time.perf_counter() - t2)
            # full pair lists of a sample, expanded from the GATHERED compact op streams
            rng = np.random.default_rng(0)
            samp = np.unique(np.concatenate([np.arange(min(500, args.reads)),
                                             rng.integers(0, args.reads, size=min(1500, args.reads))]))
            ores, opairs, ooff, onp = O.run_batch(batch.windows[samp], batch.query, batch.query_uc,
                                                  nthreads=threads)
            pairs_ok = True
            for j, i in enumerate(samp.tolist()):
                p, _ = ctx.pairs(batch.windows, batch.query, batch.query_uc, res, cops, coff, i)
                if p.tobytes() != opairs[ooff[j]:ooff[j] + onp[j]].tobytes():
                    pairs_ok = False
                    break
            parity = {"windows_checked": args.reads, "fields": list(fields), "scores_and_counts_bit_exact": bool(same),
                      "pair_lists_checked": int(samp.size), "pair_lists_bit_exact": bool(pairs_ok),
                      "source": "results + compact op streams gathered to rank 0 (%d rank%s)"
                                % (world, "s" if world > 1 else "")}
            cpu = {"value": round(args.reads / t_cpu, 1), "unit": "reads/s", "cores": threads, "kind": "port",
                   "host_cpus": host_cpus, "cpu_model": cpu_model,
                   "sample": "the whole %d-read C3 batch once (oracle/ restatement, %d pthreads, %.1f s); "
                             "1 thread: %.0f reads/s on %d reads" % (args.reads, threads, t_cpu, cpu1, one)}
        out = {
            "metric": "aligned reads/sec (whole node), 150 bp vs GRCh38; bit-exact vs CPU dynprog",
            "value": round(value, 1),
            "unit": "reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (GRCh38-shaped genome: 24 chromosomes with the GRCh38 lengths, uniform ACGT, 0.1% N "
                    "runs; 150 bp reads from both strands, 2% subs, 0.1% N, 30% with a 1-3 bp indel)",
            "config": {"workload": "C3: Dynprog_single_gap, one fixed batch of %d x 150 bp reads vs a %.2f Gnt "
                                   "GRCh38-sized genome, extraband 15 (band 31), widebandp, HIGHQ, both strands; "
                                   "split per read over %d GPU%s, RCCL gather of results + compact op streams "
                                   "to rank 0" % (args.reads, g.total / 1e9, world, "s" if world > 1 else ""),
                       "reads": args.reads, "genome_nt": g.total, "reads_per_gpu": sizes,
                       "parallelism": "dp%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2) if achieved_gbs else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 5) if achieved_gbs else None,
                         "traffic": traffic[0] if traffic else None,
                         "traffic_source": traffic[1] if traffic else None,
                         "algorithmic_bytes": round(dom_bytes), "kernel": DOMINANT,
                         "bytes_note": "per window: L1 query bytes (query and query_uc are one buffer here, "
                                       "counted once) + 12 B per genome block touched + 68 B descriptor + "
                                       "48 B result + 4 B per op",
                         "kernel_ms": round(dom_ms, 4), "kernel_ms_rocprof": round(rp[0], 4) if rp else None,
                         "rocprof_source": rp[1] if rp else None, "windows_in_kernel": int(dom.sum())},
            "roofline_valu": {"bound": "valu-int32", "unit": "int32 ops/s",
                              "achieved": round(cells_local * OPS_PER_CELL / (fill_ms * 1e-3), 1) if fill_ms else None,
                              "peak": VALU_INT32_PEAK,
                              "frac": round(cells_local * OPS_PER_CELL / (fill_ms * 1e-3) / VALU_INT32_PEAK, 4)
                              if fill_ms else None,
                              "note": "14 ops per in-band cell over all k_fill launches (SURVEY.md 8(d)); peak at "
                                      "the measured 4-cycle int32 issue (tools/ubench/valu_rate.hip)"},
            "kernel_ms_per_step": {k: round(v, 4) for k, v in kernel_ms.items()},
            "gcups": round(float(cells.sum()) * args.steps / elapsed / 1e9, 2),
            "steady_state": steady,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if world == 1 and not args.no_slices and not args.no_side:
            out["projected_scaling"] = measure_slices(ctx, batch, cells, dev, sp, ms_per_step)
        if world == 1 and not args.no_side:
            genome = W.synthetic_genome(GENOME_NT, seed=1)
            out["c2"] = measure_c2(genome, C2_READS, 20, args.warmup, dev)
            # the host-buffer boundary (gsnapdp_run_host: H2D of windows and queries, the same
            # kernels, D2H of results and the compacted op streams) on 100k reads of the batch,
            # from page-locked host buffers -- never `value`
            from gsnapdp import pinned_copy, pinned_empty
            m = 100_000
            hw, hq = pinned_copy(batch.windows[:m]), pinned_copy(batch.query[:m * stride])
            hoff = pinned_copy(op_offsets(hw))
            hres, hops = pinned_empty(m, RESULT), pinned_empty(int(hoff[-1]) + 1, np.uint32)
            ctx.run(hw, hq, hq, out=(hres, hops, hoff))
            reps = 10
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.run(hw, hq, hq, out=(hres, hops, hoff))
            host_ms = 1000.0 * (time.perf_counter() - t0) / reps
            out["pcie_inclusive"] = {"value": round(m / (host_ms * 1e-3), 1), "unit": "reads/s",
                                     "ms_per_batch": round(host_ms, 4), "reads": m,
                                     "entry": "gsnapdp_run_host (page-locked host buffers in and out, "
                                              "one buffer for query and query_uc; compacted op streams D2H)"}
            if not args.no_c4:
                out["c4"] = measure_c4(genome, args.c4_windows, 20, args.warmup, dev, not args.no_cpu)
            if not args.no_c5:
                out["c5"] = measure_c5(genome, C5_READS, 20, args.warmup, dev, not args.no_cpu)
            if not args.no_extra:
                out["splicejunction"] = measure_sj(genome, 100_000, 20, args.warmup, dev, not args.no_cpu)
                out["microexon"] = measure_micro(genome, 20_000, 20, args.warmup, dev, not args.no_cpu)
                out["stage3_pass"] = measure_stage3()
                out["stage3_compute"] = measure_stage3_compute(cpu=not args.no_cpu)
            if not args.no_c4t:
                out["c4_transcripts"] = measure_c4_transcripts(args.c4_transcripts, not args.no_cpu)
        print(json.dumps(out), flush=True)
    shard.finish(ranks)
    ctx.close()


if __name__ == "__main__":
    main()
