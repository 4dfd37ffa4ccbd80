#!/usr/bin/env python3
"""Benchmark: GMAP/GSNAP stage-3 single-gap DP on MI355X (BASELINE config 2).

One step = one pass of the hot path (Dynprog_single_gap fill + endpoint +
traceback, batched through gsnapdp_run_device) over one batch of 100k
synthetic 150 bp reads (band 31, 2 % substitutions, 30 % with a 1-3 bp indel)
already resident in HBM.  N GPUs: one process per GPU, each aligning its own
100k-read shard against a replicated genome (weak scaling, no data-path
collective: windows are independent).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1 under torch.distributed.run, see the task contract)
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

from gsnapdp import Context, op_offsets, shard  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import RESULT  # noqa: E402

HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# int32 VALU: measured 4 cycles per wave64 instruction on gfx950 (v_max_i32,
# v_add_u32, v_alignbit_b32; tools/ubench/valu_rate.hip), i.e. 16 lanes/clk per
# SIMD (fp32 FMA issues at 2 cycles): 256 CU x 4 SIMD x 16 lanes x 2.4 GHz
VALU_INT32_PEAK = 256 * 4 * 16 * 2.4e9
OPS_PER_CELL = 14             # gap1 4 + gap2 4 + nogap 6 int32 ops
READS_PER_GPU = 100_000
GENOME_NT = 64_000_000
DOMINANT = "k_fill"           # every C2 window is a register-band (k_fill) window
C4_WINDOWS = 200_000          # intron windows per config-4 step
C5_READS = 100_000            # reads per config-5 step (3 DP windows each)


def window_bytes(w: np.ndarray, nops: np.ndarray) -> np.ndarray:
    """Algorithmic HBM bytes of one window (DESIGN.md "Roofline"): query and
    uppercase query (L1 each), the packed genome blocks its columns touch
    (12 B per 32 nt), the 68 B descriptor, the 48 B result and 4 B per op."""
    span_blocks = (w["length2"].astype(np.int64) + 31) // 32 + 1
    return (2 * w["length1"].astype(np.int64) + 12 * span_blocks + 68 + 48 + 4 * nops.astype(np.int64))


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


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/*_traffic.json, written by tools/pmc_traffic.py), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("kernel") == kernel:
            best = (d["traffic_bytes"], os.path.basename(f))
    return best


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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=READS_PER_GPU)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-c4", action="store_true", help="skip the config-4 (genome gap) side line")
    ap.add_argument("--c4-windows", type=int, default=C4_WINDOWS)
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 (GSNAP windows) side line")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the splice-junction / microexon side lines")
    args = ap.parse_args()

    ranks = shard.init_from_env("nccl")
    world, rank, local = ranks.world, ranks.rank, ranks.local
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    # ---- workload (identical genome on every rank, a disjoint read shard per rank)
    genome = W.synthetic_genome(GENOME_NT, seed=1)
    blocks = W.pack_genome(genome)
    batch = W.c2_windows(genome, n=args.reads, seed=shard.shard_seed(2, rank))
    n = len(batch)
    off = op_offsets(batch.windows)
    ctx = Context(blocks, mode=0, device=local)

    d_w = torch.from_numpy(batch.windows.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(batch.query.copy()).to(dev)
    d_u = torch.from_numpy(batch.query_uc.copy()).to(dev)
    d_off = torch.from_numpy(off.copy()).to(dev)
    d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step():
        ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(),
                       d_ops.data_ptr(), d_off.data_ptr())

    def sync():
        ctx.sync()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    sync()

    # ---- timed region: exactly K steps, barrier + sync on both sides, max over ranks
    elapsed = shard.timed_steps(ranks, step, args.steps, sync)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = shard.aggregate_rate(n, ranks, args.steps, elapsed)

    # ---- per-kernel durations (HIP events on the launch stream), same K steps
    names = ctx.profile(True)
    acc = np.zeros(len(names), dtype=np.float64)
    for _ in range(args.steps):
        step()
        ctx.profile_read(acc)
    ctx.profile(False)
    kernel_ms = {nm: acc[i] / args.steps for i, nm in enumerate(names) if acc[i] > 0}

    # ---- results of the last step: sanity + algorithmic bytes
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=RESULT)
    Wd = (batch.windows["extraband"].astype(np.int64) * 2 + 1
          + np.abs(batch.windows["length2"].astype(np.int64) - batch.windows["length1"]))
    dom = (Wd <= 48) & (batch.windows["length2"] <= 640)  # k_fill's windows (FAST_WMAX, FAST_L2MAX)
    dom_bytes = float(window_bytes(batch.windows[dom], res["nops"][dom]).sum())
    dom_ms = kernel_ms.get(DOMINANT, float("nan"))
    achieved_gbs = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms == dom_ms else None
    cells = band_cells(batch.windows)
    fill_ms = sum(v for k, v in kernel_ms.items() if k.startswith("k_fill"))

    traffic = pmc_traffic(DOMINANT)
    out = None
    if rank == 0:
        cpu = None
        parity = None
        if not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O  # CPU restatement: baseline + checker only
            O.setup(blocks)
            cores = 16
            sample = min(n, 100_000)
            ws = batch.windows[:sample]
            t1 = time.perf_counter()
            reps = 0
            while True:
                ores, _, _, _ = O.run_batch(ws, batch.query, batch.query_uc, nthreads=cores)
                reps += 1
                if time.perf_counter() - t1 > 3.0:
                    break
            cpu_rate = reps * sample / (time.perf_counter() - t1)
            t2 = time.perf_counter()
            O.run_batch(ws[:10_000], batch.query, batch.query_uc, nthreads=1)
            cpu1 = 10_000 / (time.perf_counter() - t2)
            same = all(np.array_equal(res[f][:sample], ores[f]) for f in
                       ("finalscore", "nmatches", "nmismatches", "nopens", "nindels"))
            parity = {"windows_checked": sample, "scores_and_counts_bit_exact": bool(same)}
            cpu = {"value": round(cpu_rate, 1), "unit": "reads/s", "cores": cores, "kind": "port",
                   "sample": "%d C2 windows x %d passes (oracle/ restatement, pthreads); 1 core: %.0f reads/s"
                             % (sample, reps, cpu1)}
        out = {
            "metric": "aligned reads/sec (whole node), 150 bp vs GRCh38; bit-exact vs CPU dynprog",
            "value": round(value, 1),
            "unit": "reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (64 Mbp uniform genome with N runs; 150 bp reads, 2% subs, 30% 1-3 bp indels)",
            "config": {"workload": "C2: Dynprog_single_gap, %d x 150 bp reads per GPU, extraband 15 (band 31), "
                                   "widebandp, HIGHQ, both strands" % n,
                       "reads_per_gpu": n, "genome_nt": GENOME_NT, "parallelism": "dp%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2) if achieved_gbs else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 5) if achieved_gbs else None,
                         "traffic": traffic[0] if traffic else None,
                         "traffic_source": traffic[1] if traffic else None,
                         "algorithmic_bytes": round(dom_bytes), "kernel": DOMINANT,
                         "kernel_ms": round(dom_ms, 4), "windows_in_kernel": int(dom.sum())},
            "roofline_valu": {"bound": "valu-int32", "unit": "int32 ops/s",
                              "achieved": round(cells * OPS_PER_CELL / (fill_ms * 1e-3), 1) if fill_ms else None,
                              "peak": VALU_INT32_PEAK,
                              "frac": round(cells * OPS_PER_CELL / (fill_ms * 1e-3) / VALU_INT32_PEAK, 4)
                              if fill_ms else None,
                              "note": "14 ops per in-band cell over all k_fill launches (SURVEY.md 8(d))"},
            "kernel_ms_per_step": {k: round(v, 4) for k, v in kernel_ms.items()},
            "gcups": round(cells * args.steps * world / elapsed / 1e9, 2),
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if world == 1:
            # the host-buffer boundary (gsnapdp_run_host: H2D of windows and queries, the same
            # kernels, D2H of results and op streams) on the same batch -- never `value`
            ctx.run(batch.windows, batch.query, batch.query_uc)
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.run(batch.windows, batch.query, batch.query_uc)
            host_ms = 1000.0 * (time.perf_counter() - t0) / reps
            out["pcie_inclusive"] = {"value": round(n / (host_ms * 1e-3), 1), "unit": "reads/s",
                                     "ms_per_batch": round(host_ms, 4), "reads": n,
                                     "entry": "gsnapdp_run_host (host buffers in and out)"}
        if not args.no_c4 and world == 1:
            out["c4"] = measure_c4(genome, args.c4_windows, args.steps, args.warmup, dev, not args.no_cpu)
        if not args.no_c5 and world == 1:
            out["c5"] = measure_c5(genome, C5_READS, args.steps, args.warmup, dev, not args.no_cpu)
        if not args.no_extra and world == 1:
            out["splicejunction"] = measure_sj(genome, 100_000, args.steps, args.warmup, dev, not args.no_cpu)
            out["microexon"] = measure_micro(genome, 20_000, args.steps, args.warmup, dev, not args.no_cpu)
        print(json.dumps(out), flush=True)
    shard.finish(ranks)
    ctx.close()


if __name__ == "__main__":
    main()
