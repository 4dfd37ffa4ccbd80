"""ctypes binding of the CPU restatement (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
library (gmap-gsnap_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp.records import (CGAP_RESULT, CGAP_WINDOW, GGAP_RESULT, GGAP_WINDOW, INTRON,  # noqa: E402
                             INTRON_PATH, INTRON_SCORES, MICRO_RESULT, MICRO_WINDOW, PAIR, PATH_PAIR,
                             RESULT, SJ_WINDOW, WINDOW)

LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
TABLES_PATH = os.path.join(ROOT, "gmap-gsnap_amd", "data", "maxent_hr_tables.bin")

_lib = None
_keep = {}


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(HERE, f) for f in ("dp_oracle.c", "maxent_oracle.c", "dp_oracle.h")]
        if not os.path.exists(LIB_PATH) or any(os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in srcs):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        L.orc_init.argtypes = [i32]
        L.orc_set_genome.argtypes = [vp]
        L.orc_maxent_load.argtypes = [vp, ctypes.c_size_t]
        L.orc_maxent_load.restype = i32
        L.orc_run_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, i32]
        L.orc_run_ggap_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
        L.orc_run_cgap_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orc_run_sj_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
        L.orc_run_micro_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
        L.orc_maxent_batch.argtypes = [vp, vp, vp, vp, i32]
        L.orc_path_introns.argtypes = [vp, i32, i32, i32, vp, i32]
        L.orc_path_introns.restype = i32
        L.orc_score_introns.argtypes = [vp, i32, vp, vp]
        L.orc_pairdistance.argtypes = [i32, i32, i32]
        L.orc_pairdistance.restype = i32
        L.orc_consistent.argtypes = [i32, i32]
        L.orc_consistent.restype = i32
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def setup(blocks: np.ndarray, mode: int = 0, tables: np.ndarray | None = None) -> None:
    """Dynprog_init(mode) + Genome_user_setup/Maxent_hr_setup(blocks)."""
    L = lib()
    L.orc_init(mode)
    b = np.ascontiguousarray(blocks, dtype=np.uint32)
    _keep["blocks"] = b
    L.orc_set_genome(_p(b))
    if tables is None and os.path.exists(TABLES_PATH):
        tables = np.fromfile(TABLES_PATH, dtype="<f8")
    if tables is not None:
        t = np.ascontiguousarray(tables, dtype="<f8")
        _keep["tables"] = t
        if L.orc_maxent_load(_p(t), t.size) != 0:
            raise RuntimeError("maxent table size mismatch")


def pair_offsets_for(windows: np.ndarray, slack: int = 8) -> np.ndarray:
    """Worst-case list length per window: every pair of the window rectangle
    (a diagonal pair per row + a dash per column) + 2 gapholders."""
    if "length1L" in windows.dtype.names:  # cDNA gaps: both tracebacks + insertion pairs
        cap = (windows["length1L"].astype(np.int64) + windows["length1R"] + 2 * windows["length2"].astype(np.int64)
               + 18 + slack)
        off = np.zeros(len(windows) + 1, dtype=np.int64)
        np.cumsum(cap.clip(slack), out=off[1:])
        return off
    l1 = windows["length1"].astype(np.int64) if "length1" in windows.dtype.names else None
    if "revoffset2R" in windows.dtype.names and "length2L" not in windows.dtype.names:  # microexons
        off = np.zeros(len(windows) + 1, dtype=np.int64)
        np.cumsum(l1 + 2 + slack, out=off[1:])
        return off
    if "length2L" in windows.dtype.names:
        cap = 2 * l1 + windows["length2L"] + windows["length2R"] + slack
    else:
        cap = l1 + windows["length2"].astype(np.int64) + slack
    off = np.zeros(len(windows) + 1, dtype=np.int64)
    np.cumsum(cap, out=off[1:])
    return off


def run_batch(windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray, nthreads: int = 1):
    """Returns (results[RESULT], pairs[PAIR], pair_offsets[int64], npairs[int32])."""
    L = lib()
    w = np.ascontiguousarray(windows, dtype=WINDOW)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    u = np.ascontiguousarray(query_uc, dtype=np.uint8)
    res = np.zeros(len(w), dtype=RESULT)
    off = pair_offsets_for(w)
    pairs = np.zeros(int(off[-1]), dtype=PAIR)
    npairs = np.zeros(len(w), dtype=np.int32)
    L.orc_run_batch(_p(w), len(w), _p(q), _p(u), _p(res), _p(pairs), _p(off), _p(npairs), nthreads)
    return res, pairs, off, npairs


def run_ggap_batch(windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
    L = lib()
    w = np.ascontiguousarray(windows, dtype=GGAP_WINDOW)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    u = np.ascontiguousarray(query_uc, dtype=np.uint8)
    res = np.zeros(len(w), dtype=GGAP_RESULT)
    off = pair_offsets_for(w)
    pairs = np.zeros(int(off[-1]), dtype=PAIR)
    npairs = np.zeros(len(w), dtype=np.int32)
    L.orc_run_ggap_batch(_p(w), len(w), _p(q), _p(u), _p(res), _p(pairs), _p(off), _p(npairs))
    return res, pairs, off, npairs


def run_cgap_batch(windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray, gseg: np.ndarray,
                   gseg_off: np.ndarray):
    L = lib()
    w = np.ascontiguousarray(windows, dtype=CGAP_WINDOW)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    u = np.ascontiguousarray(query_uc, dtype=np.uint8)
    gs = np.ascontiguousarray(gseg, dtype=np.uint8)
    go = np.ascontiguousarray(gseg_off, dtype=np.int64)
    res = np.zeros(len(w), dtype=CGAP_RESULT)
    off = pair_offsets_for(w)
    pairs = np.zeros(int(off[-1]), dtype=PAIR)
    npairs = np.zeros(len(w), dtype=np.int32)
    L.orc_run_cgap_batch(_p(w), len(w), _p(q), _p(u), _p(gs), _p(go), _p(res), _p(pairs), _p(off), _p(npairs))
    return res, pairs, off, npairs


def run_sj_batch(windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
    """Dynprog_end5/3_splicejunction over gsnapdp_sj_window records."""
    L = lib()
    w = np.ascontiguousarray(windows, dtype=SJ_WINDOW)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    u = np.ascontiguousarray(query_uc, dtype=np.uint8)
    res = np.zeros(len(w), dtype=RESULT)
    off = pair_offsets_for(w)
    pairs = np.zeros(int(off[-1]), dtype=PAIR)
    npairs = np.zeros(len(w), dtype=np.int32)
    L.orc_run_sj_batch(_p(w), len(w), _p(q), _p(u), _p(res), _p(pairs), _p(off), _p(npairs))
    return res, pairs, off, npairs


def run_micro_batch(windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
    """Dynprog_microexon_int over gsnapdp_micro_window records (needs setup())."""
    L = lib()
    w = np.ascontiguousarray(windows, dtype=MICRO_WINDOW)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    u = np.ascontiguousarray(query_uc, dtype=np.uint8)
    res = np.zeros(len(w), dtype=MICRO_RESULT)
    off = pair_offsets_for(w)
    pairs = np.zeros(int(off[-1]), dtype=PAIR)
    npairs = np.zeros(len(w), dtype=np.int32)
    L.orc_run_micro_batch(_p(w), len(w), _p(q), _p(u), _p(res), _p(pairs), _p(off), _p(npairs))
    return res, pairs, off, npairs


def maxent(model: np.ndarray, pos: np.ndarray, chroffset: np.ndarray) -> np.ndarray:
    L = lib()
    m = np.ascontiguousarray(model, dtype=np.uint8)
    p = np.ascontiguousarray(pos, dtype=np.uint32)
    c = np.ascontiguousarray(chroffset, dtype=np.uint32)
    out = np.zeros(len(m), dtype=np.float64)
    L.orc_maxent_batch(_p(m), _p(p), _p(c), _p(out), len(m))
    return out


def path_introns(pairs: np.ndarray, nullgap: int, path: int = 0) -> np.ndarray:
    """score_introns' intron walk over one path's PATH_PAIR records (stage3.c:7960-8146)."""
    L = lib()
    pr = np.ascontiguousarray(pairs, dtype=PATH_PAIR)
    n = L.orc_path_introns(_p(pr), len(pr), nullgap, path, None, 0)
    if n < 0:
        raise ValueError("an intron at the end of the path (the reference dereferences NULL)")
    out = np.zeros(max(n, 1), dtype=INTRON)
    L.orc_path_introns(_p(pr), len(pr), nullgap, path, _p(out), n)
    return out[:n]


def score_introns(paths: np.ndarray, introns: np.ndarray) -> np.ndarray:
    """score_introns' averages and bad-intron counts (stage3.c:7992-8157), per path."""
    L = lib()
    pa = np.ascontiguousarray(paths, dtype=INTRON_PATH)
    it = np.ascontiguousarray(introns, dtype=INTRON)
    out = np.zeros(len(pa), dtype=INTRON_SCORES)
    L.orc_score_introns(_p(pa), len(pa), _p(it) if it.size else None, _p(out))
    return out


def pairs_of(pairs: np.ndarray, off: np.ndarray, npairs: np.ndarray, i: int) -> np.ndarray:
    return pairs[off[i]:off[i] + npairs[i]]


# ---- the stage-3 pass on the CPU (oracle/_build/libstage3_cpu.so): the pass's host
# code with its DP batches served by this restatement, on GSNAPDP_S3_THREADS threads.
# bench.py's same-box baseline for the pass, and the checker of the full C4 set.
S3LIB_PATH = os.path.join(HERE, "_build", "libstage3_cpu.so")
_s3lib = None


def s3lib():
    global _s3lib
    if _s3lib is None:
        if not os.path.exists(S3LIB_PATH):
            build()
        L = ctypes.CDLL(S3LIB_PATH)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.gsnapdp_create.argtypes = [i32, vp, ctypes.c_size_t, i32]
        L.gsnapdp_create.restype = vp
        L.gsnapdp_destroy.argtypes = [vp]
        L.gsnapdp_load_maxent_tables.argtypes = [vp, vp, ctypes.c_size_t]
        L.gsnapdp_load_maxent_tables.restype = i32
        L.gsnapdp_stage3_pass.argtypes = [vp, vp, i32, vp, i64, vp, vp, ctypes.c_size_t, vp, vp, i64, vp]
        L.gsnapdp_stage3_pass.restype = i32
        L.gsnapdp_stage3_pass_compact.argtypes = [vp, vp, i32, vp, i64, vp, vp, ctypes.c_size_t, vp, vp, i64, vp,
                                                  i64, vp]
        L.gsnapdp_stage3_pass_compact.restype = i32
        L.gsnapdp_stage3_score_introns.argtypes = [vp, vp, i32, vp, vp, vp]
        L.gsnapdp_stage3_score_introns.restype = i32
        L.gsnapdp_stage3_pass_runs.argtypes = [vp, vp, i32, vp, i64, vp, vp, vp, vp, ctypes.c_size_t, vp, vp, i64,
                                               vp, i64, vp]
        L.gsnapdp_stage3_pass_runs.restype = i32
        L.gsnapdp_stage3_score_introns_runs.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
        L.gsnapdp_stage3_score_introns_runs.restype = i32
        L.gsnapdp_iit_from_intervals.argtypes = [vp, i32]
        L.gsnapdp_iit_from_intervals.restype = vp
        L.gsnapdp_iit_free.argtypes = [vp]
        L.gsnapdp_oracle_stash_reset.argtypes = []
        L.gsnapdp_stage3_compute.argtypes = [vp, vp, i32, vp, i64, vp, vp, ctypes.c_size_t, vp, i32, vp, i64, vp]
        L.gsnapdp_stage3_compute.restype = i32
        L.gsnapdp_stage3_path_compute.argtypes = [vp, vp, i32, vp, i64, vp, vp, ctypes.c_size_t, vp, vp, vp, i64,
                                                  vp, vp]
        L.gsnapdp_stage3_path_compute.restype = i32
        L.gsnapdp_stage3_set_stage2.argtypes = [vp, vp]
        L.s2dbl_new.argtypes = [vp, i32, vp, i32]
        L.s2dbl_new.restype = vp
        L.s3cpu_last_error.restype = ctypes.c_char_p
        _s3lib = L
    return _s3lib


class Stage3Cpu:
    """gsnapdp_stage3_pass / gsnapdp_stage3_score_introns with the batches served
    by the restatement (test / baseline infrastructure)."""

    def __init__(self, blocks: np.ndarray):
        from gsnapdp.records import S3_CALL, S3_PAIR, S3_STATS, IIT_INTERVAL  # noqa: F401
        L = s3lib()
        self.blocks = np.ascontiguousarray(blocks, dtype=np.uint32)
        self.h = L.gsnapdp_create(0, self.blocks.ctypes.data, self.blocks.size, 0)
        tables = np.fromfile(TABLES_PATH, dtype=np.float64)
        if not self.h or L.gsnapdp_load_maxent_tables(self.h, tables.ctypes.data, tables.size):
            raise RuntimeError("libstage3_cpu: context")

    def set_stage2_recording(self, s2_calls, s2_pairs):
        """traverse_dual_break's stage 2 served from a gmap_trace recording (tests/dropin/stage2_double.c)"""
        L = s3lib()
        self._s2 = (np.ascontiguousarray(s2_calls), np.ascontiguousarray(s2_pairs))
        h = L.s2dbl_new(self._s2[0].ctypes.data, self._s2[0].size, self._s2[1].ctypes.data, self._s2[1].size)
        self._s2cb = (ctypes.c_void_p * 2)(h, ctypes.cast(L.s2dbl_compute_one, ctypes.c_void_p).value)
        L.gsnapdp_stage3_set_stage2(self.h, ctypes.addressof(self._s2cb))

    def compute(self, queries, paths_in, query, query_uc, min_intronlength=9):
        """gsnapdp_stage3_compute (passes 2A-6): (queries with out fields, lists, S3_COMPUTE_STATS)"""
        from gsnapdp.records import S3_CALL, S3_COMPUTE_STATS, S3_PAIR
        L = s3lib()
        c = np.array(queries, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(paths_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = 2 * int((2 * (c["querylength"].astype(np.int64) + c["npairs"]) + 64).sum()) + 1024
        out = np.empty(cap, dtype=S3_PAIR)
        st = np.zeros(1, dtype=S3_COMPUTE_STATS)
        try:
            if L.gsnapdp_stage3_compute(self.h, c.ctypes.data, len(c), pi.ctypes.data, pi.size, q.ctypes.data,
                                        qu.ctypes.data, min(q.size, qu.size), None, int(min_intronlength),
                                        out.ctypes.data, cap, st.ctypes.data):
                raise RuntimeError("libstage3_cpu compute: %s" % L.s3cpu_last_error().decode())
        finally:
            L.gsnapdp_oracle_stash_reset()
        return c, out[:int(c["nout"].sum())], st[0]

    def path_compute(self, queries, paths_in, query, query_uc, min_intronlength=9, maxintronlen_bound=1000000):
        """gsnapdp_stage3_path_compute (pass 2A to path_compute's return value):
        (queries with out fields, lists, their (donor_prob, acceptor_prob), S3_COMPUTE_STATS)"""
        from gsnapdp.records import S3_CALL, S3_COMPUTE_STATS, S3_PAIR, S3_PATH_OPTS
        L = s3lib()
        c = np.array(queries, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(paths_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = 2 * int((2 * (c["querylength"].astype(np.int64) + c["npairs"]) + 64).sum()) + 1024
        out = np.empty(cap, dtype=S3_PAIR)
        probs = np.empty((cap, 2), dtype=np.float64)
        o = np.zeros(1, dtype=S3_PATH_OPTS)
        o["min_intronlength"], o["maxintronlen_bound"] = min_intronlength, maxintronlen_bound
        st = np.zeros(1, dtype=S3_COMPUTE_STATS)
        try:
            if L.gsnapdp_stage3_path_compute(self.h, c.ctypes.data, len(c), pi.ctypes.data, pi.size, q.ctypes.data,
                                             qu.ctypes.data, min(q.size, qu.size), None, o.ctypes.data,
                                             out.ctypes.data, cap, probs.ctypes.data, st.ctypes.data):
                raise RuntimeError("libstage3_cpu path_compute: %s" % L.s3cpu_last_error().decode())
        finally:
            L.gsnapdp_oracle_stash_reset()
        n = int(c["nout"].sum())
        return c, out[:n], probs[:n], st[0]

    def run_compact(self, calls, pairs_in, query, query_uc):
        """gsnapdp_stage3_pass_compact: (calls, cells, new pairs, S3_STATS)"""
        from gsnapdp.records import S3_CALL, S3_PAIR, S3_STATS
        L = s3lib()
        c = np.array(calls, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = int((2 * (c["querylength"].astype(np.int64) + c["npairs"]) + 64).sum()) if len(c) else 1
        ncap = int((2 * c["querylength"].astype(np.int64) + 256).sum()) if len(c) else 1
        cells = np.empty(max(cap, 1), dtype=np.int32)
        new = np.empty(max(ncap, 1), dtype=S3_PAIR)
        st = np.zeros(1, dtype=S3_STATS)
        try:
            if L.gsnapdp_stage3_pass_compact(self.h, c.ctypes.data, len(c), pi.ctypes.data, pi.size, q.ctypes.data,
                                             qu.ctypes.data, min(q.size, qu.size), None, cells.ctypes.data, cap,
                                             new.ctypes.data, ncap, st.ctypes.data):
                raise RuntimeError("libstage3_cpu pass: %s" % L.s3cpu_last_error().decode())
        finally:
            L.gsnapdp_oracle_stash_reset()
        return c, cells[:int(c["nout"].sum())], new[:int(st[0]["new_pairs"])], st[0]

    def run_runs(self, calls, pairs_in, query, query_uc, gaps=None, gap_off=None, introns=False):
        """gsnapdp_stage3_pass_runs (+ gsnapdp_stage3_score_introns_runs):
        (calls, runs, new pairs, S3_STATS[, INTRON_SCORES])"""
        from gsnapdp.records import INTRON_SCORES, S3_CALL, S3_PAIR, S3_RUN, S3_STATS
        L = s3lib()
        c = np.array(calls, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        g = go = None
        if gaps is not None:
            g = np.ascontiguousarray(gaps, dtype=np.int32)
            go = np.ascontiguousarray(gap_off, dtype=np.int64)
        gp = (g.ctypes.data if g.size else go.ctypes.data) if g is not None else None
        gop = go.ctypes.data if go is not None else None
        cap = int((2 * (c["querylength"].astype(np.int64) + c["npairs"]) + 64).sum()) if len(c) else 1
        ncap = int((2 * c["querylength"].astype(np.int64) + 256).sum()) if len(c) else 1
        runs = np.empty(max(cap, 1), dtype=S3_RUN)
        new = np.empty(max(ncap, 1), dtype=S3_PAIR)
        st = np.zeros(1, dtype=S3_STATS)
        try:
            if L.gsnapdp_stage3_pass_runs(self.h, c.ctypes.data, len(c), pi.ctypes.data, pi.size, gp, gop,
                                          q.ctypes.data, qu.ctypes.data, min(q.size, qu.size), None,
                                          runs.ctypes.data, runs.size, new.ctypes.data, new.size, st.ctypes.data):
                raise RuntimeError("libstage3_cpu pass_runs: %s" % L.s3cpu_last_error().decode())
            res = (c, runs[:int(c["nout"].sum())], new[:int(st[0]["new_pairs"])], st[0])
            if introns:
                sc = np.zeros(len(c), dtype=INTRON_SCORES)
                if L.gsnapdp_stage3_score_introns_runs(self.h, c.ctypes.data, len(c), pi.ctypes.data, gp, gop,
                                                       runs.ctypes.data, new.ctypes.data, None, sc.ctypes.data):
                    raise RuntimeError("libstage3_cpu score_introns_runs: %s" % L.s3cpu_last_error().decode())
                res = res + (sc,)
        finally:
            L.gsnapdp_oracle_stash_reset()
        return res

    def run(self, calls, pairs_in, query, query_uc, intervals=None, introns=False):
        """(calls with out fields, the returned lists, S3_STATS[, INTRON_SCORES])"""
        from gsnapdp.records import IIT_INTERVAL, S3_CALL, S3_PAIR, S3_STATS
        L = s3lib()
        c = np.array(calls, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = int((2 * (c["querylength"].astype(np.int64) + c["npairs"]) + 64).sum()) if len(c) else 1
        out = np.empty(max(cap, 1), dtype=S3_PAIR)
        st = np.zeros(1, dtype=S3_STATS)
        iit = None
        if intervals is not None:
            iv = np.ascontiguousarray(intervals, dtype=IIT_INTERVAL)
            iit = L.gsnapdp_iit_from_intervals(iv.ctypes.data if iv.size else None, iv.size)
        try:
            if L.gsnapdp_stage3_pass(self.h, c.ctypes.data, len(c), pi.ctypes.data, pi.size, q.ctypes.data,
                                     qu.ctypes.data, min(q.size, qu.size), iit, out.ctypes.data, cap,
                                     st.ctypes.data):
                raise RuntimeError("libstage3_cpu pass: %s" % L.s3cpu_last_error().decode())
            n = int(c["nout"].sum())
            res = (c, out[:n], st[0])
            if introns:
                sc = np.zeros(len(c), dtype=INTRON_SCORES)
                if L.gsnapdp_stage3_score_introns(self.h, c.ctypes.data, len(c), out.ctypes.data, iit,
                                                  sc.ctypes.data):
                    raise RuntimeError("libstage3_cpu score_introns: %s" % L.s3cpu_last_error().decode())
                res = res + (sc,)
        finally:
            if iit:
                L.gsnapdp_iit_free(iit)
            L.gsnapdp_oracle_stash_reset()
        return res

    def close(self):
        if self.h:
            s3lib().gsnapdp_destroy(self.h)
            self.h = None
