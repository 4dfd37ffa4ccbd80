"""Host-side mirror of GMAP/GSNAP's stage-3 DP interface over the MI355X C-ABI.

The native library ``gmap-gsnap_amd/lib/libgsnapdp.so`` (HIP kernels for
gfx950 + the C-ABI of include/gsnapdp.h) is the product; this module is a thin
ctypes binding used by tests and bench.py.  There is no CPU fallback: if the
library or a gfx950 device is missing, ``Context`` raises.

Entry-point mapping (reference src/dynprog.c):
    Context.run(batch)           Dynprog_single_gap / Dynprog_end5_gap / Dynprog_end3_gap
                                 (batched; one gsnapdp_window per call)
    Context.pairs(batch, i, ...) the List_T of Pair_T the call returns
    Context.maxent(...)          Maxent_hr_{donor,acceptor,antidonor,antiacceptor}_prob
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .records import S3_DISALLOWED, S3_GAPP  # noqa: E402
from .records import (CGAP_RESULT, CGAP_WINDOW, GGAP_RESULT, GGAP_TRACE, GGAP_WINDOW,  # noqa: F401
                      IIT_INTERVAL, INTRON, INTRON_PATH, INTRON_SCORES, MAXENT_IN, MICRO_RESULT, MICRO_WINDOW, PAIR,
                      PATH_PAIR, RESULT, S3_CALL, S3_PAIR, S3_STATS, SJ_WINDOW, WINDOW)

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_PATH = os.environ.get("GSNAPDP_LIB") or os.path.join(PKG, "lib", "libgsnapdp.so")
TABLES_PATH = os.path.join(PKG, "data", "maxent_hr_tables.bin")

_lib = None
ST_INTERNAL = 6  # a kernel invariant failed (gsnapdp_internal.h)


class GsnapdpError(RuntimeError):
    pass


def lib():
    """Load the native library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GsnapdpError("native library missing: %s (run `make -C gmap-gsnap_amd`)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.gsnapdp_create.argtypes = [i32, vp, sz, i32]
        L.gsnapdp_create.restype = vp
        L.gsnapdp_destroy.argtypes = [vp]
        L.gsnapdp_last_error.restype = ctypes.c_char_p
        L.gsnapdp_device_arch.argtypes = [vp]
        L.gsnapdp_device_arch.restype = ctypes.c_char_p
        L.gsnapdp_run_host.argtypes = [vp, vp, i32, vp, vp, sz, vp, vp, vp]
        L.gsnapdp_run_host.restype = i32
        L.gsnapdp_run_device.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp]
        L.gsnapdp_run_device.restype = i32
        L.gsnapdp_sync.argtypes = [vp]
        L.gsnapdp_sync.restype = i32
        L.gsnapdp_expand.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32, vp]
        L.gsnapdp_expand.restype = i32
        L.gsnapdp_load_maxent_tables.argtypes = [vp, vp, sz]
        L.gsnapdp_load_maxent_tables.restype = i32
        L.gsnapdp_maxent_host.argtypes = [vp, vp, vp, vp, vp, i32]
        L.gsnapdp_maxent_host.restype = i32
        L.gsnapdp_maxent_device.argtypes = [vp, vp, vp, vp, vp, i32, vp]
        L.gsnapdp_maxent_device.restype = i32
        L.gsnapdp_scratch_bytes.argtypes = [vp, i32, i32, i32]
        L.gsnapdp_scratch_bytes.restype = sz
        L.gsnapdp_profile.argtypes = [vp, i32]
        L.gsnapdp_profile.restype = i32
        L.gsnapdp_profile_read.argtypes = [vp, vp, i32]
        L.gsnapdp_profile_read.restype = i32
        L.gsnapdp_stage_name.argtypes = [i32]
        L.gsnapdp_debug_buckets.argtypes = [vp, i32, vp, vp, ctypes.c_int64, vp, vp, i32]
        L.gsnapdp_debug_buckets.restype = ctypes.c_int64
        L.gsnapdp_stage_name.restype = ctypes.c_char_p
        L.gsnapdp_ggap_run_host.argtypes = [vp, vp, i32, vp, vp, sz, vp, vp, vp, vp]
        L.gsnapdp_ggap_run_host.restype = i32
        L.gsnapdp_ggap_run_device.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
        L.gsnapdp_ggap_run_device.restype = i32
        L.gsnapdp_ggap_expand.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i32]
        L.gsnapdp_ggap_expand.restype = i32
        L.gsnapdp_cgap_run_host.argtypes = [vp, vp, i32, vp, vp, sz, vp, vp, vp]
        L.gsnapdp_cgap_run_host.restype = i32
        L.gsnapdp_cgap_run_device.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp]
        L.gsnapdp_cgap_run_device.restype = i32
        L.gsnapdp_cgap_expand.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i32]
        L.gsnapdp_cgap_expand.restype = i32
        L.gsnapdp_sj_run_host.argtypes = [vp, vp, i32, vp, vp, sz, vp, vp, vp]
        L.gsnapdp_sj_run_host.restype = i32
        L.gsnapdp_sj_run_device.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp]
        L.gsnapdp_sj_run_device.restype = i32
        L.gsnapdp_sj_expand.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32]
        L.gsnapdp_sj_expand.restype = i32
        L.gsnapdp_micro_run_host.argtypes = [vp, vp, i32, vp, vp, sz, vp]
        L.gsnapdp_micro_run_host.restype = i32
        L.gsnapdp_micro_run_device.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        L.gsnapdp_micro_run_device.restype = i32
        L.gsnapdp_micro_expand.argtypes = [vp, vp, vp, vp, vp, vp, i32]
        L.gsnapdp_micro_expand.restype = i32
        L.gsnapdp_host_alloc.argtypes = [sz]
        L.gsnapdp_host_alloc.restype = vp
        L.gsnapdp_host_free.argtypes = [vp]
        L.gsnapdp_compact_ops_device.argtypes = [vp, vp, i32, vp, vp, vp, ctypes.c_int64, vp, vp]
        L.gsnapdp_compact_ops_device.restype = i32
        L.gsnapdp_path_introns.argtypes = [vp, i32, i32, i32, vp, i32]
        L.gsnapdp_path_introns.restype = i32
        L.gsnapdp_score_introns_host.argtypes = [vp, vp, i32, vp, i32, vp]
        L.gsnapdp_score_introns_host.restype = i32
        L.gsnapdp_score_introns_device.argtypes = [vp, vp, i32, vp, vp, vp]
        L.gsnapdp_score_introns_device.restype = i32
        L.gsnapdp_stage3_pass.argtypes = [vp, vp, i32, vp, ctypes.c_int64, vp, vp, sz, vp, vp, ctypes.c_int64, vp]
        L.gsnapdp_stage3_pass.restype = i32
        L.gsnapdp_stage3_pass_compact.argtypes = [vp, vp, i32, vp, ctypes.c_int64, vp, vp, sz, vp, vp,
                                                  ctypes.c_int64, vp, ctypes.c_int64, vp]
        L.gsnapdp_stage3_pass_compact.restype = i32
        L.gsnapdp_stage3_compute.argtypes = [vp, vp, i32, vp, ctypes.c_int64, vp, vp, sz, vp, i32, vp,
                                             ctypes.c_int64, vp]
        L.gsnapdp_stage3_compute.restype = i32
        L.gsnapdp_stage3_path_compute.argtypes = [vp, vp, i32, vp, ctypes.c_int64, vp, vp, sz, vp, vp, vp,
                                                  ctypes.c_int64, vp, vp]
        L.gsnapdp_stage3_path_compute.restype = i32
        L.gsnapdp_stage3_set_stage2.argtypes = [vp, vp]
        L.gsnapdp_scan_site_probs.argtypes = [vp, vp, i32, vp]
        L.gsnapdp_scan_site_probs.restype = i32
        L.gsnapdp_stage3_set_stage2.restype = i32
        L.gsnapdp_stage3_score_introns.argtypes = [vp, vp, i32, vp, vp, vp]
        L.gsnapdp_stage3_score_introns.restype = i32
        L.gsnapdp_stage3_pass_runs.argtypes = [vp, vp, i32, vp, ctypes.c_int64, vp, vp, vp, vp, sz, vp, vp,
                                               ctypes.c_int64, vp, ctypes.c_int64, vp]
        L.gsnapdp_stage3_pass_runs.restype = i32
        L.gsnapdp_stage3_score_introns_runs.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
        L.gsnapdp_stage3_score_introns_runs.restype = i32
        L.gsnapdp_iit_from_intervals.argtypes = [vp, i32]
        L.gsnapdp_iit_from_intervals.restype = vp
        L.gsnapdp_iit_free.argtypes = [vp]
        L.gsnapdp_known_site_record.argtypes = [vp, i32, i32, ctypes.c_uint32, ctypes.c_uint32] + [i32] * 6 + \
            [vp, i32, vp]
        L.gsnapdp_known_site_record.restype = i32
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def path_introns(pairs: np.ndarray, nullgap: int, path: int = 0) -> np.ndarray:
    """score_introns' intron walk over one path's PATH_PAIR records
    (gsnapdp_path_introns, host code, stage3.c:7960-8146)."""
    pr = np.ascontiguousarray(pairs, dtype=PATH_PAIR)
    n = lib().gsnapdp_path_introns(_p(pr), len(pr), nullgap, path, None, 0)
    if n < 0:
        raise GsnapdpError("gsnapdp_path_introns: an intron at the end of the path")
    out = np.zeros(max(n, 1), dtype=INTRON)
    lib().gsnapdp_path_introns(_p(pr), len(pr), nullgap, path, _p(out), n)
    return out[:n]


class _Pinned:
    """Page-locked host memory (gsnapdp_host_alloc) exposed to numpy."""

    def __init__(self, nbytes: int):
        self.nbytes = max(1, int(nbytes))
        self.p = lib().gsnapdp_host_alloc(self.nbytes)
        if not self.p:
            raise GsnapdpError("gsnapdp_host_alloc(%d) failed" % self.nbytes)
        self.__array_interface__ = {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.p, False),
                                    "version": 3}

    def __del__(self):
        if getattr(self, "p", None):
            lib().gsnapdp_host_free(self.p)
            self.p = None


def pinned_empty(n: int, dtype) -> np.ndarray:
    """An uninitialised numpy array of n elements in page-locked host memory
    (the buffer lives as long as the array)."""
    dt = np.dtype(dtype)
    return np.asarray(_Pinned(n * dt.itemsize))[:n * dt.itemsize].view(dt)


def pinned_copy(a: np.ndarray) -> np.ndarray:
    out = pinned_empty(a.size, a.dtype)
    out[...] = a.reshape(-1)
    return out


def op_offsets(windows: np.ndarray) -> np.ndarray:
    """Per-window op capacity: a traceback takes at most L1 + L2 steps and
    every op consumes at least one step."""
    cap = windows["length1"].astype(np.int64).clip(0) + windows["length2"].astype(np.int64).clip(0) + 2
    off = np.zeros(len(windows) + 1, dtype=np.int64)
    np.cumsum(cap, out=off[1:])
    return off


def ggap_op_offsets(windows: np.ndarray) -> np.ndarray:
    """Per-intron-window op capacity: two tracebacks of at most L1 + L2 + 1 steps."""
    L1 = windows["length1"].astype(np.int64).clip(0)
    cap = 2 * L1 + windows["length2L"].astype(np.int64).clip(0) + windows["length2R"].astype(np.int64).clip(0) + 4
    off = np.zeros(len(windows) + 1, dtype=np.int64)
    np.cumsum(cap, out=off[1:])
    return off


def cgap_op_offsets(windows: np.ndarray) -> np.ndarray:
    """Per-cDNA-gap-window op capacity: two tracebacks of at most length1 + length2 + 1 steps."""
    cap = (windows["length1L"].astype(np.int64).clip(0) + windows["length1R"].astype(np.int64).clip(0)
           + 2 * windows["length2"].astype(np.int64).clip(0) + 4)
    off = np.zeros(len(windows) + 1, dtype=np.int64)
    np.cumsum(cap, out=off[1:])
    return off


class SplicingIIT:
    """A splicing IIT for the batched ABI (gsnapdp_iit_from_intervals): intervals
    as iit_store writes them (IIT_INTERVAL records: start > end is the minus
    sign; type -1 none, 0 donor, 1 acceptor)."""

    def __init__(self, intervals: np.ndarray):
        self.iv = np.ascontiguousarray(intervals, dtype=IIT_INTERVAL)
        self.h = lib().gsnapdp_iit_from_intervals(_p(self.iv) if self.iv.size else None, self.iv.size)
        if not self.h:
            raise GsnapdpError("gsnapdp_iit_from_intervals: %s" % lib().gsnapdp_last_error().decode())

    def close(self):
        if self.h:
            lib().gsnapdp_iit_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """A device context: packed genome resident in HBM (Genome_user_setup +
    Maxent_hr_setup) and the substitution tables of Dynprog_init(mode)."""

    def __init__(self, blocks: np.ndarray, mode: int = 0, device: int = 0, maxent_tables=None):
        L = lib()
        self._blocks = np.ascontiguousarray(blocks, dtype=np.uint32)
        h = L.gsnapdp_create(device, _p(self._blocks), self._blocks.size, mode)
        if not h:
            raise GsnapdpError("gsnapdp_create failed: %s" % L.gsnapdp_last_error().decode())
        self.h = ctypes.c_void_p(h)
        self.mode = mode
        if maxent_tables is None and os.path.exists(TABLES_PATH):
            maxent_tables = np.fromfile(TABLES_PATH, dtype="<f8")
        if maxent_tables is not None:
            t = np.ascontiguousarray(maxent_tables, dtype="<f8")
            if L.gsnapdp_load_maxent_tables(self.h, _p(t), t.size) != 0:
                raise GsnapdpError(L.gsnapdp_last_error().decode())

    def close(self):
        if getattr(self, "h", None):
            lib().gsnapdp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def arch(self) -> str:
        return lib().gsnapdp_device_arch(self.h).decode()

    def run(self, windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray, out=None):
        """Fill + endpoint + traceback on the GPU (gsnapdp_run_host).  Returns
        (results, ops, op_offsets); `out` = preallocated (results, ops, op_offsets)."""
        w = np.ascontiguousarray(windows, dtype=WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        if out is not None:
            res, ops, off = out
        else:
            off = op_offsets(w)
            res = np.zeros(len(w), dtype=RESULT)
            ops = np.zeros(max(1, int(off[-1])), dtype=np.uint32)
        rc = lib().gsnapdp_run_host(self.h, _p(w), len(w), _p(q), _p(u), q.size, _p(res), _p(ops), _p(off))
        if rc != 0:
            raise GsnapdpError("gsnapdp_run_host: %s" % lib().gsnapdp_last_error().decode())
        return res, ops, off

    def debug_buckets(self, n: int):
        """Test hook: the last single/end-gap batch's bucketing (gsnapdp_debug_buckets):
        (keys[n], perm[nperm], class_start[ncls + 1], class_wave[ncls])."""
        ncls = int(lib().gsnapdp_debug_buckets(self.h, 0, None, None, 0, None, None, 0))
        keys = np.zeros(max(n, 1), dtype=np.int32)
        cs = np.zeros(ncls + 1, dtype=np.int32)
        cw = np.zeros(ncls, dtype=np.int32)
        nperm = int(lib().gsnapdp_debug_buckets(self.h, n, _p(keys), None, 0, _p(cs), _p(cw), ncls))
        if nperm < 0:
            raise GsnapdpError("gsnapdp_debug_buckets: %s" % lib().gsnapdp_last_error().decode())
        perm = np.zeros(max(nperm, 1), dtype=np.int32)
        if lib().gsnapdp_debug_buckets(self.h, n, None, _p(perm), nperm, None, None, ncls) != nperm:
            raise GsnapdpError("gsnapdp_debug_buckets: %s" % lib().gsnapdp_last_error().decode())
        return keys[:n], perm[:nperm], cs, cw

    def pairs(self, windows, query, query_uc, results, ops, off, i: int) -> tuple[np.ndarray, int]:
        """The pair list window i's reference call returns (gsnapdp_expand)."""
        w = np.ascontiguousarray(windows[i:i + 1], dtype=WINDOW)
        r = np.ascontiguousarray(results[i:i + 1], dtype=RESULT)
        cap = int(w["length1"][0]) + int(w["length2"][0]) + 8
        out = np.zeros(cap, dtype=PAIR)
        fs = np.zeros(1, dtype=np.int32)
        o = ops[off[i]:]
        n = lib().gsnapdp_expand(self.h, _p(w), _p(r), _p(o), _p(query), _p(query_uc), _p(out), cap, _p(fs))
        if n < 0:
            raise GsnapdpError("gsnapdp_expand failed for window %d" % i)
        return out[:n], int(fs[0])

    def all_pairs(self, windows, query, query_uc, results, ops, off):
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        outs, counts = [], np.zeros(len(windows), dtype=np.int32)
        for i in range(len(windows)):
            p, _ = self.pairs(windows, q, u, results, ops, off, i)
            outs.append(p)
            counts[i] = p.size
        return (np.concatenate(outs) if outs else np.zeros(0, PAIR)), counts

    def ggap_run(self, windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
        """Dynprog_genome_gap on the GPU.  Returns (results, traces, ops, op_offsets)."""
        w = np.ascontiguousarray(windows, dtype=GGAP_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        off = ggap_op_offsets(w)
        res = np.zeros(len(w), dtype=GGAP_RESULT)
        trc = np.zeros(len(w), dtype=GGAP_TRACE)
        ops = np.zeros(max(1, int(off[-1])), dtype=np.uint32)
        rc = lib().gsnapdp_ggap_run_host(self.h, _p(w), len(w), _p(q), _p(u), q.size, _p(res), _p(trc),
                                         _p(ops), _p(off))
        if rc != 0:
            raise GsnapdpError("gsnapdp_ggap_run_host: %s" % lib().gsnapdp_last_error().decode())
        bad = np.nonzero(trc["status"] == ST_INTERNAL)[0]
        if bad.size:
            raise GsnapdpError("genome-gap kernel invariant failed in windows %s" % bad[:8])
        return res, trc, ops, off

    def ggap_run_device(self, d_windows: int, n: int, d_query: int, d_query_uc: int, d_results: int,
                        d_traces: int, d_ops: int, d_op_offsets: int, stream: int = 0) -> None:
        rc = lib().gsnapdp_ggap_run_device(
            self.h, ctypes.c_void_p(d_windows), n, ctypes.c_void_p(d_query), ctypes.c_void_p(d_query_uc),
            ctypes.c_void_p(d_results), ctypes.c_void_p(d_traces), ctypes.c_void_p(d_ops),
            ctypes.c_void_p(d_op_offsets), ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise GsnapdpError("gsnapdp_ggap_run_device: %s" % lib().gsnapdp_last_error().decode())

    def ggap_all_pairs(self, windows, query, query_uc, results, traces, ops, off):
        """The lists Dynprog_genome_gap returns, concatenated, and their lengths."""
        w = np.ascontiguousarray(windows, dtype=GGAP_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        res = np.ascontiguousarray(results, dtype=GGAP_RESULT)
        trc = np.ascontiguousarray(traces, dtype=GGAP_TRACE)
        outs, counts = [], np.zeros(len(w), dtype=np.int32)
        for i in range(len(w)):
            cap = 2 * int(w["length1"][i]) + int(w["length2L"][i]) + int(w["length2R"][i]) + 8
            out = np.zeros(cap, dtype=PAIR)
            n = lib().gsnapdp_ggap_expand(self.h, _p(w[i:i + 1]), _p(res[i:i + 1]), _p(trc[i:i + 1]),
                                          _p(ops[off[i]:]), _p(q), _p(u), _p(out), cap)
            if n < 0:
                raise GsnapdpError("gsnapdp_ggap_expand failed for window %d" % i)
            outs.append(out[:n])
            counts[i] = n
        return (np.concatenate(outs) if outs else np.zeros(0, PAIR)), counts

    def cgap_run(self, windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
        """Dynprog_cdna_gap on the GPU.  Returns (results, ops, op_offsets)."""
        w = np.ascontiguousarray(windows, dtype=CGAP_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        off = cgap_op_offsets(w)
        res = np.zeros(len(w), dtype=CGAP_RESULT)
        ops = np.zeros(max(1, int(off[-1])), dtype=np.uint32)
        rc = lib().gsnapdp_cgap_run_host(self.h, _p(w), len(w), _p(q), _p(u), q.size, _p(res), _p(ops), _p(off))
        if rc != 0:
            raise GsnapdpError("gsnapdp_cgap_run_host: %s" % lib().gsnapdp_last_error().decode())
        return res, ops, off

    def cgap_all_pairs(self, windows, query, query_uc, results, ops, off, gseg=None, gseg_off=None):
        """The lists Dynprog_cdna_gap returns, concatenated, and their lengths."""
        w = np.ascontiguousarray(windows, dtype=CGAP_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        res = np.ascontiguousarray(results, dtype=CGAP_RESULT)
        gs = None if gseg is None else np.ascontiguousarray(gseg, dtype=np.uint8)
        outs, counts = [], np.zeros(len(w), dtype=np.int32)
        for i in range(len(w)):
            cap = int(w["length1L"][i]) + int(w["length1R"][i]) + 2 * int(w["length2"][i]) + 32
            out = np.zeros(max(cap, 1), dtype=PAIR)
            s2 = None if gs is None else ctypes.c_void_p(gs.ctypes.data + int(gseg_off[i]))
            n = lib().gsnapdp_cgap_expand(self.h, _p(w[i:i + 1]), _p(res[i:i + 1]), _p(ops[off[i]:]),
                                          _p(q), _p(u), s2, _p(out), out.size)
            if n < 0:
                raise GsnapdpError("gsnapdp_cgap_expand failed for window %d" % i)
            outs.append(out[:n])
            counts[i] = n
        return (np.concatenate(outs) if outs else np.zeros(0, PAIR)), counts

    def sj_run(self, windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
        """Dynprog_end5/3_splicejunction on the GPU.  Returns (results, ops, op_offsets)."""
        w = np.ascontiguousarray(windows, dtype=SJ_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        off = op_offsets(w)
        res = np.zeros(len(w), dtype=RESULT)
        ops = np.zeros(max(1, int(off[-1])), dtype=np.uint32)
        rc = lib().gsnapdp_sj_run_host(self.h, _p(w), len(w), _p(q), _p(u), q.size, _p(res), _p(ops), _p(off))
        if rc != 0:
            raise GsnapdpError("gsnapdp_sj_run_host: %s" % lib().gsnapdp_last_error().decode())
        return res, ops, off

    def sj_run_device(self, d_windows: int, n: int, d_query: int, d_query_uc: int, d_results: int, d_ops: int,
                      d_op_offsets: int, stream: int = 0) -> None:
        rc = lib().gsnapdp_sj_run_device(self.h, ctypes.c_void_p(d_windows), n, ctypes.c_void_p(d_query),
                                         ctypes.c_void_p(d_query_uc), ctypes.c_void_p(d_results),
                                         ctypes.c_void_p(d_ops), ctypes.c_void_p(d_op_offsets),
                                         ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise GsnapdpError("gsnapdp_sj_run_device: %s" % lib().gsnapdp_last_error().decode())

    def micro_run_device(self, d_windows: int, n: int, d_query: int, d_query_uc: int, d_results: int,
                         stream: int = 0) -> None:
        rc = lib().gsnapdp_micro_run_device(self.h, ctypes.c_void_p(d_windows), n, ctypes.c_void_p(d_query),
                                            ctypes.c_void_p(d_query_uc), ctypes.c_void_p(d_results),
                                            ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise GsnapdpError("gsnapdp_micro_run_device: %s" % lib().gsnapdp_last_error().decode())

    def sj_all_pairs(self, windows, query, query_uc, results, ops, off):
        """The lists Dynprog_end5/3_splicejunction return, concatenated, and their lengths."""
        w = np.ascontiguousarray(windows, dtype=SJ_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        res = np.ascontiguousarray(results, dtype=RESULT)
        outs, counts = [], np.zeros(len(w), dtype=np.int32)
        for i in range(len(w)):
            cap = int(w["length1"][i]) + int(w["length2"][i]) + 8
            out = np.zeros(max(cap, 1), dtype=PAIR)
            n = lib().gsnapdp_sj_expand(self.h, _p(w[i:i + 1]), _p(res[i:i + 1]), _p(ops[off[i]:]),
                                        _p(q), _p(u), _p(out), out.size)
            if n < 0:
                raise GsnapdpError("gsnapdp_sj_expand failed for window %d" % i)
            outs.append(out[:n])
            counts[i] = n
        return (np.concatenate(outs) if outs else np.zeros(0, PAIR)), counts

    def micro_run(self, windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray) -> np.ndarray:
        """Dynprog_microexon_int on the GPU.  Returns the MICRO_RESULT records."""
        w = np.ascontiguousarray(windows, dtype=MICRO_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        res = np.zeros(len(w), dtype=MICRO_RESULT)
        rc = lib().gsnapdp_micro_run_host(self.h, _p(w), len(w), _p(q), _p(u), q.size, _p(res))
        if rc != 0:
            raise GsnapdpError("gsnapdp_micro_run_host: %s" % lib().gsnapdp_last_error().decode())
        return res

    def micro_all_pairs(self, windows, query, query_uc, results):
        """The lists Dynprog_microexon_int returns, concatenated, and their lengths."""
        w = np.ascontiguousarray(windows, dtype=MICRO_WINDOW)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        u = np.ascontiguousarray(query_uc, dtype=np.uint8)
        res = np.ascontiguousarray(results, dtype=MICRO_RESULT)
        outs, counts = [], np.zeros(len(w), dtype=np.int32)
        for i in range(len(w)):
            out = np.zeros(int(w["length1"][i]) + 4, dtype=PAIR)
            n = lib().gsnapdp_micro_expand(self.h, _p(w[i:i + 1]), _p(res[i:i + 1]), _p(q), _p(u), _p(out),
                                           out.size)
            if n < 0:
                raise GsnapdpError("gsnapdp_micro_expand failed for window %d" % i)
            outs.append(out[:n])
            counts[i] = n
        return (np.concatenate(outs) if outs else np.zeros(0, PAIR)), counts

    def run_device(self, d_windows: int, n: int, d_query: int, d_query_uc: int, d_results: int,
                   d_ops: int, d_op_offsets: int, stream: int = 0) -> None:
        """Device-resident batch (raw device pointers, e.g. torch tensor.data_ptr())."""
        rc = lib().gsnapdp_run_device(self.h, ctypes.c_void_p(d_windows), n, ctypes.c_void_p(d_query),
                                      ctypes.c_void_p(d_query_uc), ctypes.c_void_p(d_results),
                                      ctypes.c_void_p(d_ops), ctypes.c_void_p(d_op_offsets),
                                      ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise GsnapdpError("gsnapdp_run_device: %s" % lib().gsnapdp_last_error().decode())

    def compact_ops_device(self, d_results: int, n: int, d_ops: int, d_op_offsets: int, d_out: int,
                           out_cap: int, d_header: int, stream: int = 0) -> None:
        """Op streams of a finished batch, packed in window order (gsnapdp_compact_ops_device);
        d_header (2 x int64) receives {total ops, overflow}."""
        rc = lib().gsnapdp_compact_ops_device(self.h, ctypes.c_void_p(d_results), n, ctypes.c_void_p(d_ops),
                                              ctypes.c_void_p(d_op_offsets), ctypes.c_void_p(d_out), out_cap,
                                              ctypes.c_void_p(d_header),
                                              ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise GsnapdpError("gsnapdp_compact_ops_device: %s" % lib().gsnapdp_last_error().decode())

    def profile(self, enable: bool) -> list:
        """Enable per-kernel HIP-event timing; returns the stage names."""
        n = lib().gsnapdp_profile(self.h, 1 if enable else 0)
        return [lib().gsnapdp_stage_name(i).decode() for i in range(n)]

    def profile_read(self, acc: np.ndarray) -> None:
        """Add the last run's per-stage milliseconds into acc (float64)."""
        if lib().gsnapdp_profile_read(self.h, _p(acc), acc.size) < 0:
            raise GsnapdpError(lib().gsnapdp_last_error().decode())

    def sync(self):
        if lib().gsnapdp_sync(self.h) != 0:
            raise GsnapdpError(lib().gsnapdp_last_error().decode())

    def score_introns(self, paths: np.ndarray, introns: np.ndarray) -> np.ndarray:
        """score_introns (stage3.c:7935-8162) for every path in one k_introns launch."""
        pa = np.ascontiguousarray(paths, dtype=INTRON_PATH)
        it = np.ascontiguousarray(introns, dtype=INTRON)
        out = np.zeros(len(pa), dtype=INTRON_SCORES)
        rc = lib().gsnapdp_score_introns_host(self.h, _p(pa), len(pa), _p(it) if it.size else None, len(it),
                                              _p(out))
        if rc != 0:
            raise GsnapdpError("gsnapdp_score_introns_host: %s" % lib().gsnapdp_last_error().decode())
        return out

    @staticmethod
    def stage3_capacity(calls: np.ndarray) -> int:
        """pairs_out capacity that always suffices for these calls"""
        return int((2 * (calls["querylength"].astype(np.int64) + calls["npairs"]) + 64).sum()) if len(calls) else 1

    def stage3_pass(self, calls: np.ndarray, pairs_in: np.ndarray, query: np.ndarray, query_uc: np.ndarray,
                    out: np.ndarray = None, iit: "SplicingIIT" = None):
        """build_pairs_introns (stage3.c:7735-7901) over every call's path at once
        (gsnapdp_stage3_pass).  Returns (calls with the out fields written, the
        returned lists concatenated, S3_STATS).  `out`: a reusable S3_PAIR buffer
        of stage3_capacity(calls) pairs; `iit`: the splicing IIT (SplicingIIT) or None."""
        c = np.array(calls, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = self.stage3_capacity(c)
        if out is None or out.dtype != S3_PAIR or out.size < cap:
            out = np.empty(max(cap, 1), dtype=S3_PAIR)  # only the lists written are touched
        st = np.zeros(1, dtype=S3_STATS)
        rc = lib().gsnapdp_stage3_pass(self.h, _p(c), len(c), _p(pi) if pi.size else _p(out), pi.size, _p(q),
                                       _p(qu), min(q.size, qu.size), iit.h if iit is not None else None, _p(out),
                                       cap, _p(st))
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_pass: %s" % lib().gsnapdp_last_error().decode())
        n = int(c["nout"].sum())
        return c, out[:n], st[0]

    def stage3_pass_compact(self, calls: np.ndarray, pairs_in: np.ndarray, query: np.ndarray,
                            query_uc: np.ndarray, iit: "SplicingIIT" = None, bufs=None):
        """gsnapdp_stage3_pass_compact: (calls, cells, new pairs, S3_STATS); a cell is
        the input pair's index (| S3_CELL_DISALLOWED) or -1 - k for new[k]
        (expand_compact rebuilds the lists).  `bufs`: reusable (cells, new) arrays."""
        c = np.array(calls, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = self.stage3_capacity(c)
        ncap = int((2 * c["querylength"].astype(np.int64) + 256).sum()) if len(c) else 1
        if bufs is None or bufs[0].size < cap or bufs[1].size < ncap:
            bufs = (np.empty(max(cap, 1), dtype=np.int32), np.empty(max(ncap, 1), dtype=S3_PAIR))
        st = np.zeros(1, dtype=S3_STATS)
        rc = lib().gsnapdp_stage3_pass_compact(self.h, _p(c), len(c), _p(pi) if pi.size else _p(bufs[1]), pi.size,
                                               _p(q), _p(qu), min(q.size, qu.size),
                                               iit.h if iit is not None else None, _p(bufs[0]), bufs[0].size,
                                               _p(bufs[1]), bufs[1].size, _p(st))
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_pass_compact: %s" % lib().gsnapdp_last_error().decode())
        return c, bufs[0][:int(c["nout"].sum())], bufs[1][:int(st[0]["new_pairs"])], st[0]

    def stage3_pass_runs(self, calls: np.ndarray, pairs_in: np.ndarray, query: np.ndarray, query_uc: np.ndarray,
                         gaps: np.ndarray = None, gap_off: np.ndarray = None, iit: "SplicingIIT" = None, bufs=None):
        """gsnapdp_stage3_pass_runs: (calls, runs, new pairs, S3_STATS, bufs); call
        i's list is runs[first_out : first_out + nout] (S3_RUN: input pairs start,
        start - 1, .. or new[-1 - start ..]; expand_runs rebuilds the lists).
        `gaps` / `gap_off` as gap_lists makes them (None: the pass finds them).
        `bufs`: reusable (runs, new) arrays; the returned bufs may be larger."""
        from .records import S3_RUN
        c = np.array(calls, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        g = go = None
        if gaps is not None:
            g = np.ascontiguousarray(gaps, dtype=np.int32)
            go = np.ascontiguousarray(gap_off, dtype=np.int64)
        cap = 8 * (len(g) if g is not None else 0) + 16 * len(c) + 1024
        ncap = int((2 * c["querylength"].astype(np.int64) + 256).sum()) if len(c) else 1
        if bufs is None or bufs[0].size < cap or bufs[1].size < ncap:
            bufs = (np.empty(max(cap, 1 if bufs is None else bufs[0].size), dtype=S3_RUN),
                    np.empty(max(ncap, 1), dtype=S3_PAIR))
        for attempt in range(2):
            c = np.array(calls, dtype=S3_CALL, copy=True)
            st = np.zeros(1, dtype=S3_STATS)
            rc = lib().gsnapdp_stage3_pass_runs(self.h, _p(c), len(c), _p(pi) if pi.size else _p(bufs[1]), pi.size,
                                                _p(g) if g is not None and g.size else (_p(go) if g is not None else None),
                                                _p(go) if go is not None else None, _p(q), _p(qu),
                                                min(q.size, qu.size), iit.h if iit is not None else None,
                                                _p(bufs[0]), bufs[0].size, _p(bufs[1]), bufs[1].size, _p(st))
            need, nnew = int(st[0]["out_needed"]), int(st[0]["new_pairs"])
            if rc != 0 and attempt == 0 and (need > bufs[0].size or nnew > bufs[1].size):
                # the runs or the new-pair output was too small: once more, both grown to what was asked
                bufs = (bufs[0] if need <= bufs[0].size else np.empty(need + 1024, dtype=S3_RUN),
                        bufs[1] if nnew <= bufs[1].size else np.empty(nnew + 1024, dtype=S3_PAIR))
                continue
            break
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_pass_runs: %s" % lib().gsnapdp_last_error().decode())
        return c, bufs[0][:int(c["nout"].sum())], bufs[1][:int(st[0]["new_pairs"])], st[0], bufs

    def stage3_score_introns_runs(self, calls: np.ndarray, pairs_in: np.ndarray, runs: np.ndarray, new: np.ndarray,
                                  gaps: np.ndarray = None, gap_off: np.ndarray = None, iit: "SplicingIIT" = None):
        """score_introns on stage3_pass_runs' output (gsnapdp_stage3_score_introns_runs)"""
        from .records import S3_RUN
        c = np.ascontiguousarray(calls, dtype=S3_CALL)
        pi = np.ascontiguousarray(pairs_in, dtype=S3_PAIR)
        r = np.ascontiguousarray(runs, dtype=S3_RUN)
        nw = np.ascontiguousarray(new, dtype=S3_PAIR)
        g = go = None
        if gaps is not None:
            g = np.ascontiguousarray(gaps, dtype=np.int32)
            go = np.ascontiguousarray(gap_off, dtype=np.int64)
        out = np.zeros(len(c), dtype=INTRON_SCORES)
        rc = lib().gsnapdp_stage3_score_introns_runs(
            self.h, _p(c), len(c), _p(pi) if pi.size else None,
            (_p(g) if g.size else _p(go)) if g is not None else None, _p(go) if go is not None else None,
            _p(r) if r.size else _p(out), _p(nw) if nw.size else None, iit.h if iit is not None else None, _p(out))
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_score_introns_runs: %s" % lib().gsnapdp_last_error().decode())
        return out

    def stage3_compute(self, queries: np.ndarray, paths_in: np.ndarray, query: np.ndarray, query_uc: np.ndarray,
                       iit: "SplicingIIT" = None, min_intronlength: int = 9, out: np.ndarray = None):
        """Passes 2A-6 of path_compute (stage3.c:8639-8876) for every query
        (gsnapdp_stage3_compute).  Returns (queries with the out fields written,
        the lists after pass 6 concatenated, S3_COMPUTE_STATS)."""
        from .records import S3_COMPUTE_STATS
        c = np.array(queries, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(paths_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = 2 * self.stage3_capacity(c) + 1024
        if out is None or out.dtype != S3_PAIR or out.size < cap:
            out = np.empty(cap, dtype=S3_PAIR)
        st = np.zeros(1, dtype=S3_COMPUTE_STATS)
        rc = lib().gsnapdp_stage3_compute(self.h, _p(c), len(c), _p(pi) if pi.size else _p(out), pi.size, _p(q),
                                          _p(qu), min(q.size, qu.size), iit.h if iit is not None else None,
                                          int(min_intronlength), _p(out), out.size, _p(st))
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_compute: %s" % lib().gsnapdp_last_error().decode())
        return c, out[:int(c["nout"].sum())], st[0]

    def stage3_path_compute(self, queries: np.ndarray, paths_in: np.ndarray, query: np.ndarray,
                            query_uc: np.ndarray, iit: "SplicingIIT" = None, min_intronlength: int = 9,
                            maxintronlen_bound: int = 1000000, gsnap: bool = False, out: np.ndarray = None):
        """path_compute (stage3.c:8586-9220) from pass 2A to its return value
        for every query (gsnapdp_stage3_path_compute; GMAP's paired_favor_mode 0).
        Returns (queries with the out fields written, the returned lists
        concatenated, their pairs' (donor_prob, acceptor_prob) as an (n, 2)
        array, S3_COMPUTE_STATS)."""
        from .records import S3_COMPUTE_STATS, S3_PATH_OPTS
        c = np.array(queries, dtype=S3_CALL, copy=True)
        pi = np.ascontiguousarray(paths_in, dtype=S3_PAIR)
        q = np.ascontiguousarray(query, dtype=np.uint8)
        qu = np.ascontiguousarray(query_uc, dtype=np.uint8)
        cap = 2 * self.stage3_capacity(c) + 1024
        if out is None or out.dtype != S3_PAIR or out.size < cap:
            out = np.empty(cap, dtype=S3_PAIR)
        probs = np.empty((out.size, 2), dtype=np.float64)
        o = np.zeros(1, dtype=S3_PATH_OPTS)
        o["min_intronlength"], o["maxintronlen_bound"] = min_intronlength, maxintronlen_bound
        o["gsnap"] = 1 if gsnap else 0
        st = np.zeros(1, dtype=S3_COMPUTE_STATS)
        rc = lib().gsnapdp_stage3_path_compute(self.h, _p(c), len(c), _p(pi) if pi.size else _p(out), pi.size,
                                               _p(q), _p(qu), min(q.size, qu.size),
                                               iit.h if iit is not None else None, _p(o), _p(out), out.size,
                                               _p(probs), _p(st))
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_path_compute: %s" % lib().gsnapdp_last_error().decode())
        n = int(c["nout"].sum())
        return c, out[:n], probs[:n], st[0]

    def scan_site_probs(self, sites: np.ndarray) -> np.ndarray:
        """GSNAP's splice-site scan candidates (SCAN_SITE records) in one batch
        (gsnapdp_scan_site_probs): 1.0 for a known site, else the MaxEnt
        probability at segment_left + splice_pos."""
        from .records import SCAN_SITE
        s = np.ascontiguousarray(sites, dtype=SCAN_SITE)
        out = np.zeros(s.size, dtype=np.float64)
        if lib().gsnapdp_scan_site_probs(self.h, _p(s) if s.size else None, s.size, _p(out)) != 0:
            raise GsnapdpError("gsnapdp_scan_site_probs: %s" % lib().gsnapdp_last_error().decode())
        return out

    def set_stage2(self, compute_one: int, user: int):
        """traverse_dual_break's stage-2 realignment (gsnapdp_stage3_set_stage2):
        `compute_one` the address of a C callback with gsnapdp_s3_stage2's
        signature, `user` its first argument; 0, 0 clears it."""
        self._stage2 = (ctypes.c_void_p * 2)(user or None, compute_one or None)
        if lib().gsnapdp_stage3_set_stage2(self.h, ctypes.addressof(self._stage2)) != 0:
            raise GsnapdpError("gsnapdp_stage3_set_stage2: %s" % lib().gsnapdp_last_error().decode())

    def stage3_score_introns(self, calls: np.ndarray, pairs_out: np.ndarray, iit: "SplicingIIT" = None):
        """score_introns (stage3.c:7935-8162) on the lists stage3_pass returned
        (gsnapdp_stage3_score_introns): one INTRON_SCORES per call."""
        c = np.ascontiguousarray(calls, dtype=S3_CALL)
        po = np.ascontiguousarray(pairs_out, dtype=S3_PAIR)
        out = np.zeros(len(c), dtype=INTRON_SCORES)
        rc = lib().gsnapdp_stage3_score_introns(self.h, _p(c), len(c), _p(po) if po.size else None,
                                                iit.h if iit is not None else None, _p(out))
        if rc != 0:
            raise GsnapdpError("gsnapdp_stage3_score_introns: %s" % lib().gsnapdp_last_error().decode())
        return out

    def maxent(self, model: np.ndarray, pos: np.ndarray, chroffset: np.ndarray) -> np.ndarray:
        m = np.ascontiguousarray(model, dtype=np.uint8)
        p = np.ascontiguousarray(pos, dtype=np.uint32)
        c = np.ascontiguousarray(chroffset, dtype=np.uint32)
        out = np.zeros(m.size, dtype=np.float64)
        if lib().gsnapdp_maxent_host(self.h, _p(m), _p(p), _p(c), _p(out), m.size) != 0:
            raise GsnapdpError("maxent: %s" % lib().gsnapdp_last_error().decode())
        return out

    def maxent_device(self, d_model: int, d_pos: int, d_chroff: int, d_out: int, n: int, stream: int = 0):
        rc = lib().gsnapdp_maxent_device(self.h, ctypes.c_void_p(d_model), ctypes.c_void_p(d_pos),
                                         ctypes.c_void_p(d_chroff), ctypes.c_void_p(d_out), n,
                                         ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise GsnapdpError("maxent_device: %s" % lib().gsnapdp_last_error().decode())


def expand_compact(calls: np.ndarray, pairs_in: np.ndarray, cells: np.ndarray, new: np.ndarray) -> np.ndarray:
    """The full returned lists (as Context.stage3_pass writes them) from a compact
    pass's cells: input pairs with src set (and DISALLOWED where the cell says),
    new pairs as made."""
    from .records import S3_CELL_DISALLOWED
    out = np.empty(cells.size, dtype=S3_PAIR)
    owner = np.repeat(np.arange(len(calls)), calls["nout"])
    kept = cells >= 0
    src = (cells & (S3_CELL_DISALLOWED - 1))[kept]
    x = pairs_in[calls["first_pair"][owner[kept]] + src].copy()
    x["src"] = src
    x["flags"] |= np.where((cells[kept] & S3_CELL_DISALLOWED) != 0, S3_DISALLOWED, 0).astype(np.uint8)
    out[kept] = x
    out[~kept] = new[-1 - cells[~kept]]
    return out


def gap_lists(calls: np.ndarray, pairs_in: np.ndarray):
    """(gaps, gap_off) for gsnapdp_stage3_pass_runs: each call's GAPP pairs, as
    indices within its path, ascending."""
    gp = np.flatnonzero((pairs_in["flags"] & S3_GAPP) != 0)
    first = calls["first_pair"].astype(np.int64)
    lo = np.searchsorted(gp, first)
    hi = np.searchsorted(gp, first + calls["npairs"])
    cnt = hi - lo
    gap_off = np.zeros(len(calls) + 1, dtype=np.int64)
    np.cumsum(cnt, out=gap_off[1:])
    owner = np.repeat(np.arange(len(calls)), cnt)
    idx = np.repeat(lo - gap_off[:-1], cnt) + np.arange(int(gap_off[-1]))
    gaps = (gp[idx] - first[owner]).astype(np.int32)
    return gaps, gap_off


def expand_runs(calls: np.ndarray, pairs_in: np.ndarray, runs: np.ndarray, new: np.ndarray):
    """The full returned lists (as Context.stage3_pass writes them) from
    stage3_pass_runs' runs, and the calls with first_out / nout in pairs."""
    from .records import S3_CELL_DISALLOWED
    cnt = (runs["count"] & (S3_CELL_DISALLOWED - 1)).astype(np.int64)
    owner = np.repeat(np.arange(len(calls)), calls["nout"])
    k = np.repeat(np.arange(runs.size), cnt)  # the run of each pair
    off = np.arange(k.size) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    st = runs["start"].astype(np.int64)[k]
    out = np.empty(k.size, dtype=S3_PAIR)
    inp = st >= 0
    src = (st - off)[inp]
    x = pairs_in[calls["first_pair"].astype(np.int64)[owner[k[inp]]] + src].copy()
    x["src"] = src
    x["flags"] |= np.where((runs["count"][k[inp]] & S3_CELL_DISALLOWED) != 0, S3_DISALLOWED, 0).astype(np.uint8)
    out[inp] = x
    out[~inp] = new[(-1 - st + off)[~inp]]
    c = np.array(calls, copy=True)
    per = np.bincount(owner, weights=cnt, minlength=len(calls)).astype(np.int64) if runs.size else \
        np.zeros(len(calls), np.int64)
    c["nout"] = per
    c["first_out"] = np.concatenate([[0], np.cumsum(per)[:-1]]) if len(calls) else per
    return c, out
