"""Result payloads of the multi-GPU path.

One read batch is split across ranks (``shard.balanced_ranges``); each rank
aligns its slice and hands the root rank ONE payload buffer: the result
records of its windows plus their op streams in compact form
(``gsnapdp_compact_ops_device``: window i's ``nops`` words, windows in batch
order).  Nothing else leaves a GPU -- no direction bands, no capacity-sized
op buffers.  The root gathers the payloads with one RCCL collective
(``shard.gather_to_root``) and rebuilds every window's op offset from the
``nops`` column alone.

Payload layout (bytes, every rank's buffer has the same size so one
``gather`` moves them all):

    [0, 16)                 int64 header {total ops, overflow}
    [16, 16 + 48 * cap_n)   gsnapdp_result records, window order
    [.., + 4 * budget)      compact op stream (uint32)

``cap_n`` is the largest shard and ``budget`` the op words reserved per
payload.  The header's overflow flag (total > budget) is checked after the
run; a payload that overflowed is an error, never silently truncated.
"""
from __future__ import annotations

import numpy as np

from .records import RESULT

HEADER = 16


class Layout:
    def __init__(self, cap_n: int, budget_words: int):
        self.cap_n = int(cap_n)
        self.budget = int(budget_words)
        self.res_off = HEADER
        self.ops_off = HEADER + RESULT.itemsize * self.cap_n
        self.nbytes = (self.ops_off + 4 * self.budget + 255) & ~255


def op_budget(cap_n: int, per_window: int = 4) -> int:
    """Op words reserved per payload: `per_window` on average (a C2/C3 window
    emits 1 op, 3 with one indel; the header's overflow flag guards the rest)."""
    return max(1024, int(cap_n) * per_window)


def compact_ops(results: np.ndarray, ops: np.ndarray, off: np.ndarray) -> np.ndarray:
    """Host mirror of gsnapdp_compact_ops_device (window i's
    min(nops, capacity) words, windows in order)."""
    cap = np.diff(off)
    cnt = np.minimum(np.maximum(results["nops"].astype(np.int64), 0), cap)
    idx = np.repeat(off[:-1], cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    return ops[idx].astype(np.uint32)


def pack(layout: Layout, results: np.ndarray, compact: np.ndarray) -> np.ndarray:
    """Host-built payload (the CPU test path builds what the GPU path writes)."""
    buf = np.zeros(layout.nbytes, dtype=np.uint8)
    total = compact.size
    hdr = np.array([total, 1 if total > layout.budget else 0], dtype=np.int64)
    buf[:HEADER] = hdr.view(np.uint8)
    rb = np.ascontiguousarray(results, dtype=RESULT).view(np.uint8)
    buf[layout.res_off:layout.res_off + rb.size] = rb
    k = min(total, layout.budget)
    buf[layout.ops_off:layout.ops_off + 4 * k] = compact[:k].view(np.uint8)
    return buf


def unpack(layout: Layout, buf: np.ndarray, n: int):
    """(results[n], compact ops, op offsets[n+1]) of one rank's payload."""
    buf = np.asarray(buf, dtype=np.uint8)
    total, overflow = (int(x) for x in buf[:HEADER].view(np.int64))
    if overflow or total > layout.budget:
        raise RuntimeError("payload op budget overflow: %d ops > %d reserved" % (total, layout.budget))
    res = buf[layout.res_off:layout.res_off + RESULT.itemsize * n].view(RESULT).copy()
    ops = buf[layout.ops_off:layout.ops_off + 4 * total].view(np.uint32).copy()
    off = offsets_from_nops(res)
    if int(off[-1]) != total:
        raise RuntimeError("payload inconsistent: sum(nops) %d != header %d" % (int(off[-1]), total))
    return res, ops, off


def offsets_from_nops(results: np.ndarray) -> np.ndarray:
    off = np.zeros(len(results) + 1, dtype=np.int64)
    np.cumsum(np.maximum(results["nops"].astype(np.int64), 0), out=off[1:])
    return off


def reassemble(layout: Layout, bufs, sizes):
    """The whole batch's (results, compact ops, offsets) from the gathered
    payloads, in rank order (= batch order for contiguous shards)."""
    parts = [unpack(layout, b, n) for b, n in zip(bufs, sizes)]
    res = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, RESULT)
    ops = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, np.uint32)
    return res, ops, offsets_from_nops(res)
