"""Synthetic workloads.

* ``synthetic_genome``: uniform ACGT with 0.1 % N in runs of 1-10 (seed 1).
* ``c2_windows``: the BASELINE config-2 batch -- 150 bp reads taken from the
  genome (either strand), 2 % substitutions, 0.1 % N, 30 % with one 1-3 bp
  indel, aligned with Dynprog_single_gap, extraband_single 15 (band 31),
  widebandp, defect_rate 0.001, jump_late_p = !watsonp (stage1hr.c:11288).
* ``random_windows``: broad parity mix over every window kind, strand,
  tie rule, quality bin, band, lowercase / ambiguity codes and chromosome
  edges ('*' columns).

Deterministic for a given seed (numpy PCG64).
"""
from __future__ import annotations

import numpy as np

from . import genome as _genome
from .records import (BEST_LOCAL, END3_GAP, END5_GAP, MAXLENGTH1, MAXLENGTH2, QUERYEND_GAP,
                      QUERYEND_INDELS, QUERYEND_NOGAPS, SINGLE_GAP, WINDOW)

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.arange(256, dtype=np.uint8)
for _a, _b in (("A", "T"), ("C", "G"), ("G", "C"), ("T", "A"), ("N", "N")):
    _COMP[ord(_a)] = ord(_b)
    _COMP[ord(_a.lower())] = ord(_b.lower())


def revcomp(s: np.ndarray) -> np.ndarray:
    return _COMP[s[::-1]]


def synthetic_genome(nbases: int, seed: int = 1, n_rate: float = 0.001) -> np.ndarray:
    """Uniform ACGT with ~n_rate N bases in runs of 1-10."""
    rng = np.random.default_rng(seed)
    g = ACGT[rng.integers(0, 4, size=nbases)]
    nruns = int(nbases * n_rate / 5.5)
    if nruns:
        starts = rng.integers(0, nbases, size=nruns)
        lens = rng.integers(1, 11, size=nruns)
        for s, l in zip(starts.tolist(), lens.tolist()):
            g[s:s + l] = ord("N")
    return g


class Batch:
    """A batch of windows plus the query buffers they address."""

    def __init__(self, windows: np.ndarray, query: np.ndarray, query_uc: np.ndarray):
        self.windows = windows
        self.query = query
        self.query_uc = query_uc

    def __len__(self) -> int:
        return len(self.windows)


def _mutate(rng, q: np.ndarray, sub_rate: float, n_rate: float) -> np.ndarray:
    q = q.copy()
    m = rng.random(q.size)
    subs = m < sub_rate
    if subs.any():
        q[subs] = ACGT[(np.searchsorted(ACGT, q[subs]) + rng.integers(1, 4, size=int(subs.sum()))) % 4]
    ns = (m >= sub_rate) & (m < sub_rate + n_rate)
    q[ns] = ord("N")
    return q


def c2_windows(gseq: np.ndarray, n: int = 100_000, seed: int = 2, read_len: int = 150,
               extraband: int = 15, indel_frac: float = 0.3, sub_rate: float = 0.02,
               n_rate: float = 0.001, margin: int = 8) -> Batch:
    """BASELINE config 2: single-gap windows of 150 bp reads against the genome."""
    rng = np.random.default_rng(seed)
    G = gseq.size
    w = np.zeros(n, dtype=WINDOW)
    qbuf = np.full(n * (read_len + 8), ord("#"), dtype=np.uint8)
    qpos = 0
    has_indel = rng.random(n) < indel_frac
    indel_len = rng.integers(1, 4, size=n)
    indel_sign = rng.integers(0, 2, size=n) * 2 - 1  # +1: genome longer (deletion in read)
    watson = rng.integers(0, 2, size=n).astype(bool)
    starts = rng.integers(margin, G - read_len - 16 - margin, size=n)
    for i in range(n):
        L2 = read_len + (int(indel_sign[i] * indel_len[i]) if has_indel[i] else 0)
        seg_start = int(starts[i]) - margin
        seglen = L2 + 2 * margin
        seg = gseq[seg_start:seg_start + seglen]
        gwin = seg[margin:margin + L2] if watson[i] else revcomp(seg)[margin:margin + L2]
        if L2 > read_len:  # genome has extra bases: delete them from the read
            k = L2 - read_len
            p = int(rng.integers(10, read_len - 10))
            q = np.concatenate([gwin[:p], gwin[p + k:]])
        elif L2 < read_len:  # read has extra bases
            k = read_len - L2
            p = int(rng.integers(10, L2 - 10))
            q = np.concatenate([gwin[:p], ACGT[rng.integers(0, 4, size=k)], gwin[p:]])
        else:
            q = gwin.copy()
        q = _mutate(rng, q, sub_rate, n_rate)
        qbuf[qpos:qpos + read_len] = q
        w[i]["qpos"] = qpos
        qpos += read_len + 8
        w[i]["length2"] = L2
        w[i]["chrpos"] = seg_start
        w[i]["genomiclength"] = seglen
        w[i]["watsonp"] = 1 if watson[i] else 0
    w["kind"] = SINGLE_GAP
    w["length1"] = read_len
    w["offset1"] = 0
    w["offset2"] = margin
    w["chroffset"] = 0
    w["chrhigh"] = G
    w["cdna_direction"] = 1
    w["extraband"] = extraband
    w["dynprogindex"] = 1
    w["maxlength1"] = MAXLENGTH1
    w["maxlength2"] = MAXLENGTH2
    w["defect_rate"] = 0.001
    w["jump_late_p"] = 1 - w["watsonp"]
    w["widebandp"] = 1
    qbuf = qbuf[:qpos]
    return Batch(w, qbuf, qbuf.copy())


_AMBIG = np.frombuffer(b"RYWSMKHBVDNXU", dtype=np.uint8)


def random_windows(gseq: np.ndarray, n: int, seed: int, kinds=(SINGLE_GAP, END5_GAP, END3_GAP),
                   max_len1: int = 60, max_len2: int = 70, chroms: int = 4,
                   allow_weird_chars: bool = True, endaligns=(QUERYEND_GAP, QUERYEND_INDELS,
                                                              QUERYEND_NOGAPS, BEST_LOCAL),
                   max_band: int = 12) -> Batch:
    """Broad parity mix.  The genome is split into `chroms` chromosomes so
    windows near chromosome ends produce '*' columns (dynprog.c:409-419)."""
    rng = np.random.default_rng(seed)
    G = gseq.size
    bounds = np.linspace(0, G, chroms + 1).astype(np.int64)
    w = np.zeros(n, dtype=WINDOW)
    qchunks, uchunks = [], []
    qpos = 0
    for i in range(n):
        kind = int(kinds[rng.integers(0, len(kinds))])
        L1 = int(rng.integers(1, max_len1 + 1))
        L2 = int(max(1, L1 + rng.integers(-8, 9))) if rng.random() < 0.7 else int(rng.integers(1, max_len2 + 1))
        ci = int(rng.integers(0, chroms))
        chroffset, chrhigh = int(bounds[ci]), int(bounds[ci + 1])
        chrlen = chrhigh - chroffset
        genomiclength = L2 + int(rng.integers(0, 20))

        # chrpos mostly inside; sometimes the segment hangs past the chromosome
        # end (into the next chromosome, still inside the genome) or starts at
        # or past chrhigh (every column '*').  get_genomic_nt only tests
        # chroffset+chrpos against chrhigh (dynprog.c:415-419).
        if rng.random() < 0.1:
            chrpos = int(rng.integers(max(0, chrlen - genomiclength), chrlen + 5))
            if chrpos < chrlen and chroffset + chrpos + genomiclength > G:
                chrpos = chrlen
        else:
            chrpos = int(rng.integers(0, max(1, chrlen - genomiclength)))
        watson = int(rng.integers(0, 2))
        off2_max = max(0, genomiclength - L2)
        offset2 = int(rng.integers(0, off2_max + 1))
        if kind == END5_GAP:
            offset2 = offset2 + L2 - 1  # revoffset2: last genome column
        # genome segment as seen through get_genomic_nt
        gpos = np.arange(genomiclength)
        absp = chroffset + chrpos + (gpos if watson else genomiclength - 1 - gpos)
        valid = (chroffset + chrpos < chrhigh) & (absp < G)
        seg = np.full(genomiclength, ord("A"), dtype=np.uint8)
        seg[valid] = gseq[absp[valid]]
        if not watson:
            seg = _COMP[seg]
        if kind == END5_GAP:
            core = seg[max(0, offset2 - L1 + 1):offset2 + 1]
        else:
            core = seg[offset2:offset2 + L1]
        q = np.empty(L1, dtype=np.uint8)
        q[:] = ACGT[rng.integers(0, 4, size=L1)]
        m = min(core.size, L1)
        if kind == END5_GAP:
            q[L1 - m:] = core[core.size - m:]
        else:
            q[:m] = core[:m]
        q = _mutate(rng, q, 0.05, 0.01)
        if rng.random() < 0.3 and L1 > 6:  # a gap
            p = int(rng.integers(1, L1 - 3))
            k = int(rng.integers(1, min(12, L1 - p)))
            if rng.random() < 0.5:
                q = np.concatenate([q[:p], q[p + k:], ACGT[rng.integers(0, 4, size=k)]])
            else:
                q = np.concatenate([q[:p], ACGT[rng.integers(0, 4, size=k)], q[p:L1 - k]])
        uc = q.copy()
        if allow_weird_chars and rng.random() < 0.3:
            lc = rng.random(L1) < 0.2
            q[lc] = q[lc] + 32 * (q[lc] < 97)
            amb = rng.random(L1) < 0.05
            q[amb] = _AMBIG[rng.integers(0, _AMBIG.size, size=int(amb.sum()))]
            uc = q.copy()
            low = (uc >= 97) & (uc <= 122)
            uc[low] -= 32
        qchunks.append(q)
        uchunks.append(uc)
        rec = w[i]
        rec["kind"] = kind
        rec["length1"] = L1
        rec["length2"] = L2
        rec["offset1"] = int(rng.integers(0, 500)) + (L1 - 1 if kind == END5_GAP else 0)
        rec["offset2"] = offset2
        rec["chroffset"] = chroffset
        rec["chrhigh"] = chrhigh
        rec["chrpos"] = chrpos
        rec["genomiclength"] = genomiclength
        rec["qpos"] = qpos + (L1 - 1 if kind == END5_GAP else 0)
        rec["cdna_direction"] = int(rng.choice([-1, 0, 1]))
        rec["extraband"] = int(rng.integers(0, max_band + 1))
        rec["dynprogindex"] = int(rng.choice([-3, 1, 5]))
        rec["maxlength1"] = MAXLENGTH1
        rec["maxlength2"] = MAXLENGTH2
        rec["defect_rate"] = float(rng.choice([0.001, 0.005, 0.02]))
        rec["watsonp"] = watson
        rec["jump_late_p"] = int(rng.integers(0, 2))
        rec["widebandp"] = int(rng.integers(0, 2)) if kind == SINGLE_GAP else 1
        rec["endalign"] = int(rng.choice(list(endaligns))) if kind != SINGLE_GAP else 0
        if kind == SINGLE_GAP and not rec["widebandp"] and abs(L2 - L1) > rec["extraband"]:
            # outside the reference's domain: the sentinel write at dynprog.c:1504
            # lands past row length1 (every caller passes widebandp=true,
            # stage3.c:5453,5593,5783)
            rec["widebandp"] = 1
        qpos += L1 + 4
        qchunks.append(np.full(4, ord("#"), dtype=np.uint8))
        uchunks.append(np.full(4, ord("#"), dtype=np.uint8))
    return Batch(w, np.concatenate(qchunks), np.concatenate(uchunks))


def pack_genome(gseq: np.ndarray) -> np.ndarray:
    return _genome.pack(gseq)
