"""Synthetic workloads.

* ``synthetic_genome``: uniform ACGT with 0.1 % N in runs of 1-10 (seed 1).
* ``c2_windows``: the BASELINE config-2 batch -- 150 bp reads taken from the
  genome (either strand), 2 % substitutions, 0.1 % N, 30 % with one 1-3 bp
  indel, aligned with Dynprog_single_gap, extraband_single 15 (band 31),
  widebandp, defect_rate 0.001, jump_late_p = !watsonp (stage1hr.c:11288).
* ``random_windows``: broad parity mix over every window kind, strand,
  tie rule, quality bin, band, lowercase / ambiguity codes and chromosome
  edges ('*' columns).
* ``ggap_windows``: Dynprog_genome_gap intron windows shaped like
  traverse_genome_gap's (stage3.c:5770-5809), with planted canonical /
  semi-canonical splice sites, plus (``mix=True``) every parameter the entry
  point reads, long and odd-shaped windows and the early-return cases.
* ``c4_windows``: the BASELINE config-4 intron batch (length1 22, length2
  30, extraband_paired 7), vectorised.
* ``cgap_windows``: Dynprog_cdna_gap windows shaped like traverse_cdna_gap's
  (stage3.c:5518-5627): a query gap longer than the genome gap by a cDNA
  insertion of 10-40 bases; length1L = length1R = genomejump + 8.
* ``sj_windows``: Dynprog_end5/3_splicejunction windows shaped like
  Splicetrie_solve_end5/3's (splicetrie.c:325-372, 620-660): a query end
  whose last (end5) or first (end3) ``contlength`` bases continue the anchor
  exon and whose rest comes from a far exon, against the splice junction
  Dynprog_make_splicejunction_5/3 builds (distal + proximal genome), plus
  random segments, planted introns and the early-return cases.
* ``micro_windows``: Dynprog_microexon_int calls shaped like
  traverse_single_gap's (stage3.c:5915): a query gap of cL + microexon + cR
  bases against an intron gap, with a planted AG-microexon-GT (or the
  antisense CT..AC) inside, decoys, and windows with nothing to find.
* ``c5_windows``: the DP windows GSNAP issues for 100 bp reads (BASELINE
  config 5 reduced to its DP part): per read one single gap over
  the read (extraband_single 3) and two end gaps (end5 + end3, length1 1-30,
  length2 = length1 + extramaterial_end 10, extraband_end 3, QUERYEND_GAP).

Deterministic for a given seed (numpy PCG64).
"""
from __future__ import annotations

import os

import numpy as np

from . import genome as _genome
from .records import (BEST_LOCAL, CGAP_WINDOW, MICRO_WINDOW, SJ_WINDOW, END3_GAP, END5_GAP, GGAP_WINDOW, MAXLENGTH1, MAXLENGTH2,
                      QUERYEND_GAP, QUERYEND_INDELS, QUERYEND_NOGAPS, SINGLE_GAP, WINDOW)

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


def concat_batches(parts) -> "Batch":
    """One batch from several (query positions rebased)."""
    ws, qs, us, base = [], [], [], 0
    for b in parts:
        w = b.windows.copy()
        w["qpos"] = w["qpos"] + base
        ws.append(w)
        qs.append(b.query)
        us.append(b.query_uc)
        base += b.query.size
    return Batch(np.concatenate(ws), np.concatenate(qs), np.concatenate(us))


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


_SITES_FWD = (("GT", "AG"), ("GC", "AG"), ("AT", "AC"))
_SITES_REV = (("CT", "AC"), ("CT", "GC"), ("GT", "AT"))


def ggap_windows(gseq: np.ndarray, n: int, seed: int, mix: bool = True):
    """Intron windows on a copy of gseq (splice sites are planted into it).
    Returns (genome, Batch of GGAP_WINDOW)."""
    rng = np.random.default_rng(seed)
    g = gseq.copy()
    Gn = g.size
    w = np.zeros(n, dtype=GGAP_WINDOW)
    qs, us = [], []
    qpos = 0
    for i in range(n):
        u = rng.random()
        if not mix:
            L1 = int(rng.integers(2, 30))
        elif u < 0.55:
            L1 = int(rng.integers(2, 32))
        elif u < 0.80:
            L1 = int(rng.integers(32, 64))
        elif u < 0.92:
            L1 = int(rng.integers(64, 200))
        elif u < 0.95:
            L1 = int(rng.integers(200, 400))
        else:
            L1 = int(rng.integers(0, 3))
        if mix and rng.random() < 0.3:
            L2L = max(1, L1 + int(rng.integers(-1, 41)))
            L2R = max(1, L1 + int(rng.integers(-1, 41)))
            if rng.random() < 0.03:
                L2R = max(1, L1 - int(rng.integers(2, 6)))  # shorter than length1 - 1
        else:
            L2L = L2R = L1 + 8
        intron = int(rng.integers(40, 400))
        glen = max(L2L, L2R) + L1 + intron + 60
        chrpos = int(rng.integers(0, Gn - glen - 1))
        watson = int(rng.integers(0, 2))
        cdir = int(rng.choice([1, -1, 0]))
        k = int(rng.integers(0, L1 + 1))
        offset2L = int(rng.integers(5, 25))
        donor = offset2L + k
        acceptor_end = donor + intron
        revoffset2R = acceptor_end + (L1 - k) - 1
        if revoffset2R >= glen:
            revoffset2R = glen - 1
        if mix and rng.random() < 0.04:  # flanks running off the window: '*' columns
            if rng.random() < 0.5:
                offset2L = -int(rng.integers(1, 6))
            else:
                glen = revoffset2R - int(rng.integers(0, 4))

        def absolute(x):
            return chrpos + (x if watson else glen - 1 - x)

        def put(x, ch):
            if 0 <= x < glen:
                c = ord(ch)
                g[absolute(x)] = c if watson else _COMP[c]

        r = rng.random()
        sites = _SITES_FWD if cdir >= 0 else _SITES_REV
        site = sites[0] if r < 0.6 else sites[1] if r < 0.75 else sites[2] if r < 0.85 else None
        if site:
            put(donor, site[0][0])
            put(donor + 1, site[0][1])
            put(acceptor_end - 2, site[1][0])
            put(acceptor_end - 1, site[1][1])
        lo, hi = max(0, offset2L), min(glen, acceptor_end + L1)
        view = np.full(max(hi, 1), ord("A"), dtype=np.uint8)
        xs = np.arange(lo, hi)
        if xs.size:
            view[lo:hi] = g[chrpos + xs] if watson else _COMP[g[chrpos + glen - 1 - xs]]
        a = view[max(0, offset2L):max(0, offset2L) + k]
        b = view[acceptor_end:acceptor_end + (L1 - k)] if acceptor_end < view.size else view[:0]
        q = np.concatenate([a, b])
        if q.size < L1:
            q = np.concatenate([q, ACGT[rng.integers(0, 4, size=L1 - q.size)]])
        q = _mutate(rng, q, 0.04, 0.01)
        if rng.random() < 0.15 and L1 > 6:
            p = int(rng.integers(1, L1 - 2))
            q = np.concatenate([q[:p], q[p + 1:], ACGT[rng.integers(0, 4, size=1)]])
        quc = q.copy()
        if mix and rng.random() < 0.1 and L1 > 0:  # lowercase and ambiguity codes
            m = rng.random(L1) < 0.3
            q = q.copy()
            q[m] = np.where(rng.random(int(m.sum())) < 0.7, q[m] + 32, _AMBIG[rng.integers(0, _AMBIG.size, int(m.sum()))])
            quc = np.where((q >= 97) & (q <= 122), q - 32, q).astype(np.uint8)
        qs += [q, np.full(4, ord("#"), np.uint8)]
        us += [quc, np.full(4, ord("#"), np.uint8)]
        rec = w[i]
        rec["length1"], rec["length2L"], rec["length2R"] = L1, L2L, L2R
        rec["offset1"] = int(rng.integers(0, 300))
        rec["offset2L"], rec["revoffset2R"] = offset2L, revoffset2R
        rec["chroffset"] = 0
        rec["chrhigh"] = Gn
        rec["chrpos"] = chrpos
        rec["genomiclength"] = glen
        rec["qpos"] = qpos
        rec["cdna_direction"] = cdir
        rec["extraband_paired"] = int(rng.choice([7, 3, 10, 0])) if mix else 7
        rec["maxpeelback"] = int(rng.choice([11, 5, 40])) if mix else 11
        rec["dynprogindex"] = int(rng.choice([-1, 2]))
        small = mix and rng.random() < 0.01
        rec["maxlength1"] = 20 if small else MAXLENGTH1
        rec["maxlength2"] = 30 if small else MAXLENGTH2
        rec["defect_rate"] = float(rng.choice([0.001, 0.005, 0.02]))
        rec["watsonp"] = watson
        rec["jump_late_p"] = int(rng.integers(0, 2))
        rec["halfp"] = int(rng.random() < 0.2)
        rec["finalp"] = int(rng.random() < 0.6)
        rec["use_probabilities_p"] = int(rng.random() < 0.35)
        rec["splicingp"] = int(rng.random() < 0.9)
        rec["score_threshold"] = int(rng.integers(-20, 40)) if rec["use_probabilities_p"] else 0
        qpos += L1 + 4
    return g, Batch(w, np.concatenate(qs), np.concatenate(us))


def c4_windows(gseq: np.ndarray, n: int, seed: int = 4, use_probabilities: bool = False,
               length1: int = 22, extramaterial: int = 8, extraband: int = 7):
    """BASELINE config 4: one Dynprog_genome_gap per intron, length1 =
    2 x maxpeelback (11), length2L = length2R = length1 + 8, extraband_paired 7,
    GT-AG introns of 80-5000 bp (60 % canonical, 25 % semi-canonical, 15 % none),
    1 % substitutions; splice sites are planted into a copy of gseq.
    Returns (genome, Batch)."""
    rng = np.random.default_rng(seed)
    g = gseq.copy()
    L1, L2 = length1, length1 + extramaterial
    intron = rng.integers(80, 5001, size=n)
    k = rng.integers(0, L1 + 1, size=n)                  # query bases in exon 1
    offset2L = np.full(n, 10)
    glen = offset2L + L1 + intron + L2 + 10
    chrpos = rng.integers(0, g.size - int(glen.max()) - 1, size=n)
    donor = offset2L + k
    acc_end = donor + intron
    revoffset2R = acc_end + (L1 - k) - 1
    watson = rng.integers(0, 2, size=n)
    cdir = np.where(rng.random(n) < 0.5, 1, -1)
    u = rng.random(n)
    kind = np.where(u < 0.6, 0, np.where(u < 0.85, 1, 2))  # GT-AG, GC-AG, none

    def absolute(x):
        return np.where(watson == 1, chrpos + x, chrpos + glen - 1 - x)

    def plant(x, chars_fwd, chars_rev, sel):
        c = np.where(cdir > 0, np.frombuffer(chars_fwd, np.uint8)[kind.clip(0, 1)],
                     np.frombuffer(chars_rev, np.uint8)[kind.clip(0, 1)])
        c = np.where(watson == 1, c, _COMP[c])
        g[absolute(x)[sel]] = c[sel]

    has = kind < 2
    plant(donor, b"GG", b"CC", has)        # GT / GC   |  CT / CT
    plant(donor + 1, b"TC", b"TT", has)
    plant(acc_end - 2, b"AA", b"AG", has)  # AG / AG   |  AC / GC
    plant(acc_end - 1, b"GG", b"CC", has)
    # query = exon-1 tail + exon-2 head in window orientation
    j = np.arange(L1)[None, :]
    x = np.where(j < k[:, None], offset2L[:, None] + j, acc_end[:, None] + (j - k[:, None]))
    gi = np.where(watson[:, None] == 1, chrpos[:, None] + x, chrpos[:, None] + glen[:, None] - 1 - x)
    q = g[gi]
    q = np.where(watson[:, None] == 1, q, _COMP[q])
    m = rng.random(q.shape) < 0.01
    q[m] = ACGT[(np.searchsorted(ACGT, q[m]) + rng.integers(1, 4, size=int(m.sum()))) % 4]
    q = np.concatenate([q, np.full((n, 4), ord("#"), np.uint8)], axis=1)
    w = np.zeros(n, dtype=GGAP_WINDOW)
    w["length1"] = L1
    w["length2L"] = L2
    w["length2R"] = L2
    w["offset1"] = rng.integers(0, 300, size=n)
    w["offset2L"] = offset2L
    w["revoffset2R"] = revoffset2R
    w["chroffset"] = 0
    w["chrhigh"] = g.size
    w["chrpos"] = chrpos
    w["genomiclength"] = glen
    w["qpos"] = np.arange(n) * (L1 + 4)
    w["cdna_direction"] = cdir
    w["extraband_paired"] = extraband
    w["maxpeelback"] = 11
    w["dynprogindex"] = 1
    w["maxlength1"] = MAXLENGTH1
    w["maxlength2"] = MAXLENGTH2
    w["defect_rate"] = 0.001
    w["watsonp"] = watson
    w["jump_late_p"] = 0
    w["halfp"] = 0
    w["finalp"] = 1
    w["use_probabilities_p"] = 1 if use_probabilities else 0
    w["splicingp"] = 1
    w["score_threshold"] = 0
    qf = q.reshape(-1).copy()
    return g, Batch(w, qf, qf.copy())


class CgapBatch(Batch):
    """cDNA-gap windows plus each window's genomic segment (the reference's
    sequence2 argument, read only by its INSERT_PAIRS branch)."""

    def __init__(self, windows, query, query_uc, gseg, gseg_off):
        super().__init__(windows, query, query_uc)
        self.gseg = gseg
        self.gseg_off = gseg_off


def cgap_windows(gseq: np.ndarray, n: int, seed: int, mix: bool = True, max_gap: int = 40) -> CgapBatch:
    rng = np.random.default_rng(seed)
    Gn = gseq.size
    w = np.zeros(n, dtype=CGAP_WINDOW)
    qs, us, segs, soff = [], [], [], [0]
    qpos = 0
    for i in range(n):
        G = int(rng.integers(2, max_gap + 1)) if not mix or rng.random() < 0.97 else int(rng.integers(0, 2))
        ins = int(rng.integers(10, 41))
        glen = 200 + G
        chrpos = int(rng.integers(0, Gn - glen - 1))
        watson = int(rng.integers(0, 2))
        off2 = int(rng.integers(20, 60))
        xs = np.arange(glen)
        view = gseq[chrpos + xs] if watson else _COMP[gseq[chrpos + glen - 1 - xs]]
        a = int(rng.integers(0, G + 1))
        pad5, pad3 = int(rng.integers(0, 20)), int(rng.integers(0, 20))
        if mix and G >= 12 and rng.random() < 0.3:
            # a 9-base genome block replaced by 9 + extra random query bases: the
            # bridge may leave exactly 9 x 9 unaligned (INSERT_PAIRS, dynprog.c:4730)
            # (queryjump = genomejump here: outside traverse_cdna_gap's shapes,
            # inside Dynprog_cdna_gap's domain)
            a = int(rng.integers(2, G - 9))
            core = np.concatenate([view[off2:off2 + a], ACGT[rng.integers(0, 4, size=9)],
                                   view[off2 + a + 9:off2 + G]])
        else:
            core = np.concatenate([view[off2:off2 + a], ACGT[rng.integers(0, 4, size=ins)], view[off2 + a:off2 + G]])
        q = np.concatenate([ACGT[rng.integers(0, 4, size=pad5)], core, ACGT[rng.integers(0, 4, size=pad3)]])
        q = _mutate(rng, q, 0.02, 0.005)
        quc = q.copy()
        if mix and rng.random() < 0.1:
            m = rng.random(q.size) < 0.3
            q[m] = np.where(rng.random(int(m.sum())) < 0.7, q[m] + 32,
                            _AMBIG[rng.integers(0, _AMBIG.size, int(m.sum()))])
            quc = np.where((q >= 97) & (q <= 122), q - 32, q).astype(np.uint8)
        Q = core.size
        qd5 = 100 + pad5          # query coordinate of querydp5
        rec = w[i]
        rec["length2"] = G
        rec["length1L"] = rec["length1R"] = G + 8  # queryjump = genomejump + extramaterial_paired
        rec["offset1L"] = qd5
        rec["revoffset1R"] = qd5 + Q - 1
        rec["offset2"] = off2
        rec["chroffset"] = 0
        rec["chrhigh"] = Gn
        rec["chrpos"] = chrpos
        rec["genomiclength"] = glen
        rec["qposL"] = qpos + pad5
        rec["qposR"] = qpos + pad5 + Q - 1
        rec["cdna_direction"] = int(rng.choice([1, -1, 0]))
        rec["extraband_paired"] = int(rng.choice([7, 3, 10])) if mix else 7
        rec["dynprogindex"] = int(rng.choice([-1, 2]))
        small = mix and rng.random() < 0.01
        rec["maxlength1"] = 20 if small else MAXLENGTH1
        rec["maxlength2"] = 30 if small else MAXLENGTH2
        rec["defect_rate"] = float(rng.choice([0.001, 0.005, 0.02]))
        rec["watsonp"] = watson
        rec["jump_late_p"] = int(rng.integers(0, 2))
        qs += [q, np.full(4, ord("#"), np.uint8)]
        us += [quc, np.full(4, ord("#"), np.uint8)]
        qpos += q.size + 4
        seg = view[off2:off2 + max(G, 0)] if G > 0 else view[:0]
        segs.append(np.concatenate([seg, np.zeros(4, np.uint8)]))
        soff.append(soff[-1] + segs[-1].size)
    gs = np.concatenate(segs)
    # sequence2[k] is addressed relative to offset2
    return CgapBatch(w, np.concatenate(qs), np.concatenate(us), gs, np.array(soff[:-1], dtype=np.int64))


def sj_windows(gseq: np.ndarray, n: int, seed: int, mix: bool = True) -> Batch:
    rng = np.random.default_rng(seed)
    Gn = gseq.size
    w = np.zeros(n, dtype=SJ_WINDOW)
    qs, us = [], []
    qpos = 0
    for i in range(n):
        end5 = bool(rng.integers(0, 2))
        r = rng.random()
        L1 = int(rng.integers(1, 41)) if r < 0.85 else int(rng.integers(41, 160))
        extra = 10 if rng.random() < 0.7 else int(rng.integers(0, 40))
        L2 = L1 + extra
        cont = int(rng.integers(0, L1))
        spl = L2 - cont
        a = int(rng.integers(0, Gn - cont - 1))
        f = int(rng.integers(0, Gn - spl - 1))
        prox = gseq[a:a + cont]
        dist = gseq[f:f + spl]
        if not bool(rng.integers(0, 2)):  # minus-strand junctions are complemented in place (:6091)
            prox, dist = _COMP[prox], _COMP[dist]
        if mix and rng.random() < 0.15:
            dist = dist.copy()
            k = int(rng.integers(0, max(1, spl - 30)))
            dist[k:k + 2] = np.frombuffer(b"GT", np.uint8)[:dist[k:k + 2].size]
            dist[k + 14:k + 16] = np.frombuffer(b"AG", np.uint8)[:dist[k + 14:k + 16].size]
        if end5:
            seg = np.concatenate([dist, prox])          # distal first (:6068), proximal at [splicelength]
            q = np.concatenate([dist[spl - (L1 - cont):] if L1 > cont else dist[:0], prox])
        else:
            seg = np.concatenate([prox, dist])          # proximal first, distal at [contlength] (:6152)
            q = np.concatenate([prox, dist[:L1 - cont]])
        if mix and rng.random() < 0.2:
            seg = ACGT[rng.integers(0, 4, size=L2)]
        q = _mutate(rng, q, 0.03, 0.01)
        if mix and rng.random() < 0.2 and L1 > 6:  # a small indel
            p = int(rng.integers(1, L1 - 2))
            if rng.random() < 0.5:
                q = np.concatenate([q[:p], q[p + 1:], ACGT[rng.integers(0, 4, size=1)]])
            else:
                q = np.concatenate([q[:p], ACGT[rng.integers(0, 4, size=1)], q[p:-1]])
        quc = q.copy()
        if mix and rng.random() < 0.1:
            m = rng.random(q.size) < 0.3
            q = q.copy()
            q[m] = np.where(rng.random(int(m.sum())) < 0.7, q[m] + 32,
                            _AMBIG[rng.integers(0, _AMBIG.size, int(m.sum()))])
            quc = np.where((q >= 97) & (q <= 122), q - 32, q).astype(np.uint8)
        rec = w[i]
        rec["kind"] = END5_GAP if end5 else END3_GAP
        rec["length1"] = L1
        rec["length2"] = L2
        rec["contlength"] = cont
        base1 = int(rng.integers(0, 400))
        anchor = int(rng.integers(50, 400))
        intron = int(rng.integers(60, 5000))
        if end5:
            rec["offset1"] = base1 + L1 - 1                  # revoffset1
            rec["offset2_anchor"] = anchor
            rec["offset2_far"] = anchor - intron             # splicetrie.c:346-351
            rec["qpos"] = qpos + L1 - 1
            rec["spos"] = qpos + L1 + 4 + L2 - 1
        else:
            rec["offset1"] = base1
            rec["offset2_anchor"] = anchor
            rec["offset2_far"] = anchor + intron
            rec["qpos"] = qpos
            rec["spos"] = qpos + L1 + 4
        rec["cdna_direction"] = int(rng.choice([1, -1, 0]))
        rec["extraband_end"] = int(rng.choice([3, 3, 5, 10])) if mix else 3
        rec["dynprogindex"] = int(rng.choice([-1, 2]))
        small = mix and rng.random() < 0.02
        rec["maxlength1"] = 20 if small else MAXLENGTH1
        rec["maxlength2"] = 30 if small else MAXLENGTH2
        rec["defect_rate"] = float(rng.choice([0.001, 0.005, 0.02]))
        rec["watsonp"] = int(rng.integers(0, 2))
        rec["jump_late_p"] = int(rng.integers(0, 2))
        pad = np.full(4, ord("#"), np.uint8)
        qs += [q, pad, seg, pad]
        us += [quc, pad, seg, pad]
        qpos += L1 + 4 + L2 + 4
    if mix and n >= 4:  # early returns: empty query / segment
        w[0]["length1"] = 0
        w[1]["length2"] = 0
    return Batch(w, np.concatenate(qs), np.concatenate(us))


def micro_windows(gseq: np.ndarray, n: int, seed: int, mix: bool = True):
    """Returns (genome with the planted sites, Batch of MICRO_WINDOW records)."""
    rng = np.random.default_rng(seed)
    g = gseq.copy()
    Gn = g.size
    w = np.zeros(n, dtype=MICRO_WINDOW)
    qs, us = [], []
    qpos = 0
    for i in range(n):
        cdir = 1 if rng.random() < 0.5 else -1
        cL = int(rng.integers(1, 12))
        mid = int(rng.integers(3, 13))
        cR = int(rng.integers(1, 12))
        L1 = cL + mid + cR
        I1 = int(rng.integers(20, 400))
        I2 = int(rng.integers(20, 400))
        o = int(rng.integers(5, 40))
        m = o + cL + I1
        r0 = m + mid + I2
        rev2R = r0 + cR - 1
        glen = rev2R + int(rng.integers(5, 40))
        chrpos = int(rng.integers(0, Gn - glen - 1))
        watson = int(rng.integers(0, 2))

        def absolute(x):
            return chrpos + (x if watson else glen - 1 - x)

        def put(x, seq):
            for k, ch in enumerate(seq):
                c = ord(ch) if isinstance(ch, str) else int(ch)
                g[absolute(x + k)] = c if watson else _COMP[c]

        dl, dr = ("GT", "AG") if cdir > 0 else ("CT", "AC")
        plant = not mix or rng.random() < 0.8
        if plant:
            put(o + cL, dl)
            put(m - 2, dr)
            put(m + mid, dl)
            put(r0 - 2, dr)
            if mix and rng.random() < 0.3:  # a second copy of the microexon (ties, hit order)
                m2 = o + cL + 9 + int(rng.integers(2, max(3, I1 - mid - 12)))
                if m2 + mid + 2 < m - 2:
                    view = [g[absolute(x)] if watson else _COMP[g[absolute(x)]] for x in range(m, m + mid)]
                    put(m2 - 2, dr)
                    put(m2, view)
                    put(m2 + mid, dl)
        xs = np.arange(glen)
        view = g[chrpos + xs] if watson else _COMP[g[chrpos + glen - 1 - xs]]
        q = np.concatenate([view[o:o + cL], view[m:m + mid], view[r0:r0 + cR]])
        if mix and rng.random() < 0.3:
            q = _mutate(rng, q, 0.05, 0.0)
        quc = q.copy()
        if mix and rng.random() < 0.05:
            q = q.copy()
            q[int(rng.integers(0, L1))] += 32  # lowercase query byte
            quc = np.where((q >= 97) & (q <= 122), q - 32, q).astype(np.uint8)
        rec = w[i]
        rec["length1"] = L1
        rec["offset1"] = int(rng.integers(0, 200))
        rec["offset2L"] = o
        rec["revoffset2R"] = rev2R
        rec["cdna_direction"] = cdir
        rec["dynprogindex"] = int(rng.choice([-1, 2]))
        rec["chroffset"] = 0
        rec["chrhigh"] = Gn
        rec["chrpos"] = chrpos
        rec["genomiclength"] = glen
        rec["qpos"] = qpos
        rec["ppos"] = qpos
        rec["defect_rate"] = float(rng.choice([0.001, 0.005, 0.02]))
        rec["watsonp"] = watson
        qs += [q, np.full(4, ord("#"), np.uint8)]
        us += [quc, np.full(4, ord("#"), np.uint8)]
        qpos += L1 + 4
    return g, Batch(w, np.concatenate(qs), np.concatenate(us))


def c5_windows(gseq: np.ndarray, nreads: int, seed: int = 5, read_len: int = 100,
               extraband_single: int = 3, extraband_end: int = 3, extramaterial_end: int = 10) -> Batch:
    singles = c2_windows(gseq, nreads, seed=seed, read_len=read_len, extraband=extraband_single)
    rng = np.random.default_rng(seed + 1000)
    n = 2 * nreads
    G = gseq.size
    margin, stride = 8, 48
    L1 = rng.integers(1, 31, size=n)
    L2 = L1 + extramaterial_end
    end5 = (np.arange(n) % 2) == 0
    watson = rng.integers(0, 2, size=n).astype(bool)
    glen = L2 + 2 * margin
    chrpos = rng.integers(0, G - int(glen.max()) - 1, size=n)
    # window genome (get_genomic_nt orientation): columns margin .. margin+L2-1
    j = np.arange(int(glen.max()))[None, :]
    gi = np.where(watson[:, None], chrpos[:, None] + j, chrpos[:, None] + glen[:, None] - 1 - j)
    gi = np.minimum(gi, G - 1)
    seg = gseq[gi]
    seg = np.where(watson[:, None], seg, _COMP[seg])
    # the query: end3 aligns its first bases to the first columns, end5 its last
    # bases to the last columns (read backwards from revoffset2)
    k = np.arange(30)[None, :]
    col = np.where(end5[:, None], margin + L2[:, None] - L1[:, None] + k, margin + k)
    q = np.take_along_axis(seg, np.minimum(col, seg.shape[1] - 1), axis=1)
    m = rng.random(q.shape) < 0.02
    q[m] = ACGT[(np.searchsorted(ACGT, q[m]) + rng.integers(1, 4, size=int(m.sum()))) % 4]
    q[k >= L1[:, None]] = ord("#")
    qbuf = np.full((n, stride), ord("#"), dtype=np.uint8)
    qbuf[:, :30] = q
    w = np.zeros(n, dtype=WINDOW)
    w["kind"] = np.where(end5, END5_GAP, END3_GAP)
    w["length1"] = L1
    w["length2"] = L2
    w["offset1"] = np.where(end5, L1 - 1, read_len - L1)
    w["offset2"] = np.where(end5, margin + L2 - 1, margin)
    w["chroffset"] = 0
    w["chrhigh"] = G
    w["chrpos"] = chrpos
    w["genomiclength"] = glen
    w["qpos"] = np.arange(n) * stride + np.where(end5, L1 - 1, 0)  # rebased by concat_batches
    w["cdna_direction"] = 1
    w["extraband"] = extraband_end
    w["dynprogindex"] = 1
    w["maxlength1"] = MAXLENGTH1
    w["maxlength2"] = MAXLENGTH2
    w["defect_rate"] = 0.001
    w["watsonp"] = watson.astype(np.uint8)
    w["jump_late_p"] = 1 - w["watsonp"]
    w["widebandp"] = 1
    w["endalign"] = QUERYEND_GAP
    ends = Batch(w, qbuf.reshape(-1), qbuf.reshape(-1).copy())
    both = concat_batches([singles, ends])
    return Batch(both.windows, both.query, both.query_uc)


def pack_genome(gseq: np.ndarray) -> np.ndarray:
    return _genome.pack(gseq)


def synthetic_transcripts(seed: int = 7, ngenes: int = 16, genome_len: int = 160_000, cins: float = 0.0,
                          small_frac: float = 0.12, small_len=(12, 30), intron_len=(70, 1501)):
    """End-to-end gmap inputs (tests/test_gmap_e2e.py): a genomic segment
    carrying ``ngenes`` spliced genes and one cDNA per gene.

    Each gene has 2-12 exons of 12-260 nt (a few microexon-sized ones:
    `small_frac` of them, `small_len` nt) and introns of 70-1500 nt
    (`intron_len`).  Intron ends are GT-AG (80 %), GC-AG (8 %), AT-AC
    (5 %) or random (7 %); the canonical ones sit in splice-site context
    (exon ..AG | GTRAGT donor, a pyrimidine tract and YAG | G acceptor) so that
    GMAP's MaxEnt-guided stage 3 accepts them.  A third of the genes lie on
    the minus strand, and their cDNAs are given reverse-complemented (gmap -g
    at this version reports no alignment on the segment's minus strand, even
    with its own dynprog.o, so every cDNA is placed to align on the plus
    strand: sense or antisense).  The
    cDNAs carry 1 % substitutions, occasional N, a 1-6 nt indel in a third of
    them, and a poly-A tail on some.  Returns (genome bytes, [(name, cDNA)]).
    """
    rng = np.random.default_rng(seed)
    g = ACGT[rng.integers(0, 4, size=genome_len)]
    b = lambda t: np.frombuffer(t, np.uint8)  # noqa: E731
    queries = []
    pos = 2000
    for k in range(ngenes):
        nex = int(rng.integers(2, 13))
        exl = rng.integers(40, 261, size=nex)
        small = rng.random(nex) < small_frac
        exl[small] = rng.integers(small_len[0], small_len[1], size=int(small.sum()))
        exl[0] = max(exl[0], 60)
        exl[-1] = max(exl[-1], 60)
        inl = rng.integers(intron_len[0], intron_len[1], size=nex - 1)
        span = int(exl.sum() + inl.sum())
        if pos + span + 2000 > genome_len:
            break
        gene = g[pos:pos + span].copy()
        spans, p = [], 0
        for e in range(nex):
            spans.append((p, int(exl[e])))
            p += int(exl[e])
            if e == nex - 1:
                break
            r, n = rng.random(), int(inl[e])
            kind = 0 if r < 0.80 else 1 if r < 0.88 else 2 if r < 0.93 else 3
            if kind < 3:
                donor = (b"GT", b"GC", b"AT")[kind] + (b"AAGT", b"GAGT", b"AAGA")[int(rng.integers(0, 3))]
                accept = b"AG" if kind < 2 else b"AC"
                gene[p:p + 6] = b(donor)
                gene[p - 2:p] = b(b"AG")
                tract = np.where(rng.random(14) < 0.9, b(b"CT")[rng.integers(0, 2, size=14)],
                                 ACGT[rng.integers(0, 4, size=14)])
                gene[p + n - 18:p + n - 4] = tract
                gene[p + n - 3:p + n] = b(b"C" + accept)
                gene[p + n] = ord("G")
            p += n
        exons = [gene[s0:s0 + L].copy() for s0, L in spans]
        minus = rng.random() < 1 / 3
        g[pos:pos + span] = revcomp(gene) if minus else gene
        if cins > 0:
            # query-side insertions of 11-60 nt (beyond EXTRAQUERYGAP, stage3.c:7783):
            # inside an exon or at an exon boundary, so that stage 2 leaves a gap
            # with queryjump > genomejump + 10 for traverse_cdna_gap (:5518)
            for e in range(nex):
                if rng.random() < cins:
                    n = int(rng.integers(11, 61))
                    at = int(rng.integers(0, exons[e].size + 1)) if rng.random() < 0.6 else \
                        (exons[e].size if rng.random() < 0.5 else 0)
                    exons[e] = np.concatenate([exons[e][:at], ACGT[rng.integers(0, 4, size=n)], exons[e][at:]])
        cdna = np.concatenate(exons)
        cdna = _mutate(rng, cdna, 0.01, 0.001)
        if rng.random() < 1 / 3:
            at = int(rng.integers(30, cdna.size - 30))
            n = int(rng.integers(1, 7))
            if rng.random() < 0.5:
                cdna = np.concatenate([cdna[:at], cdna[at + n:]])
            else:
                cdna = np.concatenate([cdna[:at], ACGT[rng.integers(0, 4, size=n)], cdna[at:]])
        if rng.random() < 0.3:
            cdna = np.concatenate([cdna, np.full(int(rng.integers(10, 30)), ord("A"), np.uint8)])
        if minus:
            cdna = revcomp(cdna)
        queries.append(("synth%02d" % k, cdna.tobytes()))
        pos += span + int(rng.integers(500, 3000))
    return g.tobytes(), queries


def write_fasta(path: str, records, width: int = 60) -> None:
    """records: [(name, bytes)] -> FASTA file."""
    with open(path, "wb") as f:
        for name, seq in records:
            f.write(b">" + name.encode() + b"\n")
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width] + b"\n")


# ---------------------------------------------------------------------------
# BASELINE config 3: 150 bp reads against a GRCh38-sized genome.
# No GRCh38 index exists here (no network), so the genome is synthetic with
# the 24 primary GRCh38 chromosome lengths (chr1..chr22, X, Y; 3.09 Gnt, 1.16 GB
# packed), generated directly in the packed block format: for a uniform ACGT
# genome the (high, low) words of a block are uniform random 32-bit words.
GRCH38_CHROMS = (
    ("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
    ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
    ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
    ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
    ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
    ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415),
)


class PackedGenome:
    """Packed blocks (genome.c:9325 layout, +4 guard words) plus the chromosome
    table GMAP keeps beside them (chroffset = cumulative start, chrhigh =
    chroffset + length)."""

    def __init__(self, blocks: np.ndarray, names, lengths: np.ndarray):
        self.blocks = blocks
        self.names = list(names)
        self.lengths = np.asarray(lengths, dtype=np.int64)
        self.offsets = np.concatenate([[0], np.cumsum(self.lengths)[:-1]]).astype(np.int64)
        self.total = int(self.lengths.sum())

    def decode(self, pos: np.ndarray) -> np.ndarray:
        """Genome characters at absolute positions (uncompress_one_char, genome.c:9325)."""
        return decode_blocks(self.blocks, pos)


def decode_blocks(blocks: np.ndarray, pos: np.ndarray) -> np.ndarray:
    pos = np.asarray(pos, dtype=np.int64)
    ptr = (pos >> 5) * 3
    bit = (pos & 31).astype(np.uint32)
    word = np.where(bit < 16, blocks[ptr + 1], blocks[ptr])
    c = (word >> ((bit & 15) * 2)) & 3
    ch = ACGT[c]
    return np.where(((blocks[ptr + 2] >> bit) & 1) == 1, np.uint8(ord("N")), ch).astype(np.uint8)


def c3_genome(seed: int = 3, scale: float = 1.0, n_rate: float = 0.001) -> PackedGenome:
    """GRCh38-shaped synthetic genome in packed form.  `scale` < 1 shrinks every
    chromosome (tests); 1.0 is the C3 size.  ~n_rate N bases in runs of 1-10."""
    rng = np.random.default_rng(seed)
    lengths = np.array([max(4096, int(l * scale)) for _, l in GRCH38_CHROMS], dtype=np.int64)
    total = int(lengths.sum())
    nblocks = (total + 31) // 32
    hl = rng.integers(0, 1 << 32, size=2 * nblocks, dtype=np.uint32)
    high, low = hl[:nblocks], hl[nblocks:]
    flags = np.zeros(nblocks, dtype=np.uint32)
    nruns = int(total * n_rate / 5.5)
    if nruns:
        starts = rng.integers(0, total, size=nruns)
        lens = rng.integers(1, 11, size=nruns)
        pos = np.repeat(starts, lens) + (np.arange(int(lens.sum())) - np.repeat(np.cumsum(lens) - lens, lens))
        pos = np.unique(pos[pos < total])
        blk, bit = pos >> 5, (pos & 31).astype(np.uint32)
        np.bitwise_or.at(flags, blk, np.uint32(1) << bit)
        lo = bit < 16  # N = A + flag: clear the 2-bit code
        np.bitwise_and.at(low, blk[lo], ~(np.uint32(3) << (2 * bit[lo])))
        np.bitwise_and.at(high, blk[~lo], ~(np.uint32(3) << (2 * (bit[~lo] - 16))))
    tail = nblocks * 32 - total  # X past the end (Genome_create_blocks)
    if tail:
        for b in range(32 - tail, 32):
            flags[-1] |= np.uint32(1) << np.uint32(b)
            if b < 16:
                low[-1] |= np.uint32(3) << np.uint32(2 * b)
            else:
                high[-1] |= np.uint32(3) << np.uint32(2 * (b - 16))
    blocks = np.empty(3 * nblocks + 4, dtype=np.uint32)
    blocks[0:3 * nblocks:3] = high
    blocks[1:3 * nblocks:3] = low
    blocks[2:3 * nblocks:3] = flags
    blocks[3 * nblocks:] = 0xFFFFFFFF
    return PackedGenome(blocks, [n for n, _ in GRCH38_CHROMS], lengths)


def c3_windows(g: PackedGenome, n: int = 1_000_000, seed: int = 33, read_len: int = 150,
               extraband: int = 15, indel_frac: float = 0.3, sub_rate: float = 0.02,
               n_rate: float = 0.001, margin: int = 8, chunk: int = 131072) -> Batch:
    """BASELINE config 3: `n` Dynprog_single_gap windows of 150 bp reads drawn
    from every chromosome (length-weighted), either strand, 2 % substitutions,
    0.1 % N, 30 % with one 1-3 bp indel; extraband 15, widebandp, HIGHQ,
    jump_late_p = !watsonp (stage1hr.c:11288).  Vectorised (same read model as
    c2_windows, its own random stream)."""
    rng = np.random.default_rng(seed)
    stride = read_len + 8
    w = np.zeros(n, dtype=WINDOW)
    qbuf = np.full((n, stride), ord("#"), dtype=np.uint8)
    ci = rng.choice(len(g.lengths), size=n, p=g.lengths / g.lengths.sum())
    chrlen = g.lengths[ci]
    has = rng.random(n) < indel_frac
    ilen = rng.integers(1, 4, size=n)
    sign = rng.integers(0, 2, size=n) * 2 - 1  # +1: genome longer (deletion in the read)
    L2 = read_len + np.where(has, sign * ilen, 0)
    watson = rng.integers(0, 2, size=n).astype(bool)
    start = (rng.random(n) * (chrlen - read_len - 16 - 3 * margin)).astype(np.int64) + 2 * margin
    seg_start = start - margin
    glen = L2 + 2 * margin
    kdel = np.maximum(L2 - read_len, 0)
    kins = np.maximum(read_len - L2, 0)
    p = np.where(kdel > 0, rng.integers(10, read_len - 10, size=n),
                 (rng.random(n) * (L2 - 20)).astype(np.int64) + 10)
    ins_bases = rng.integers(0, 4, size=(n, 3))
    k = np.arange(read_len)[None, :]
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        s = slice(lo, hi)
        pk, kd, ki = p[s, None], kdel[s, None], kins[s, None]
        j = k + np.where(k >= pk, kd, 0) - np.where(k >= pk + ki, ki, 0)  # window column of base k
        inserted = (k >= pk) & (k < pk + ki)
        base = g.offsets[ci[s], None] + seg_start[s, None]
        gp = np.where(watson[s, None], base + margin + j, base + glen[s, None] - 1 - margin - j)
        q = g.decode(np.where(inserted, base + margin, gp))
        q = np.where(watson[s, None], q, _COMP[q])
        rnd = ACGT[ins_bases[s][np.arange(hi - lo)[:, None], np.clip(k - pk, 0, 2)]]
        q = np.where(inserted, rnd, q)
        m = rng.random(q.shape)
        sub = m < sub_rate
        q[sub] = ACGT[(np.searchsorted(ACGT, q[sub]) + rng.integers(1, 4, size=int(sub.sum()))) % 4]
        q[(m >= sub_rate) & (m < sub_rate + n_rate)] = ord("N")
        qbuf[s, :read_len] = q
    w["kind"] = SINGLE_GAP
    w["length1"] = read_len
    w["length2"] = L2
    w["offset1"] = 0
    w["offset2"] = margin
    w["chroffset"] = g.offsets[ci]
    w["chrhigh"] = g.offsets[ci] + chrlen
    w["chrpos"] = seg_start
    w["genomiclength"] = glen
    w["qpos"] = np.arange(n, dtype=np.int64) * stride
    w["cdna_direction"] = 1
    w["extraband"] = extraband
    w["dynprogindex"] = 1
    w["maxlength1"] = MAXLENGTH1
    w["maxlength2"] = MAXLENGTH2
    w["defect_rate"] = 0.001
    w["watsonp"] = watson.astype(np.uint8)
    w["jump_late_p"] = 1 - w["watsonp"]
    w["widebandp"] = 1
    q = qbuf.reshape(-1)
    return Batch(w, q, q.copy())


# ---------------------------------------------------------------- known splice sites
class SpliceSiteSet:
    """A splicing IIT's intervals, answering the four queries bridge_intron_gap
    makes of it (dynprog.c:3375-3550, 3598-3612), restated over plain sets:

    * ``IIT_exists_with_divno_typed_signed(x, y, type, sign)`` (iit-read.c:4011):
      an interval with low == x, high == y, that type and sign;
    * ``IIT_low_exists_signed_p(x, sign)`` / ``IIT_high_exists_signed_p`` (:3770, :3808):
      an interval whose low (high) end is x, with that sign;
    * ``IIT_exists_with_divno_signed(x, y, sign)`` (:3973): low == x, high == y, sign.

    Intervals are given as iit_store writes them (``start..end``; start > end
    means the minus sign, Interval_new, interval.c:22-40).  One division only:
    the windows' chrnum maps to it."""

    def __init__(self, intervals):
        self.typed, self.exact, self.lows, self.highs = set(), set(), set(), set()
        self.intervals = list(intervals)
        for start, end, typ in self.intervals:
            lo, hi = min(start, end), max(start, end)
            sign = 1 if start < end else (-1 if start > end else 0)
            self.typed.add((lo, hi, typ, sign))
            self.exact.add((lo, hi, sign))
            self.lows.add((lo, sign))
            self.highs.add((hi, sign))
        self.site_level = any(t == "donor" for _, _, t in self.intervals) and \
            any(t == "acceptor" for _, _, t in self.intervals)

    def iit_text(self, div: str) -> str:
        """iit_store FASTA input (">label div:start..end [type]")."""
        out = []
        for i, (start, end, typ) in enumerate(self.intervals):
            out.append(">s%d %s:%d..%d%s\n" % (i, div, start, end, " " + typ if typ else ""))
        return "".join(out)

    def flags(self, w) -> tuple:
        """left_known / right_known of one gsnapdp_ggap_window (dynprog.c:3375-3550)."""
        L2L, L2R = int(w["length2L"]), int(w["length2R"])
        lo, ro = int(w["offset2L"]), int(w["revoffset2R"])
        chrpos, gl = int(w["chrpos"]), int(w["genomiclength"])
        watson, fwd = bool(w["watsonp"]), int(w["cdna_direction"]) > 0
        left, right = np.zeros(L2L, np.uint8), np.zeros(L2R, np.uint8)
        for cL in range(L2L - 1):
            pos = chrpos + lo + cL if watson else chrpos + (gl - 1) - lo - cL + 1
            if self.site_level:
                typ = "donor" if fwd else "acceptor"
                sign = (1 if fwd else -1) if watson else (-1 if fwd else 1)
                left[cL] = (pos, pos + 1, typ, sign) in self.typed
            elif watson:
                left[cL] = (pos, 1 if fwd else -1) in self.lows
            else:
                left[cL] = (pos + 1, -1 if fwd else 1) in self.highs
        for cR in range(L2R - 1):
            pos = chrpos + ro - cR + 1 if watson else chrpos + (gl - 1) - ro + cR
            if self.site_level:
                typ = "acceptor" if fwd else "donor"
                sign = (1 if fwd else -1) if watson else (-1 if fwd else 1)
                right[cR] = (pos, pos + 1, typ, sign) in self.typed
            elif watson:
                right[cR] = (pos + 1, 1 if fwd else -1) in self.highs
            else:
                right[cR] = (pos, -1 if fwd else 1) in self.lows
        return left, right

    def intron_pairs(self, w, left, right) -> list:
        """(cL, cR), both flagged, whose intron the IIT holds (dynprog.c:3598-3612)."""
        lo, ro = int(w["offset2L"]), int(w["revoffset2R"])
        chrpos, gl, cdir = int(w["chrpos"]), int(w["genomiclength"]), int(w["cdna_direction"])
        out = []
        for cL in np.flatnonzero(left):
            for cR in np.flatnonzero(right):
                if w["watsonp"]:
                    x, y, s = chrpos + lo + cL, chrpos + ro - cR + 1 + 1, cdir
                else:
                    x, y, s = chrpos + (gl - 1) - ro + cR, chrpos + (gl - 1) - lo - cL + 1 + 1, -cdir
                if (x, y, s) in self.exact:
                    out.append((int(cL), int(cR)))
        return out


def with_known_sites(windows, query, query_uc, sites: SpliceSiteSet, novelsplicingp: bool):
    """Copy of a genome-gap batch with each window's known-site record placed
    after its query rows (include/gsnapdp.h, gsnapdp_ggap_window) and known_mode
    set the way Dynprog_setup's IIT and novelsplicingp select it (dynprog.c:3552,
    :4084-4101)."""
    if novelsplicingp:
        mode = 1  # GSNAPDP_KNOWN_REWARD
    else:
        mode = 2 if sites.site_level else 3  # GSNAPDP_KNOWN_SITES / GSNAPDP_KNOWN_INTRONS
    w = windows.copy()
    qs, us, pos = [], [], 0
    for i in range(len(w)):
        L1, q0 = int(w[i]["length1"]), int(w[i]["qpos"])
        left, right = sites.flags(w[i])
        rec = [left, right]
        pairs = sites.intron_pairs(w[i], left, right) if mode == 3 else []
        rec.append(np.array([len(pairs) & 255, len(pairs) >> 8], np.uint8))
        for cL, cR in pairs:
            rec.append(np.array([cL & 255, cL >> 8, cR & 255, cR >> 8], np.uint8))
        rec = np.concatenate(rec)
        pad = np.full(4, ord("#"), np.uint8)
        qs += [query[q0:q0 + L1], rec, pad]
        us += [query_uc[q0:q0 + L1], rec, pad]
        w[i]["qpos"] = pos
        w[i]["known_mode"] = mode
        pos += L1 + rec.size + 4
    return w, np.concatenate(qs), np.concatenate(us)


def known_site_intervals(w, res, rng, site_level: bool) -> list:
    """Splice sites / introns around each genome-gap window (test workloads):
    the sites the bridge picks without an IIT (`res`, a gsnapdp_ggap_result
    array, or None), random columns, and decoys of the wrong type or sign.  Coordinates as bridge_intron_gap queries them
    (dynprog.c:3375-3550, 3598-3612)."""
    out = []

    def lpos(x, cL):
        return (int(x["chrpos"]) + int(x["offset2L"]) + cL if x["watsonp"] else
                int(x["chrpos"]) + (int(x["genomiclength"]) - 1) - int(x["offset2L"]) - cL + 1)

    def rpos(x, cR):
        return (int(x["chrpos"]) + int(x["revoffset2R"]) - cR + 1 if x["watsonp"] else
                int(x["chrpos"]) + (int(x["genomiclength"]) - 1) - int(x["revoffset2R"]) + cR)

    for x, r in zip(w, res if res is not None else [None] * len(w)):
        L2L, L2R = int(x["length2L"]), int(x["length2R"])
        if L2L < 2 or L2R < 2:
            continue
        fwd = int(x["cdna_direction"]) > 0
        if r is not None and r["returned_null"] == 0:
            cl0 = int(r["new_leftgenomepos"]) - int(x["offset2L"]) + 1
            cr0 = int(x["revoffset2R"]) - int(r["new_rightgenomepos"]) + 1
        else:
            cl0, cr0 = int(rng.integers(0, L2L - 1)), int(rng.integers(0, L2R - 1))
        cls = {cl0} | {int(c) for c in rng.integers(0, L2L - 1, size=3)}
        crs = {cr0} | {int(c) for c in rng.integers(0, L2R - 1, size=3)}
        if site_level:
            sign = (1 if fwd else -1) if x["watsonp"] else (-1 if fwd else 1)
            lt, rt = ("donor", "acceptor") if fwd else ("acceptor", "donor")
            for cL in cls:
                p = lpos(x, cL)
                t = lt if rng.random() < 0.85 else rt           # decoy: wrong type
                sg = sign if rng.random() < 0.9 else -sign      # decoy: wrong sign
                out.append((p, p + 1, t) if sg > 0 else (p + 1, p, t))
            for cR in crs:
                p = rpos(x, cR)
                t = rt if rng.random() < 0.85 else lt
                sg = sign if rng.random() < 0.9 else -sign
                out.append((p, p + 1, t) if sg > 0 else (p + 1, p, t))
        else:
            cdir = int(x["cdna_direction"])
            for cL in cls:
                for cR in crs:
                    if rng.random() < (0.9 if (cL, cR) == (cl0, cr0) else 0.25):
                        if x["watsonp"]:
                            lo_, hi_, sg = lpos(x, cL), rpos(x, cR) + 1, cdir
                        else:
                            lo_, hi_, sg = rpos(x, cR), lpos(x, cL) + 1, -cdir
                        if sg == 0:
                            sg = 1 if rng.random() < 0.5 else -1
                        if lo_ < hi_:
                            out.append((lo_, hi_, None) if sg > 0 else (hi_, lo_, None))
            for cL in cls:  # lone donor ends (intron-level left_known without a partner)
                if rng.random() < 0.3:
                    p = lpos(x, cL)
                    out.append((p, p + 500, None) if rng.random() < 0.5 else (p + 500, p, None))
    return out


def c3_cached(reads: int, local_rank: int, seed_genome: int = 3, seed_reads: int = 33, scale: float = 1.0,
              cache_dir: str | None = None, timeout_s: float = 900.0):
    """The C3 genome and read batch, generated ONCE per node: local rank 0 builds
    them (c3_genome + c3_windows) into a cache directory (write, then rename, then
    a completion marker) and every rank maps the files read-only, so N ranks of
    one node share one copy in the page cache (1.16 GB of blocks + 0.4 GB of
    batch at the C3 size) instead of N private copies and N start-ups.
    Returns (PackedGenome, Batch)."""
    import hashlib
    import json
    import tempfile
    import time
    # the generator's own source names the cache, so an edit to c3_genome /
    # c3_windows (or anything else in this module) never reuses a stale copy
    with open(os.path.abspath(__file__), "rb") as f:
        gen = hashlib.sha1(f.read()).hexdigest()[:12]
    d = cache_dir or os.path.join(tempfile.gettempdir(), "gsnapdp_c3_g%d_r%d_s%g_n%d_%s" % (
        seed_genome, seed_reads, scale, reads, gen))
    done = os.path.join(d, "complete.json")
    failed = os.path.join(d, "error.json")
    names = ("blocks", "windows", "query", "query_uc")
    if not os.path.exists(done):
        if local_rank == 0:
            os.makedirs(d, exist_ok=True)
            try:
                g = c3_genome(seed=seed_genome, scale=scale)
                b = c3_windows(g, n=reads, seed=seed_reads)
                for k, a in zip(names, (g.blocks, b.windows, b.query, b.query_uc)):
                    tmp = os.path.join(d, k + ".tmp.npy")
                    np.save(tmp, a, allow_pickle=False)
                    os.replace(tmp, os.path.join(d, k + ".npy"))
            except BaseException as e:  # tell the waiting ranks instead of letting them time out
                with open(failed, "w") as f:
                    json.dump({"error": repr(e)}, f)
                raise
            with open(done + ".tmp", "w") as f:
                json.dump({"names": g.names, "lengths": [int(x) for x in g.lengths], "generator": gen}, f)
            os.replace(done + ".tmp", done)
        else:
            t0 = time.time()
            while not os.path.exists(done):
                if os.path.exists(failed):
                    raise RuntimeError("C3 cache %s: local rank 0 failed: %s" % (d, open(failed).read()))
                if time.time() - t0 > timeout_s:
                    raise RuntimeError("C3 cache %s not written by local rank 0 within %.0f s" % (d, timeout_s))
                time.sleep(0.2)
    meta = json.load(open(done))
    if meta.get("generator") != gen:
        raise RuntimeError("C3 cache %s was written by another generator (%s, this is %s)" % (
            d, meta.get("generator"), gen))
    a = {k: np.load(os.path.join(d, k + ".npy"), mmap_mode="r", allow_pickle=False) for k in names}
    return PackedGenome(a["blocks"], meta["names"], np.array(meta["lengths"], np.int64)), \
        Batch(a["windows"], a["query"], a["query_uc"])


def stage3_pipeline(z, copies: int = 1):
    """The path_compute calls of a recorded gmap run (tests/golden/gmap_*_stage3.npz,
    whose pass calls carry their path_compute `invocation`) as queries for
    gsnapdp_stage3_compute (passes 2A-6): each query is the invocation's first
    build_pairs_singles call (pass 2A: its path, query and arguments) with the
    final build_pairs_introns call's arguments and counters (pass 6).  Returns
    (queries, paths_in, query, query_uc, the lists pass 6 returned concatenated,
    the pass-6 calls, the pass counts per query before pass 6), `copies` times
    over; invocations without a final pass in the recording are left out."""
    from .records import S3_DUALBREAKS, S3_DUALINTRONS, S3_INTRONS, S3_SINGLES
    calls, pin, q, qu, want = stage3_calls(z)
    inv = calls["invocation"]
    order = np.argsort(inv, kind="stable")
    Q, P, W, F, counts = [], [], [], [], []
    at = 0
    for v in np.unique(inv):
        idx = order[inv[order] == v]
        cs = calls[idx]
        fin = np.nonzero((cs["pass"] == S3_INTRONS) & (cs["finalp"] == 1))[0]
        sg = np.nonzero(cs["pass"] == S3_SINGLES)[0]
        if fin.size != 1 or sg.size == 0 or sg[0] > fin[0]:
            continue
        first, last = cs[sg[0]], cs[fin[0]]
        before = cs[:fin[0] + 1]
        maj = before[np.isin(before["pass"], (S3_DUALINTRONS, S3_INTRONS))]
        k = last.copy()
        k["first_pair"], k["npairs"] = first["first_pair"], first["npairs"]
        k["qpos"], k["querylength"] = first["qpos"], first["querylength"]
        k["in_minor"], k["in_major"] = first["in_minor"], maj[0]["in_major"]
        ins = before[before["pass"] == S3_INTRONS][0]
        for f in ("in_nintrons", "in_nnonintrons", "in_intronlen", "in_nonintronlen"):
            k[f] = ins[f]
        k["finalp"] = 1
        Q.append(k)
        F.append(last)
        W.append(want[int(last["first_out"]):int(last["first_out"]) + int(last["nout"])])
        counts.append(np.bincount(before["pass"], minlength=6))
        at += 1
    queries = np.array(Q, dtype=calls.dtype)
    final = np.array(F, dtype=calls.dtype)
    wl = np.concatenate(W) if W else np.zeros(0, dtype=want.dtype)
    final["first_out"] = np.concatenate([[0], np.cumsum(final["nout"])[:-1]]).astype(np.int32)
    counts = np.array(counts)
    if copies > 1:
        n = len(queries)
        kk = np.repeat(np.arange(copies), n)
        queries = np.tile(queries, copies)
        queries["first_pair"] += (kk * pin.size).astype(np.int32)
        queries["qpos"] += (kk * q.size).astype(np.int32)
        final = np.tile(final, copies)
        final["first_out"] += (kk * wl.size).astype(np.int32)
        pin, q, qu, wl = np.tile(pin, copies), np.tile(q, copies), np.tile(qu, copies), np.tile(wl, copies)
        counts = np.tile(counts, (copies, 1))
    return queries, pin, q, qu, wl, final, counts


def stage3_path_pipeline(z, copies: int = 1):
    """The path_compute calls of a recorded gmap run (tests/golden/gmap_*_stage3.npz
    with its pc_calls / pc_pairs / pc_probs) as queries for
    gsnapdp_stage3_path_compute (pass 2A to path_compute's return value): each
    query is the invocation's first build_pairs_singles call (its path, query
    and arguments) with the last build_pairs_introns call's arguments, the
    counters at their first use, and path_compute's own arguments for passes
    7-10 (maxpeelback, extramaterial_end, extraband_end, do_final_p).  Returns
    (queries, paths_in, query, query_uc, the lists path_compute returned
    concatenated, their (donor_prob, acceptor_prob) rows, the PC_CALL records
    in query order), `copies` times over."""
    from .records import S3_DUALINTRONS, S3_INTRONS, S3_SINGLES
    calls, pin, q, qu, _ = stage3_calls(z)
    pc, pcp, pcr = z["pc_calls"], z["pc_pairs"], z["pc_probs"]
    inv = calls["invocation"]
    order = np.argsort(inv, kind="stable")
    Q, W_, R, F = [], [], [], []
    for rec in pc:
        v = int(rec["invocation"])
        idx = order[inv[order] == v]
        cs = calls[idx]
        sg = np.nonzero(cs["pass"] == S3_SINGLES)[0]
        intr = np.nonzero(cs["pass"] == S3_INTRONS)[0]
        if rec["stage3debug"] != 0 or sg.size == 0 or intr.size == 0 or sg[0] > intr[0]:
            continue
        first, last = cs[sg[0]], cs[intr[-1]]
        before = cs[:intr[-1] + 1]
        maj = before[np.isin(before["pass"], (S3_DUALINTRONS, S3_INTRONS))]
        k = last.copy()
        k["first_pair"], k["npairs"] = first["first_pair"], first["npairs"]
        k["qpos"], k["querylength"] = first["qpos"], first["querylength"]
        k["in_minor"], k["in_major"] = first["in_minor"], maj[0]["in_major"]
        ins = cs[intr[0]]
        for f in ("in_nintrons", "in_nnonintrons", "in_intronlen", "in_nonintronlen"):
            k[f] = ins[f]
        k["finalp"] = rec["do_final_p"]
        k["maxpeelback"], k["extramaterial_end"], k["extraband_end"] = (
            rec["maxpeelback"], rec["extramaterial_end"], rec["extraband_end"])
        Q.append(k)
        F.append(rec)
        W_.append(pcp[int(rec["first_out"]):int(rec["first_out"]) + int(rec["nout"])])
        R.append(pcr[int(rec["first_out"]):int(rec["first_out"]) + int(rec["nout"])])
    queries = np.array(Q, dtype=calls.dtype)
    final = np.array(F, dtype=pc.dtype)
    wl = np.concatenate(W_) if W_ else np.zeros(0, dtype=pcp.dtype)
    wr = np.concatenate(R) if R else np.zeros((0, 2), dtype=np.float64)
    final["first_out"] = np.concatenate([[0], np.cumsum(final["nout"])[:-1]]).astype(np.int32)
    if copies > 1:
        n = len(queries)
        kk = np.repeat(np.arange(copies), n)
        queries = np.tile(queries, copies)
        queries["first_pair"] += (kk * pin.size).astype(np.int32)
        queries["qpos"] += (kk * q.size).astype(np.int32)
        final = np.tile(final, copies)
        final["first_out"] += (kk * wl.size).astype(np.int32)
        pin, q, qu = np.tile(pin, copies), np.tile(q, copies), np.tile(qu, copies)
        wl, wr = np.tile(wl, copies), np.tile(wr, (copies, 1))
    return queries, pin, q, qu, wl, wr, final


def stage3_calls(z, copies: int = 1):
    """Unpack a recorded stage-3 pass (tests/golden/gmap_*_stage3.npz,
    oracle/gen_golden.py stage3_golden) into the inputs of
    Context.stage3_pass -- (calls, pairs_in, query, query_uc) -- and the lists
    the reference returned (concatenated, call by call), `copies` times over
    (every copy its own paths and query bytes)."""
    from .records import S3_PAIR
    calls = z["calls"].copy()
    pin = z["pairs_in"]
    src, flags, new = z["out_src"], z["out_flags"], z["out_new"]
    want = np.zeros(src.size, dtype=S3_PAIR)
    want[src < 0] = new
    at = 0
    for c in calls:
        n = int(c["nout"])
        s = src[at:at + n]
        keep = np.nonzero(s >= 0)[0]
        want[at + keep] = pin[int(c["first_pair"]) + s[keep]]
        want["src"][at + keep] = s[keep]
        want["flags"][at:at + n] = flags[at:at + n]
        at += n
    q, qu = z["query"], z["query_uc"]
    if copies > 1:
        n = len(calls)
        k = np.repeat(np.arange(copies), n)
        calls = np.tile(calls, copies)
        calls["first_pair"] += (k * pin.size).astype(np.int32)
        calls["qpos"] += (k * q.size).astype(np.int32)
        calls["first_out"] += (k * want.size).astype(np.int32)
        pin, q, qu, want = np.tile(pin, copies), np.tile(q, copies), np.tile(qu, copies), np.tile(want, copies)
    return calls, pin, q, qu, want


# ---------------------------------------------------------------------------
# BASELINE config 4 as stated: 50k synthetic 5 kbp transcripts through GMAP's
# final intron pass (build_pairs_introns with finalp, stage3.c:8860-8875) and
# score_introns (:9890-9941).  No gmapindex database or stage 2 exists here,
# so the generator builds what stage 2 + passes 1-5 hand to pass 6 directly:
# each transcript's path as insert_gapholders leaves it (stage3.c:817-900).

# donor and acceptor consensus in the transcript's (sense) coordinates:
# (anchor, offset, base); anchor 0 = the intron's first base, 1 = the base
# after its last one.  exon ..AG | GTAAGT ... (14 nt pyrimidine tract) CAG | G exon
_C4_DONOR = [(0, -2, "A"), (0, -1, "G"), (0, 0, "G"), (0, 1, "T"), (0, 2, "A"), (0, 3, "A"), (0, 4, "G"),
             (0, 5, "T")]
_C4_ACCEPTOR = [(1, -17 + i, b) for i, b in enumerate("TTTTCCCTTTCTTT")] + [(1, -3, "C"), (1, -2, "A"),
                                                                          (1, -1, "G"), (1, 0, "G")]
_CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


class C4Workload:
    """One pass-6 call per transcript (gsnapdp_s3_call records), the paths
    (gsnapdp_s3_pair, list order), the cDNAs, and the packed genome."""

    def __init__(self, blocks, calls, pairs_in, query, query_uc, nintrons, genome_nt):
        self.blocks, self.calls, self.pairs_in = blocks, calls, pairs_in
        self.query, self.query_uc = query, query_uc
        self.nintrons, self.genome_nt = nintrons, genome_nt


def c4_transcripts(n: int = 50_000, seed: int = 4, shift_frac: float = 0.3, weak_frac: float = 0.2,
                   sub_rate: float = 0.01, near: int = 15, chunk_genes: int = 2048) -> C4Workload:
    """BASELINE config 4: `n` synthetic transcripts of 4.5-5.5 kbp,
    8-12 exons, GT-AG introns of 80-5,000 nt, 1 % substitutions, a third of
    them antisense (the cDNA aligns to the plus strand with cdna_direction -1,
    CT-AC on the plus strand), on one genome of their gene regions.

    The path of each is what pass 6 (stage3.c:8860-8875) receives: one pair per
    aligned cDNA base in reversed alignment order (path->first is the last query
    base) and one gapholder per intron (queryjump 0, genomejump the intron span
    as insert_gapholders computes it, :868-871).  Stage 2 places ~30 % of the
    boundaries 1-6 nt off the true site (the cDNA bases there then sit in the
    intron), which pass 6 repairs; pairs within `near` of a boundary carry the
    negative dynprogindex and '*' comp an earlier intron pass leaves there, the
    rest '|' (or ' ' for a mismatch) and 0.  The donor / acceptor consensus is
    planted at every intron (weakened at `weak_frac` of them).

    Every parameter stream is its own generator ([seed, k]) drawn once per
    gene or base in order, so the first m transcripts of c4_transcripts(n) are
    c4_transcripts(m) for any n >= m (the reference pins a prefix)."""
    from .records import MAXLENGTH1, MAXLENGTH2, S3_CALL, S3_PAIR

    def S(k):
        return np.random.default_rng([seed, k])

    nex = S(1).integers(8, 13, size=n)
    T = S(2).integers(4500, 5501, size=n).astype(np.int64)
    ne, ni = int(nex.sum()), int(nex.sum()) - n
    gene_of_ex = np.repeat(np.arange(n), nex)
    first_ex = np.concatenate([[0], np.cumsum(nex)[:-1]])
    w = S(3).random(ne) * 1.4 + 0.3
    wsum = np.add.reduceat(w, first_ex)
    exl = np.maximum(30, np.floor(T[gene_of_ex] * w / wsum[gene_of_ex])).astype(np.int64)
    last = first_ex + nex - 1
    exl[last] += T - np.add.reduceat(exl, first_ex)
    assert exl.min() >= 30
    first_in = first_ex - np.arange(n)  # introns of gene i: first_in[i] .. + nex[i] - 1
    inl = S(4).integers(80, 5001, size=ni).astype(np.int64)
    anti = S(5).random(n) < 1 / 3
    u = S(6).random(ni)
    shift = np.where(u < shift_frac, S(7).integers(1, 7, size=ni) * np.where(S(8).random(ni) < 0.5, 1, -1), 0)
    weak = S(9).random(ni) < weak_frac
    # plus-strand layout: 600 nt, exon 0, intron 0, ..., exon m, 600 nt
    span = 1200 + np.add.reduceat(exl, first_ex) + np.add.reduceat(inl, first_in) * (nex > 1)
    gene_start = np.concatenate([[0], np.cumsum(span)[:-1]]).astype(np.int64)
    total = int(span.sum())
    exon_local = np.arange(ne) - first_ex[gene_of_ex]
    gene_of_in = np.repeat(np.arange(n), nex - 1)
    intron_local = np.arange(ni) - first_in[gene_of_in]
    # element lengths interleaved exon/intron per gene; exclusive sums within a gene
    el = np.zeros(ne + ni, dtype=np.int64)
    first_el = first_ex + first_in
    el[first_el[gene_of_ex] + 2 * exon_local] = exl
    el[first_el[gene_of_in] + 2 * intron_local + 1] = inl
    cs = np.cumsum(el) - el
    within = cs - cs[first_el][np.repeat(np.arange(n), 2 * nex - 1)]
    ex_start = gene_start[gene_of_ex] + 600 + within[first_el[gene_of_ex] + 2 * exon_local]
    in_start = gene_start[gene_of_in] + 600 + within[first_el[gene_of_in] + 2 * intron_local + 1]
    in_end = in_start + inl
    # the genome: random packed words (interleaved high / low), flags 0, X past the end
    nblocks = (total + 31) // 32
    hl = S(10).integers(0, 1 << 32, size=2 * nblocks, dtype=np.uint32)
    blocks = np.empty(3 * nblocks + 4, dtype=np.uint32)
    blocks[0:3 * nblocks:3] = hl[0::2]
    blocks[1:3 * nblocks:3] = hl[1::2]
    blocks[2:3 * nblocks:3] = 0
    blocks[3 * nblocks:] = 0xFFFFFFFF
    del hl
    tail = nblocks * 32 - total
    for b in range(32 - tail, 32):
        blocks[3 * (nblocks - 1) + 2] |= np.uint32(1) << np.uint32(b)
        word = 3 * (nblocks - 1) + (1 if b < 16 else 0)
        blocks[word] |= np.uint32(3) << np.uint32(2 * (b & 15))

    def plant(pos, code):  # one base per intron at a time: distinct words
        pos = np.asarray(pos, dtype=np.int64)
        bit = (pos & 31).astype(np.uint32)
        word = (pos >> 5) * 3 + np.where(bit < 16, 1, 0)
        sh = (2 * (bit & 15)).astype(np.uint32)
        blocks[word] = (blocks[word] & ~(np.uint32(3) << sh)) | (np.asarray(code, np.uint32) << sh)

    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    keep_weak_tract = np.arange(14) % 2 == 0
    for motif in (_C4_DONOR, _C4_ACCEPTOR):
        for j, (anchor, off, base) in enumerate(motif):
            sel = np.ones(ni, bool)
            if motif is _C4_DONOR and off >= 2:
                sel = ~weak  # weak donors keep random +3..+5 (and +2)
            if motif is _C4_ACCEPTOR and j < 14:
                sel = ~weak | keep_weak_tract[j]
            a = in_start[sel]
            b = in_end[sel]
            an = anti[gene_of_in[sel]]
            site = np.where(anchor == 0, a, b)
            other = np.where(anchor == 0, b, a)
            # antisense: sense offset `off` from the sense anchor, mirrored on the plus strand
            pos = np.where(an, other - 1 - off, site + off)
            code = np.where(an, _CODE[comp[base]], _CODE[base])
            plant(pos, code)
    # pass-6 calls
    calls = np.zeros(n, dtype=S3_CALL)
    npairs = T + (nex - 1)
    calls["npairs"] = npairs
    calls["first_pair"] = np.concatenate([[0], np.cumsum(npairs)[:-1]])
    qlen_pad = T + 8 - (T & 3)
    calls["qpos"] = np.concatenate([[0], np.cumsum(qlen_pad)[:-1]])
    calls["querylength"] = T
    calls["chroffset"] = 0
    calls["chrhigh"] = total
    calls["chrpos"] = gene_start
    calls["chrnum"] = 1
    calls["genomiclength"] = span
    calls["cdna_direction"] = np.where(anti, -1, 1)
    calls["watsonp"] = 1
    calls["finalp"] = 1
    for f, v in (("maxpeelback", 11), ("nullgap", 600), ("extramaterial_paired", 8), ("extraband_single", 3),
                 ("extraband_paired", 7), ("close_indels_mode", 1), ("novelsplicingp", 1), ("splicingp", 1)):
        calls[f] = v
    calls["defect_rate"] = sub_rate
    calls["maxlength1"] = MAXLENGTH1
    calls["maxlength2"] = MAXLENGTH2
    calls["in_minor"] = 1
    calls["in_major"] = -nex
    if total >= 1 << 31:
        raise ValueError("C4 genome of %d nt does not fit Genomicpos_T arithmetic on int32 paths" % total)
    pairs = np.zeros(int(npairs.sum()), dtype=S3_PAIR)
    query = np.zeros(int(qlen_pad.sum()), dtype=np.uint8)
    rs, rk = S(11), S(12)  # substitutions: one draw per cDNA base, in order
    qstart_ex = np.concatenate([[0], np.cumsum(exl)[:-1]]) - np.repeat(np.concatenate([[0], np.cumsum(T)[:-1]]), nex)
    for g0 in range(0, n, chunk_genes):
        g1 = min(n, g0 + chunk_genes)
        e0, e1 = int(first_ex[g0]), int(first_ex[g1 - 1] + nex[g1 - 1])
        i0, i1 = int(first_in[g0]), int(first_in[g1 - 1] + nex[g1 - 1] - 1)
        # every cDNA base of the chunk: its gene, query position and true genome position
        L = exl[e0:e1]
        gq = np.repeat(gene_of_ex[e0:e1], L)
        q = np.repeat(qstart_ex[e0:e1], L) + (np.arange(int(L.sum())) - np.repeat(np.cumsum(L) - L, L))
        gpos = np.repeat(ex_start[e0:e1], L) + (np.arange(int(L.sum())) - np.repeat(np.cumsum(L) - L, L))
        base = decode_blocks(blocks, gpos)
        m = rs.random(base.size) < sub_rate
        k = rk.integers(1, 4, size=base.size)
        cd = np.where(m, ACGT[(np.searchsorted(ACGT, base) + k) % 4], base).astype(np.uint8)
        # stage 2's boundary placement: the path's genome position of every cDNA base
        qb_true = (qstart_ex[e0:e1] + exl[e0:e1])[np.setdiff1d(np.arange(e1 - e0), last[g0:g1] - e0)]
        ig = np.arange(i0, i1)
        s = shift[ig]
        pg = gpos.copy()
        qofs = np.concatenate([[0], np.cumsum(T[g0:g1])[:-1]])  # chunk-local offset of each gene's bases
        gl = gene_of_in[ig] - g0
        for d in range(1, 7):
            pos_ = s >= d  # exon e continues d-1 bases into the intron
            idx = qofs[gl[pos_]] + qb_true[pos_] + (d - 1)
            pg[idx] = in_start[ig[pos_]] + (d - 1)
            neg = -s >= d  # exon e+1 starts d bases early, at the intron's end
            idx = qofs[gl[neg]] + qb_true[neg] - d
            pg[idx] = in_end[ig[neg]] - d
        qb = qb_true + s  # the path's boundary: first query base after the gap
        gch = decode_blocks(blocks, pg)
        # distance to the gene's nearest boundary, for dynprogindex / comp
        near_mask = np.zeros(base.size, bool)
        dpi = np.zeros(base.size, np.int32)
        for d in range(-near, near):
            idx = qofs[gl] + qb + d
            ok = (qb + d >= 0) & (qb + d < T[g0:g1][gl])
            near_mask[idx[ok]] = True
            dpi[idx[ok]] = -(intron_local[ig][ok] + 1)
        match = cd == gch
        # list order: path->first is the last query base; gap k of a gene sits after
        # the pair of its boundary qb_k (ascending k): before pair q lie the
        # T-1-q later pairs and the gaps whose boundary is > q
        nb_after = np.zeros(base.size, np.int64)  # gaps with qb > q, per base
        gap_rank = (nex[gene_of_in[ig]] - 2) - intron_local[ig]  # = #(qb' > qb_k) within the gene
        np.add.at(nb_after, qofs[gl] + qb - 1, 1)
        # suffix counts within each gene: gaps with boundary > q  = sum over q' >= q of marks at qb-1
        rev_cum = np.cumsum(nb_after[::-1])[::-1]
        gstart_chunk = np.repeat(qofs, T[g0:g1])
        gend_total = np.repeat(np.append(rev_cum[qofs[1:]], 0) if g1 - g0 > 1 else np.array([0]), T[g0:g1])
        after = rev_cum - gend_total  # marks at q' >= q within the gene = gaps with qb > q
        fp = calls["first_pair"][gq]
        lpos = fp + (T[gq] - 1 - q) + after
        rec = pairs[lpos] if False else None  # (written field by field below)
        pairs["querypos"][lpos] = q
        pairs["genomepos"][lpos] = pg - gene_start[gq]
        pairs["dynprogindex"][lpos] = np.where(near_mask, dpi, 0)
        pairs["cdna"][lpos] = cd
        pairs["genome"][lpos] = gch
        pairs["comp"][lpos] = np.where(match, np.where(near_mask, ord("*"), ord("|")), ord(" "))
        pairs["src"][lpos] = 0
        # gapholders: after the pair of qb (list order), between qb - 1 and qb
        gg = gene_of_in[ig]
        gpos_hi = pg[qofs[gl] + qb]
        gpos_lo = pg[qofs[gl] + qb - 1]
        gl_pos = calls["first_pair"][gg] + (T[gg] - qb) + gap_rank
        pairs["querypos"][gl_pos] = -1
        pairs["genomepos"][gl_pos] = -1
        pairs["queryjump"][gl_pos] = 0
        pairs["genomejump"][gl_pos] = gpos_hi - gpos_lo - 1
        pairs["cdna"][gl_pos] = ord(" ")
        pairs["comp"][gl_pos] = ord(" ")
        pairs["genome"][gl_pos] = ord(" ")
        pairs["flags"][gl_pos] = 1  # GSNAPDP_S3_GAPP
        # the cDNA bytes
        qp = calls["qpos"][gq] + q
        query[qp] = cd
    calls["first_pair"] = calls["first_pair"]  # (records are final)
    return C4Workload(blocks, calls, pairs, query, query.copy(), int(ni), total)
