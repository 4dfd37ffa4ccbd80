"""Packed-genome codec (host side).

The device-resident genome is the reference's ``.genomecomp`` block format,
unchanged: one block of three little-endian uint32 ``(high, low, flags)`` per
32 nt; nt *i* of a block is 2 bits at ``low >> 2i`` (i < 16) or
``high >> 2(i-16)``, A=0 C=1 G=2 T=3, and flag bit *i* marks a non-ACGT base
(N = A+flag, X = T+flag).  Writer: ``write_compressed_one``
(reference src/compress.c:321-365); reader: ``uncompress_one_char``
(src/genome.c:9325-9360); allocation with trailing X block and 4 guard words:
``Genome_create_blocks`` (src/genome-write.c:805-829).
"""
from __future__ import annotations

import numpy as np

_CODE = np.full(256, 0, dtype=np.uint32)
_FLAG = np.ones(256, dtype=np.uint32)  # unknown characters become N (compress.c:346-356)
for _ch, _c, _f in (("A", 0, 0), ("C", 1, 0), ("G", 2, 0), ("T", 3, 0), ("N", 0, 1), ("X", 3, 1)):
    for _x in (_ch, _ch.lower()):
        _CODE[ord(_x)] = _c
        _FLAG[ord(_x)] = _f


def pack(seq: bytes | np.ndarray) -> np.ndarray:
    """Pack a nucleotide string into genome blocks (+4 guard words of 0xFFFFFFFF).

    Positions past the end of the sequence in the last block are X, as in
    Genome_create_blocks.
    """
    s = np.frombuffer(bytes(seq), dtype=np.uint8) if not isinstance(seq, np.ndarray) else seq.astype(np.uint8)
    n = s.size
    nblocks = (n + 31) // 32
    codes = np.full(nblocks * 32, 3, dtype=np.uint32)  # X tail
    flags = np.ones(nblocks * 32, dtype=np.uint32)
    codes[:n] = _CODE[s]
    flags[:n] = _FLAG[s]
    codes = codes.reshape(nblocks, 32)
    flags = flags.reshape(nblocks, 32)
    shifts = (2 * np.arange(16, dtype=np.uint32))[None, :]
    low = np.bitwise_or.reduce(codes[:, :16] << shifts, axis=1).astype(np.uint32)
    high = np.bitwise_or.reduce(codes[:, 16:] << shifts, axis=1).astype(np.uint32)
    fl = np.bitwise_or.reduce(flags << np.arange(32, dtype=np.uint32)[None, :], axis=1).astype(np.uint32)
    out = np.empty(nblocks * 3 + 4, dtype=np.uint32)
    out[0:nblocks * 3:3] = high
    out[1:nblocks * 3:3] = low
    out[2:nblocks * 3:3] = fl
    out[nblocks * 3:] = 0xFFFFFFFF
    return out


def unpack(blocks: np.ndarray, start: int, length: int) -> bytes:
    """Decode ``length`` nt from ``start`` exactly like uncompress_one_char."""
    pos = np.arange(start, start + length, dtype=np.uint64)
    ptr = (pos // 32) * 3
    bit = (pos % 32).astype(np.uint32)
    flags = blocks[ptr + 2]
    low = blocks[ptr + 1]
    high = blocks[ptr]
    word = np.where(bit < 16, low, high)
    sh = np.where(bit < 16, 2 * bit, 2 * bit - 32).astype(np.uint32)
    c = (word >> sh) & 3
    ch = np.frombuffer(b"ACGT", dtype=np.uint8)[c]
    ch = np.where(((flags >> bit) & 1) == 1, ord("N"), ch).astype(np.uint8)
    return ch.tobytes()


def read_fasta(path: str) -> bytes:
    seq = []
    with open(path, "rb") as f:
        for line in f:
            if line.startswith(b">"):
                continue
            seq.append(line.strip())
    return b"".join(seq)
