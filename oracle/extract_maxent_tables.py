#!/usr/bin/env python3
"""Extract the MaxEnt parameter tables used by Maxent_hr_* into a binary blob.

The 16 ``static const double`` arrays of reference src/maxent_hr.c:25-22606
(12 x 16384 + 4 x 16 doubles = 1,573,376 bytes) are model parameters, not
derivable from anything else.  This script parses the
literals (decimal -> IEEE double, correctly rounded like the C compiler) and
writes them in declaration order as little-endian float64.  It runs in the
development container only (it needs /root/reference); the blob it writes is
git-ignored and travels to the GPU box with the working tree.

Usage: extract_maxent_tables.py [maxent_hr.c] [out.bin]
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

NAMES = [
    "donor_score_plus", "donor_discore_plus", "acc_score1_plus", "acc_score2_plus",
    "acc_score3_plus", "acc_discore_plus", "acc_score467_plus", "acc_score589_plus",
    "donor_score_minus", "donor_discore_minus", "acc_score1_minus", "acc_score2_minus",
    "acc_score3_minus", "acc_discore_minus", "acc_score467_minus", "acc_score589_minus",
]
LENGTHS = [16384, 16, 16384, 16384, 16384, 16, 16384, 16384] * 2

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_SRC = "/root/reference/src/maxent_hr.c"
DEFAULT_OUT = os.path.join(HERE, "..", "gmap-gsnap_amd", "data", "maxent_hr_tables.bin")


def extract(src: str) -> np.ndarray:
    text = open(src, "r", encoding="latin-1").read()
    out = []
    for name, n in zip(NAMES, LENGTHS):
        m = re.search(r"static\s+const\s+double\s+%s\s*\[\s*(\d+)\s*\]\s*=\s*\{" % name, text)
        if not m or int(m.group(1)) != n:
            raise SystemExit("table %s not found with length %d" % (name, n))
        body = text[m.end(): text.index("}", m.end())]
        vals = [float(x) for x in body.replace("\n", " ").split(",") if x.strip()]
        if len(vals) != n:
            raise SystemExit("table %s: parsed %d values, expected %d" % (name, len(vals), n))
        out.append(np.array(vals, dtype="<f8"))
    return np.concatenate(out)


def main() -> None:
    src = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_SRC
    dst = sys.argv[2] if len(sys.argv) > 2 else DEFAULT_OUT
    tabs = extract(src)
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    tabs.tofile(dst)
    print("wrote %s (%d doubles)" % (dst, tabs.size))


if __name__ == "__main__":
    main()
