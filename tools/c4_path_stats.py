"""The C4 transcript generator's paths (workload.c4_transcripts) beside the
paths the reference's gmap handed its final intron pass (build_pairs_introns
with finalp, stage3.c:8860) in a recorded run (tools/make_stage3_trace.py):
per path the query length, the gaps (gapholders), the exon lengths between
them, the genome jump of each gap, and the pairs per path.
usage: python tools/c4_path_stats.py TRACE.npz [N] > profiles/..._c4_path_stats.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import workload as W  # noqa: E402


def stats(calls, pairs_in):
    qlen, ngaps, exon, jump, npairs = [], [], [], [], []
    for c in calls:
        x = pairs_in[int(c["first_pair"]):int(c["first_pair"]) + int(c["npairs"])]
        g = (x["flags"] & 1) != 0
        qlen.append(int(c["querylength"]))
        npairs.append(int(c["npairs"]))
        ngaps.append(int(g.sum()))
        jump.extend(int(v) for v in x["genomejump"][g])
        idx = np.flatnonzero(g)
        bounds = np.concatenate([[-1], idx, [len(x)]])
        exon.extend(int(b - a - 1) for a, b in zip(bounds[:-1], bounds[1:]) if b - a - 1 > 0)

    def q(v):
        v = np.asarray(v, dtype=np.float64)
        return {"n": int(v.size), "mean": round(float(v.mean()), 1), "p10": float(np.percentile(v, 10)),
                "p50": float(np.percentile(v, 50)), "p90": float(np.percentile(v, 90))} if v.size else {"n": 0}
    return {"paths": len(calls), "querylength": q(qlen), "pairs_per_path": q(npairs), "gaps_per_path": q(ngaps),
            "exon_pairs": q(exon), "gap_genomejump": q(jump)}


def main():
    z = np.load(sys.argv[1], allow_pickle=False)
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    c = z["calls"]
    fin = c[(c["pass"] == 0) & (c["finalp"] == 1)]
    w = W.c4_transcripts(n)
    print(json.dumps({"trace": os.path.basename(sys.argv[1]),
                      "gmap_final_intron_pass": stats(fin, z["pairs_in"]),
                      "c4_transcripts": stats(w.calls, w.pairs_in)}, indent=1))


if __name__ == "__main__":
    main()
