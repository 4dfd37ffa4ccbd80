"""A recorded gmap run for the stage-3 throughput side lines (not committed:
bigdata/, git-ignored): synthetic spliced cDNAs (workload.synthetic_transcripts)
aligned by the reference's own gmap with every stage-3 pass call recorded
(oracle/_ref/gmap_trace), packed like the stage-3 goldens (every pass call,
path_compute invocations, traverse_dual_break's stage-2 lists).  Dev container
only (needs oracle/_ref).

    python tools/make_stage3_trace.py [NGENES] [GENOME_LEN] [SEED]  ->  bigdata/gmap_<NGENES>_stage3.npz"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gen_golden as G  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import S2_CALL, S3_PAIR  # noqa: E402


def main():
    ngenes = int(sys.argv[1]) if len(sys.argv) > 1 else 274
    glen = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 274
    g, qs = W.synthetic_transcripts(seed=seed, ngenes=ngenes, genome_len=glen)
    out = os.path.join(ROOT, "bigdata", "gmap_%d_stage3.npz" % len(qs))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        W.write_fasta(os.path.join(d, "g.fa"), [("synthchr", g)])
        W.write_fasta(os.path.join(d, "q.fa"), qs)
        env = dict(os.environ, GMAP_TRACE_DIR=os.path.join(d, "trace"))
        subprocess.run([G.GMAP_TRACE, "-A", "-g", os.path.join(d, "g.fa"), os.path.join(d, "q.fa")], env=env,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
        t = os.path.join(d, "trace", "bpi")
        blocks = np.fromfile(os.path.join(d, "trace", "dp", "genome.u32"), dtype="<u4")
        c, pi, po, q, qu = G.stage3_trace(t)
        dd = G.stage3_pack(c, pi, po, q, qu)
        np.savez_compressed(out, blocks=blocks, ncalls_traced=np.int32(c.size),
                            s2_calls=np.fromfile(os.path.join(t, "stage2_calls.bin"), dtype=S2_CALL),
                            s2_pairs=np.fromfile(os.path.join(t, "stage2_pairs.bin"), dtype=S3_PAIR),
                            **dict(zip(("pc_calls", "pc_pairs", "pc_probs"), G.path_compute_trace(t))), **dd)
    print("%s: %d cDNAs, %d pass calls (by pass %s), %d path pairs, reference %.3f s" %
          (out, len(qs), c.size, np.bincount(c["pass"], minlength=6).tolist(), dd["pairs_in"].size,
           float(c["ref_seconds"].sum())))


if __name__ == "__main__":
    main()
