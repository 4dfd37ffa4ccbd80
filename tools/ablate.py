"""Per-stage timing of the C2 bench workload (C3 with ABLATE_C3=1) for one library build (diagnostics)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch
from gsnapdp import Context, op_offsets
from gsnapdp import workload as W
from gsnapdp.records import RESULT

if os.environ.get("ABLATE_C3") == "1":  # the headline batch (bench.py's C3, node-cached)
    g3, batch = W.c3_cached(int(os.environ.get("ABLATE_READS", "1000000")), 0)
    blocks = g3.blocks
else:
    genome = W.synthetic_genome(64_000_000, seed=1)
    blocks = W.pack_genome(genome)
    batch = W.c2_windows(genome, n=100_000, seed=2, indel_frac=float(os.environ.get("INDEL_FRAC", "0.3")))
n = len(batch)
off = op_offsets(batch.windows)
ctx = Context(blocks, mode=0, device=0)
dev = torch.device("cuda", 0)
d_w = torch.from_numpy(batch.windows.view(np.uint8).copy()).to(dev)
d_q = torch.from_numpy(batch.query.copy()).to(dev)
d_u = torch.from_numpy(batch.query_uc.copy()).to(dev)
d_off = torch.from_numpy(off.copy()).to(dev)
d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
step = lambda: ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_u.data_ptr(), d_res.data_ptr(), d_ops.data_ptr(), d_off.data_ptr())
for _ in range(3):
    step()
ctx.sync()
names = ctx.profile(True)
K = int(os.environ.get("ABLATE_STEPS", "40"))
rows = []
for _ in range(K):
    acc = np.zeros(len(names))
    step()
    ctx.profile_read(acc)
    rows.append(acc)
med = np.median(np.array(rows), axis=0)  # per-stage median over the steps (ms)
print(os.environ.get("GSNAPDP_LIB", "default"), json.dumps({k: round(v, 4) for k, v in zip(names, med) if v > 0}))
