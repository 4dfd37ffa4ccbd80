"""k_fill scratch-traffic ablation (diagnostics): K device-resident steps of
the C2 batch (100k x 150 bp, 64 Mbp genome) through whichever library
GSNAPDP_LIB names, for rocprofv3 --kernel-trace / --pmc passes
(tools/traffic_ablate.sh).  Variants built by tools/build_variant.sh:
EXP_NOMATCH (no match-byte stores), EXP_NOTRACE (no traceback: no scratch
reads), EXP_NOSTORE + EXP_NOTRACE (no scratch at all)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
import torch  # noqa: E402

from gsnapdp import Context, op_offsets  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import RESULT  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
genome = W.synthetic_genome(64_000_000, seed=1)
batch = W.c2_windows(genome, n=100_000, seed=2)
n = len(batch)
off = op_offsets(batch.windows)
ctx = Context(W.pack_genome(genome))
dev = torch.device("cuda", 0)
d_w = torch.from_numpy(batch.windows.view(np.uint8).copy()).to(dev)
d_q = torch.from_numpy(batch.query.copy()).to(dev)
d_off = torch.from_numpy(off.copy()).to(dev)
d_res = torch.zeros(n * RESULT.itemsize, dtype=torch.uint8, device=dev)
d_ops = torch.zeros(int(off[-1]) + 1, dtype=torch.int32, device=dev)
for _ in range(K):
    ctx.run_device(d_w.data_ptr(), n, d_q.data_ptr(), d_q.data_ptr(), d_res.data_ptr(), d_ops.data_ptr(),
                   d_off.data_ptr())
ctx.sync()
print("ok", os.environ.get("GSNAPDP_LIB", "default"), K, "steps", flush=True)
