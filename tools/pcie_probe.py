"""The host-buffer boundary on one 100k-read C2 batch (page-locked buffers):
wall time per gsnapdp_run_host call, for rocprofv3 --kernel-trace
--memory-copy-trace (which copies and kernels the call is made of).  GPU box only."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
from gsnapdp import Context, op_offsets, pinned_copy, pinned_empty  # noqa: E402
from gsnapdp import workload as W  # noqa: E402
from gsnapdp.records import RESULT  # noqa: E402

g = W.synthetic_genome(64_000_000, seed=1)
b = W.c2_windows(g, n=100_000, seed=2)
ctx = Context(W.pack_genome(g))
hw, hq, hu = pinned_copy(b.windows), pinned_copy(b.query), pinned_copy(b.query_uc)
hoff = pinned_copy(op_offsets(hw))
hres, hops = pinned_empty(len(hw), RESULT), pinned_empty(int(hoff[-1]) + 1, np.uint32)
print("H2D bytes: windows %d, query 2 x %d, offsets %d" % (hw.nbytes, hq.nbytes, hoff.nbytes))
for rep in range(8):
    t = time.perf_counter()
    ctx.run(hw, hq, hu, out=(hres, hops, hoff))
    print("run_host %.3f ms" % (1000 * (time.perf_counter() - t)), flush=True)
