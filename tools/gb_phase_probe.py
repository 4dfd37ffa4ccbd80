import os, sys
sys.path.insert(0, "gmap-gsnap_amd")
import numpy as np
from gsnapdp import Context
z = np.load("tests/golden/ggap_chr17.npz", allow_pickle=False)
ctx = Context(z["blocks"])
res, trc, ops, off = ctx.ggap_run(z["windows"], z["query"], z["query_uc"])
print("phases", os.environ.get("GSNAPDP_GB_PHASES"), "ok", int((res["finalscore"] == z["results"]["finalscore"]).sum()), len(res), flush=True)
