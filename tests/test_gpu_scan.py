"""GSNAP's splice-site scans batched (gsnapdp_scan_site_probs; stage1hr.c:6300-7046,
8703-8976): every candidate of many reads in one call.  Pinned by the
reference's own Maxent_hr_* outputs (tests/golden/maxent_*.npz, made by
oracle/_ref/ref_driver): each golden position is split into a scan's
segment_left + splice_pos, and about a fifth of the sites are marked known
(knowni >= 0), for which the scans take 1.0 without a model run."""
import os

import numpy as np
import pytest

from gsnapdp import Context
from gsnapdp.records import SCAN_SITE

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["maxent_chr17", "maxent_synth"])
def test_gpu_scan_site_probs_match_reference(golden_dir, name):
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    rng = np.random.default_rng(17)
    n = z["model"].size
    s = np.zeros(n, dtype=SCAN_SITE)
    sp = np.minimum(rng.integers(0, 300, size=n), z["splice_pos"]).astype(np.int32)
    s["splice_pos"] = sp
    s["segment_left"] = z["splice_pos"] - sp.astype(np.uint32)
    s["chroffset"] = z["chroffset"]
    s["model"] = z["model"]
    known = rng.random(n) < 0.2
    s["knowni"] = np.where(known, rng.integers(0, 1000, size=n), -1)
    ctx = Context(z["blocks"])
    got = ctx.scan_site_probs(s)
    want = np.where(known, 1.0, z["prob"])
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, "%s: %d sites differ, first %s" % (name, bad.size, bad[:8])
    ctx.close()
