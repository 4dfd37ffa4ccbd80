"""Host-side logic that needs no GPU: genome packing, workload generators."""
import os

import numpy as np
import pytest

from gsnapdp import genome as G
from gsnapdp import workload as W


def test_pack_matches_reference_fixture():
    ref = "/root/reference/tests"
    if not os.path.exists(os.path.join(ref, "setup.genomecomp.ok")):
        pytest.skip("reference test fixtures not present on this machine")
    s = G.read_fasta(os.path.join(ref, "ss.chr17test"))
    b = G.pack(s)
    ok = np.fromfile(os.path.join(ref, "setup.genomecomp.ok"), dtype="<u4")
    assert np.array_equal(b[:ok.size], ok)


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    s = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, 10_000)]
    b = G.pack(s)
    assert G.unpack(b, 0, s.size) == s.tobytes()
    assert G.unpack(b, 1234, 77) == s[1234:1311].tobytes()


def test_c2_windows_shape_and_determinism():
    g = W.synthetic_genome(200_000, seed=1)
    a = W.c2_windows(g, n=500, seed=2)
    b = W.c2_windows(g, n=500, seed=2)
    assert np.array_equal(a.windows, b.windows) and np.array_equal(a.query, b.query)
    assert np.all(a.windows["length1"] == 150)
    d = a.windows["length2"] - 150
    assert set(np.unique(d)) <= {-3, -2, -1, 0, 1, 2, 3}
    assert 0.2 < np.mean(d != 0) < 0.4
    assert np.all(a.windows["extraband"] == 15)
