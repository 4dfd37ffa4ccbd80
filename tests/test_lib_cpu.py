"""CPU-only checks of the product library: it is built for gfx950, loads,
exports every symbol include/gsnapdp.h declares, and its record layouts are
the ones the Python mirror and the oracle use."""
import os
import re
import subprocess

import numpy as np
import pytest

import gsnapdp
from gsnapdp.records import (GGAP_RESULT, GGAP_TRACE, GGAP_WINDOW, INTRON, INTRON_PATH, INTRON_SCORES, PAIR,
                             PATH_PAIR, RESULT, WINDOW)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "gsnapdp.h")).read()
    return sorted(set(re.findall(r"\b(gsnapdp_[a-z_0-9]+)\s*\(", txt)))


def test_library_loads_and_exports_abi():
    L = gsnapdp.lib()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), "missing export %s" % s


def test_library_targets_gfx950_only():
    blob = open(os.path.join(ROOT, "gmap-gsnap_amd", "lib", "libgsnapdp.so"), "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}


def test_record_layouts_match_c(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "%s/include/gsnapdp.h"\n'
                   'int main(){printf("%%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(gsnapdp_window), '
                   'sizeof(gsnapdp_result), sizeof(gsnapdp_pair), sizeof(gsnapdp_ggap_window), '
                   'sizeof(gsnapdp_ggap_result), sizeof(gsnapdp_ggap_trace));'
                   'printf("%%zu %%zu %%zu %%zu\\n", sizeof(gsnapdp_path_pair), sizeof(gsnapdp_intron), '
                   'sizeof(gsnapdp_intron_path), sizeof(gsnapdp_intron_scores));return 0;}\n' % ROOT)
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert sizes == [WINDOW.itemsize, RESULT.itemsize, PAIR.itemsize, GGAP_WINDOW.itemsize,
                     GGAP_RESULT.itemsize, GGAP_TRACE.itemsize, PATH_PAIR.itemsize, INTRON.itemsize,
                     INTRON_PATH.itemsize, INTRON_SCORES.itemsize]


def test_no_gpu_means_loud_failure():
    """Without a gfx950 device the context must fail loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(gsnapdp.GsnapdpError):
        gsnapdp.Context(np.zeros(64, np.uint32))


@pytest.mark.parametrize("name", ["gmap_her2_introns", "gmap_synth_introns"])
def test_path_introns_host_walk_matches_restatement(golden_dir, name):
    """gsnapdp_path_introns (product host code, no GPU) picks the same introns,
    with the same flanking pairs, as the restatement of score_introns' walk
    (pinned to the reference by test_oracle_golden) on every recorded path."""
    import oracle as O
    from test_oracle_golden import golden_intron_paths
    z = np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)
    p1, i1 = golden_intron_paths(z, gsnapdp.path_introns)
    p2, i2 = golden_intron_paths(z, O.path_introns)
    assert p1.tobytes() == p2.tobytes() and i1.tobytes() == i2.tobytes() and i1.size > 0
