"""CPU-only checks of the product library: it is built for gfx950, loads,
exports every symbol include/gsnapdp.h declares, and its record layouts are
the ones the Python mirror and the oracle use."""
import os
import re
import subprocess

import numpy as np
import pytest

import gsnapdp
from gsnapdp.records import GGAP_RESULT, GGAP_TRACE, GGAP_WINDOW, PAIR, RESULT, WINDOW

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
                   'sizeof(gsnapdp_ggap_result), sizeof(gsnapdp_ggap_trace));return 0;}\n' % ROOT)
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert sizes == [WINDOW.itemsize, RESULT.itemsize, PAIR.itemsize, GGAP_WINDOW.itemsize,
                     GGAP_RESULT.itemsize, GGAP_TRACE.itemsize]


def test_no_gpu_means_loud_failure():
    """Without a gfx950 device the context must fail loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(gsnapdp.GsnapdpError):
        gsnapdp.Context(np.zeros(64, np.uint32))
