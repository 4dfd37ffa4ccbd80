"""gsnap linked against the drop-in (north_star: "gmap.c and gsnap.c link against it").

``make -C oracle gsnap`` (dev container only) compiles the reference's
``GSNAP_FILES`` (``src/Makefile.am:50-84``) with gsnap's own defines
(``-DGSNAP=1 -DMAX_READLENGTH=250``, pthreads) and links them against
``libgsnapdp_dropin.so`` in place of ``dynprog.o`` / ``maxent_hr.o`` /
``genome_hr.o``, with ``-Wl,--no-undefined``.  The genome_hr mismatch functions
live in the reference's missing ``genome_hr.c`` blob and get aborting stand-ins
(``oracle/gsnap_stubs.c``); gsnap only reaches them on a gmapindex database,
which is out of scope.  The program itself never travels to the GPU box.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GSNAP = os.path.join(ROOT, "oracle", "_ref", "gsnap_gpu")
GMAP = os.path.join(ROOT, "oracle", "_ref", "gmap_gpu")
DROPIN = os.path.join(ROOT, "gmap-gsnap_amd", "lib", "libgsnapdp_dropin.so")


def need(path):
    if not os.path.exists(path):
        pytest.skip("%s not built (make -C oracle ref, dev container)" % path)


def dynsyms(path, undefined):
    out = subprocess.run(["nm", "-D", "--undefined-only" if undefined else "--defined-only", path],
                         capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


@pytest.mark.parametrize("program", [GSNAP, GMAP], ids=["gsnap", "gmap"])
def test_program_takes_every_dp_symbol_from_the_dropin(program):
    need(program)
    need(DROPIN)
    needed = {s for s in dynsyms(program, True) if re.match(r"(Dynprog_|Maxent_hr_|Genome_hr_|Genome_prev_)", s)}
    assert any(s.startswith("Dynprog_") for s in needed)
    assert "Maxent_hr_setup" in needed and "Dynprog_setup" in needed
    missing = needed - dynsyms(DROPIN, False)
    assert not missing, missing
    # the program defines none of them itself (no dynprog.o / maxent_hr.o linked in)
    own = {s for s in dynsyms(program, False) if re.match(r"(Dynprog_|Maxent_hr_)", s)}
    assert not own, own
    # ... and resolves them at load time in the drop-in
    ldd = subprocess.run(["ldd", program], capture_output=True, text=True).stdout
    assert "libgsnapdp_dropin.so" in ldd and "not found" not in ldd, ldd


def test_gsnap_starts_against_the_dropin():
    need(GSNAP)
    r = subprocess.run([GSNAP, "--version"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "GSNAP" in (r.stdout + r.stderr) and "2012-07-03" in (r.stdout + r.stderr)
