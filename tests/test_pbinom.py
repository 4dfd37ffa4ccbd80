"""Pbinom (pbinom.c:1680), the one floating-point function that decides a list
in path_compute's host steps: chop_ends_by_changepoint trims an end when
Pbinom(k, n, theta) is not above TRIM_END_PVALUE = 1e-4 (stage3.c:2130-2306).
The product restates GSL 1.8's incomplete-beta path as the reference carries it
(gsnapdp_stage3_compute.cpp); this compares it bit for bit with the reference's
own pbinom.c, compiled from its source (oracle/Makefile pbinom_check), over
4 million arguments: every k of every n <= 300 on a 45-point theta grid, the k
around the 1e-4 crossing for every n <= 5,000 on that grid, and random
(k, n, theta) with theta formed as chop_ends_by_changepoint forms it.  Dev
container only (needs /root/reference)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="needs the reference sources")
def test_pbinom_bit_exact_against_reference():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "pbinom_check"])
    p = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "pbinom_check"),
                        os.path.join(ROOT, "gmap-gsnap_amd", "lib", "libgsnapdp.so"), "300", "5000", "200000"],
                       capture_output=True, text=True, timeout=300)
    print(p.stdout, p.stderr[-2000:])
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    import re
    ncmp, nbad, nflip, nnear = (int(x) for x in re.findall(r"(\d+) (?:compared|differ|decisions|within)", p.stdout))
    assert ncmp > 4_000_000 and nbad == 0 and nflip == 0
    assert nnear > 1000  # the decision-critical arguments were reached
