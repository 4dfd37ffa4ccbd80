"""End to end: the reference's gmap program with the drop-in in place of its DP.

SURVEY.md 8(f)1.  ``oracle/Makefile`` (``make -C oracle ref``, dev container only)
compiles the reference's gmap from its own sources twice:

* ``oracle/_ref/gmap_cpu``: with its own ``dynprog.o`` / ``maxent_hr.o`` (the
  reference, CPU);
* ``oracle/_ref/gmap_gpu``: with ``libgsnapdp_dropin.so`` in their place, so every
  ``Dynprog_*`` / ``Maxent_hr_*`` call gmap's stage 3 makes runs on the GPU.

Both use our clean-room ``genome_hr`` subset (the reference's ``genome_hr.c`` is a
missing blob).  Binaries built from reference sources never leave this container
(``.gpurunignore``), so the GPU side of the end-to-end check runs on data:

* here, ``gmap_cpu`` reproduces the reference's own ``tests/align.test.ok`` byte
  for byte (``gmap -A -g ss.chr17test ss.her2``, ``tests/align.test.in``), reading
  the reference's files in place, and aligns every synthetic spliced cDNA
  (``workload.synthetic_transcripts``);
* ``oracle/_ref/gmap_trace`` (gmap_cpu recording every gap window stage 3 issues
  on those cDNAs) made the golden sets ``gmap_synth_gap`` / ``gmap_synth_ggap``,
  which the GPU tests replay through the batched C-ABI and the drop-in
  (test_gpu_parity, test_gpu_ggap, test_dropin).
"""
import os
import re
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
GMAP_CPU = os.path.join(ROOT, "oracle", "_ref", "gmap_cpu")
GMAP_GPU = os.path.join(ROOT, "oracle", "_ref", "gmap_gpu")
REF_TESTS = "/root/reference/tests"


def need(path):
    if not os.path.exists(path):
        pytest.skip("%s not built (make -C oracle ref, dev container)" % path)


def synthetic_inputs(tmp_path, ngenes=40, genome_len=300_000, seed=7):
    from gsnapdp import workload as W

    g, q = W.synthetic_transcripts(seed=seed, ngenes=ngenes, genome_len=genome_len)
    gf, qf = str(tmp_path / "genome.fa"), str(tmp_path / "cdna.fa")
    W.write_fasta(gf, [("synthchr", g)])
    W.write_fasta(qf, q)
    return gf, qf, len(q)


def run_gmap(binary, genome_fa, query_fa, env=None):
    t = time.perf_counter()
    r = subprocess.run([binary, "-A", "-g", genome_fa, query_fa], capture_output=True, timeout=300,
                       env=env)
    return r, time.perf_counter() - t


def test_gmap_cpu_reproduces_align_test():
    need(GMAP_CPU)
    if not os.path.isdir(REF_TESTS):
        pytest.skip("reference tests not present (GPU box)")
    r, _ = run_gmap(GMAP_CPU, os.path.join(REF_TESTS, "ss.chr17test"), os.path.join(REF_TESTS, "ss.her2"))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    with open(os.path.join(REF_TESTS, "align.test.ok"), "rb") as f:
        assert r.stdout == f.read()


def test_gmap_cpu_aligns_synthetic_genes(tmp_path):
    need(GMAP_CPU)
    gf, qf, n = synthetic_inputs(tmp_path)
    r, _ = run_gmap(GMAP_CPU, gf, qf)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    out = r.stdout.decode()
    assert out.count("Paths (1)") == n
    exons = [int(x) for x in re.findall(r"Number of exons: (\d+)", out)]
    assert sum(exons) > 4 * n and max(exons) >= 10
    dirs = re.findall(r"cDNA direction: (\w+)", out)
    assert "sense" in dirs and "antisense" in dirs
