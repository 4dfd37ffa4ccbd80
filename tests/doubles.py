"""The host-program test doubles the drop-in resolves from the process
(tests/dropin/pairpool_double.c: Pairpool_push*, List_*, Stage2_compute_one).
One copy per process: the drop-in binds those symbols from the global scope,
i.e. from the first copy loaded with RTLD_GLOBAL, so a second copy's state
(the stage-2 recording of dbl_stage2_load) would never be seen."""
import ctypes
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOUBLE_SRC = os.path.join(ROOT, "tests", "dropin", "pairpool_double.c")
_PAIRPOOL = None


def pairpool_double():
    global _PAIRPOOL
    if _PAIRPOOL is None:
        d = tempfile.mkdtemp(prefix="gsnapdp_dbl_")
        so = os.path.join(d, "libpairpool_double.so")
        subprocess.check_call(["gcc", "-O1", "-shared", "-fPIC", "-o", so, DOUBLE_SRC])
        _PAIRPOOL = ctypes.CDLL(so, mode=ctypes.RTLD_GLOBAL)
    return _PAIRPOOL
