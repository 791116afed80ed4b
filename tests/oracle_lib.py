"""Loader for the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    so = os.path.join(ORACLE_DIR, "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    L = C.CDLL(so)
    L.oracle_ba_solve.argtypes = [C.c_void_p, C.c_void_p]
    _lib = L
    return L


def ba_solve(vio, prob):
    """Run the oracle on a vio.BaProblem; returns the same result dict as the HIP path."""
    L = load()
    O = vio.BaOutput(prob.K, prob.L, prob.N)
    rc = L.oracle_ba_solve(C.byref(prob.c), C.byref(O.c))
    if rc != 0:
        raise RuntimeError(f"oracle_ba_solve rc={rc}")
    return O.result()
