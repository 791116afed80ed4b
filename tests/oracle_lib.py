"""Loader for the CPU oracle (oracle/liboracle.so) — test infrastructure only."""
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
    _lib = C.CDLL(so)
    return _lib
