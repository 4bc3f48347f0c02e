"""ctypes wrapper for the C oracle (oracle/legacy_oracle.c).  Test infrastructure only."""
import ctypes
import os
import subprocess

import numpy as np

from .legacy_oracle import OracleInstance

_HERE = os.path.dirname(os.path.abspath(__file__))
# CSA_ORACLE_LIB: another build of the same source (tools/asan_host.sh: the sanitizer build)
_LIB_PATH = os.environ.get("CSA_ORACLE_LIB") or os.path.join(_HERE, "_build", "liblegacy_oracle.so")
_lib = None

P = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_draw.restype = ctypes.c_int
        L.oracle_draw.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int,
                                  ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                  P, P, P, P, ctypes.c_int]
        L.oracle_counts.restype = None
        L.oracle_counts.argtypes = [P, ctypes.c_uint64, ctypes.c_int, P]
        L.oracle_pairs.restype = None
        L.oracle_pairs.argtypes = [P, ctypes.c_uint64, ctypes.c_int, P, ctypes.c_int]
        L.oracle_unique.restype = ctypes.c_uint64
        L.oracle_unique.argtypes = [P, ctypes.c_uint64, ctypes.c_int]
        L.oracle_philox.restype = None
        L.oracle_philox.argtypes = [P, P, P]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def philox(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().oracle_philox(_ptr(c), _ptr(k), _ptr(out))
    return tuple(int(x) for x in out)


def arrays(inst: OracleInstance):
    pf = np.ascontiguousarray(np.asarray(inst.person_feat, np.int32).reshape(inst.n, inst.C))
    return (pf, np.asarray(inst.fmin, np.int32), np.asarray(inst.fmax, np.int32),
            np.asarray(inst.fcat, np.int32))


def draw(inst, k, seed, panel_begin, n_panels, max_attempts=1 << 20, want_picks=False, threads=None,
         rejects=None):
    """Returns (status, panels uint64[S,W], attempts uint32[S], picks int32[S,k] or None).
    ``rejects`` (uint32[S], optional) receives each panel's min-quota rejections; the other
    attempts - 1 restarts are SelectionErrors."""
    pf, fmin, fmax, fcat = arrays(inst)
    W = (inst.n + 63) // 64
    panels = np.zeros((n_panels, W), np.uint64)
    attempts = np.zeros(n_panels, np.uint32)
    picks = np.full((n_panels, k), -1, np.int32) if want_picks else None
    threads = threads or os.cpu_count() or 1
    rc = lib().oracle_draw(inst.n, inst.C, inst.F, _ptr(pf), _ptr(fmin), _ptr(fmax), _ptr(fcat), k,
                           seed, panel_begin, n_panels, max_attempts, _ptr(panels), _ptr(picks),
                           _ptr(attempts), _ptr(rejects), threads)
    return rc, panels, attempts, picks


def counts(panels, n):
    out = np.zeros(n, np.int64)
    p = np.ascontiguousarray(panels, np.uint64)
    lib().oracle_counts(_ptr(p), p.shape[0], n, _ptr(out))
    return out


def pairs(panels, n, threads=None):
    out = np.zeros((n, n), np.int64)
    p = np.ascontiguousarray(panels, np.uint64)
    lib().oracle_pairs(_ptr(p), p.shape[0], n, _ptr(out), threads or os.cpu_count() or 1)
    return out


def unique(panels, n):
    p = np.ascontiguousarray(panels, np.uint64)
    return int(lib().oracle_unique(_ptr(p), p.shape[0], n))
