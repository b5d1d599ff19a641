"""ctypes wrapper for the C oracle (oracle/_build/liboracle.so). TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.fuo_ca_sync.argtypes = [ctypes.c_int32, _i64p, _i32p, _i32p, _f64p, ctypes.c_int32,
                                  _f64p, _f64p, ctypes.c_int]
        L.fuo_ca_rounds.argtypes = [ctypes.c_int32, _i64p, _i32p, _i32p, _f64p, ctypes.c_int32,
                                    _f64p, _f64p, ctypes.c_int]
        L.fuo_replay.argtypes = [ctypes.c_int32, _i64p, _f64p, ctypes.c_int32, _i64p, _i32p,
                                 _i32p, _i32p, ctypes.c_int64, ctypes.c_int32, _i32p, _f64p,
                                 _f64p, _f64p, _f64p]
        L.fuo_max_threads.restype = ctypes.c_int
        L.fuo_rev64.argtypes = [ctypes.c_int32, _i64p, _i32p, _i64p, ctypes.c_int]
        L.fuo_rev64.restype = ctypes.c_int64
        L.fuo_ca_sync64.argtypes = [ctypes.c_int32, _i64p, _i32p, _i64p, _f64p, ctypes.c_int32,
                                    _f64p, _f64p, ctypes.c_int]
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def ca_sync(rowptr, col, rev, values, rounds, nthreads=1):
    """Collect-all gen-sync rounds [0, rounds) from zero state -> (a, f)."""
    rowptr = _c(rowptr, np.int64)
    n = len(rowptr) - 1
    a = np.empty(n)
    f = np.empty(int(rowptr[-1]))
    rc = lib().fuo_ca_sync(n, rowptr, _c(col, np.int32), _c(rev, np.int32),
                           _c(values, np.float64), int(rounds), a, f, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"fuo_ca_sync failed ({rc})")
    return a, f


def rev64(rowptr, col, nthreads=1):
    """The reverse-edge index as int64 (graphs of 2^31 or more directed edges)."""
    rowptr = _c(rowptr, np.int64)
    rev = np.empty(int(rowptr[-1]), dtype=np.int64)
    bad = lib().fuo_rev64(len(rowptr) - 1, rowptr, _c(col, np.int32), rev, int(nthreads))
    if bad:
        raise ValueError(f"{bad} edges have no reverse edge")
    return rev


def ca_sync64(rowptr, col, rev, values, rounds, nthreads=1):
    """ca_sync with an int64 reverse index (rev64): the same arithmetic."""
    rowptr = _c(rowptr, np.int64)
    n = len(rowptr) - 1
    a = np.empty(n)
    f = np.empty(int(rowptr[-1]))
    rc = lib().fuo_ca_sync64(n, rowptr, _c(col, np.int32), _c(rev, np.int64),
                             _c(values, np.float64), int(rounds), a, f, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"fuo_ca_sync64 failed ({rc})")
    return a, f


def ca_rounds(rowptr, col, rev, values, rounds, a, f, nthreads=1):
    """Continue `rounds` steady-state rounds in place on (a, f)."""
    rowptr = _c(rowptr, np.int64)
    rc = lib().fuo_ca_rounds(len(rowptr) - 1, rowptr, _c(col, np.int32), _c(rev, np.int32),
                             _c(values, np.float64), int(rounds), a, f, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"fuo_ca_rounds failed ({rc})")


def replay(rowptr, values, tick_task_off, tasks, events, out_ids, n_msgs, snap_ticks=()):
    rowptr = _c(rowptr, np.int64)
    n = len(rowptr) - 1
    E = int(rowptr[-1])
    st = _c(sorted(snap_ticks), np.int32) if len(snap_ticks) else np.zeros(1, np.int32)
    ns = len(snap_ticks)
    snaps = np.zeros((max(ns, 1), n))
    last = np.empty(n)
    flow = np.empty(E if E else 1)
    est = np.empty(E if E else 1)
    tto = _c(tick_task_off, np.int64)
    rc = lib().fuo_replay(n, rowptr, _c(values, np.float64), len(tto) - 1, tto,
                          _c(tasks, np.int32).reshape(-1), _c(events, np.int32).reshape(-1),
                          _c(out_ids, np.int32) if len(out_ids) else np.zeros(1, np.int32),
                          int(n_msgs), ns, st, snaps, last, flow, est)
    if rc != 0:
        raise RuntimeError(f"fuo_replay failed ({rc})")
    return last, flow[:E], est[:E], {t: snaps[k] for k, t in enumerate(sorted(snap_ticks))}


def max_threads():
    return int(lib().fuo_max_threads())
