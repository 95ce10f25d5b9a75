"""ctypes loader for the C oracle (oracle/build/libcv_oracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  See cv_oracle.h for
the semantics and the parity status ("parity unpinned": pinned by KATs and
exhaustive enumeration, not by reference fixtures, which do not exist).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

VITERBI, CP, DP, DECODE = 0, 1, 2, 3
_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "libcv_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        for name in ("cvo_decode_batch_f64", "cvo_decode_batch_f32"):
            f = getattr(L, name)
            f.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int64, P, P, ctypes.c_int, P, P, P,
                          ctypes.c_int]
            f.restype = ctypes.c_int
        for name in ("cvo_decode_batch_forced_f64", "cvo_decode_batch_forced_f32"):
            f = getattr(L, name)
            f.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int64, P, P, P, ctypes.c_int, P, P, P,
                          ctypes.c_int]
            f.restype = ctypes.c_int
        for name in ("cvo_forward_row_f64", "cvo_forward_row_f32"):
            f = getattr(L, name)
            f.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int, P, P]
            f.restype = None
        L.cvo_rescore_f64.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int, P, P]
        L.cvo_rescore_batch_f64.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int64, P, P, P, P]
        L.cvo_rescore_batch_f64.restype = None
        L.cvo_rescore_f64.restype = ctypes.c_double
        L.cvo_cp_superseq_f64.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int64, P, P, P]
        L.cvo_cp_superseq_f64.restype = ctypes.c_double
        _lib = L
    return _lib


def _p(x):
    return x.ctypes.data_as(ctypes.c_void_p)


def decode_batch(pi, a, b, offsets, obs, assoc=VITERBI, dtype=np.float64, nthreads=1, forced=None):
    """Returns (path int32[sum T], score f64[B], status u8[B]); forced[sum T] optional (-1 free)."""
    dt = np.dtype(dtype)
    pi = np.ascontiguousarray(pi, dt)
    a = np.ascontiguousarray(a, dt)
    b = np.ascontiguousarray(b, dt)
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    n, v = a.shape[0], b.shape[1]
    nseq = offsets.shape[0] - 1
    path = np.zeros(int(offsets[-1]), np.int32)
    score = np.zeros(nseq, np.float64)
    status = np.zeros(nseq, np.uint8)
    if forced is None:
        fn = lib().cvo_decode_batch_f64 if dt == np.float64 else lib().cvo_decode_batch_f32
        fn(n, v, _p(pi), _p(a), _p(b), nseq, _p(offsets), _p(obs), assoc, _p(path), _p(score), _p(status),
           int(nthreads))
    else:
        forced = np.ascontiguousarray(forced, np.int32)
        fn = lib().cvo_decode_batch_forced_f64 if dt == np.float64 else lib().cvo_decode_batch_forced_f32
        fn(n, v, _p(pi), _p(a), _p(b), nseq, _p(offsets), _p(obs), _p(forced), assoc, _p(path), _p(score),
           _p(status), int(nthreads))
    return path, score, status


def forward_row(pi, m, b, obs, dtype):
    dt = np.dtype(dtype)
    pi = np.ascontiguousarray(pi, dt)
    m = np.ascontiguousarray(m, dt)
    b = np.ascontiguousarray(b, dt)
    obs = np.ascontiguousarray(obs, np.int32)
    out = np.zeros(m.shape[0], dt)
    fn = lib().cvo_forward_row_f64 if dt == np.float64 else lib().cvo_forward_row_f32
    fn(m.shape[0], b.shape[1], _p(pi), _p(m), _p(b), obs.shape[0], _p(obs), _p(out))
    return out


def max_marginal(pi, a, b, obs, tk, dtype):
    """Spec of np_oracle.max_marginal, C-accelerated."""
    dt = np.dtype(dtype).type
    a_ = np.asarray(a, dt)
    d = forward_row(pi, a, b, obs[:tk + 1], dt)
    if tk == len(obs) - 1:
        beta = np.zeros(a_.shape[0], dt)
    else:
        g = forward_row(np.zeros(a_.shape[0]), np.ascontiguousarray(np.asarray(a).T), b, obs[tk + 1:][::-1], dt)
        beta = (g[None, :] + a_).max(axis=1).astype(dt)
    return (d + beta).astype(dt)


def constrained_forced(pi, a, b, offsets, obs, component, dtype=np.float32):
    """np_oracle.constrained_decode spec with the C-accelerated max-marginal (one-position
    sequences); several-position sequences use the numpy segment tables.
    Returns (comp_state dict, forced[sum T])."""
    import np_oracle as NO

    return NO.constrained_decode(pi, a, b, offsets, obs, component, dtype,
                                 mm=lambda pi_, a_, b_, o, t, dt: max_marginal(pi_, a_, b_, np.asarray(o), t, dt))


def rescore_f64(pi, a, b, obs, path):
    pi = np.ascontiguousarray(pi, np.float64)
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    obs = np.ascontiguousarray(obs, np.int32)
    path = np.ascontiguousarray(path, np.int32)
    return lib().cvo_rescore_f64(a.shape[0], b.shape[1], _p(pi), _p(a), _p(b), obs.shape[0], _p(obs), _p(path))


def rescore_batch_f64(pi, a, b, offsets, obs, path):
    """rescore_f64 of every sequence of a CSR batch (f64 row-A0 fold along each path)."""
    pi = np.ascontiguousarray(pi, np.float64)
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    path = np.ascontiguousarray(path, np.int32)
    out = np.zeros(offsets.shape[0] - 1, np.float64)
    lib().cvo_rescore_batch_f64(a.shape[0], b.shape[1], _p(pi), _p(a), _p(b), offsets.shape[0] - 1, _p(offsets),
                                _p(obs), _p(path), _p(out))
    return out


def cp_superseq_f64(pi, a, b, offsets, obs):
    pi = np.ascontiguousarray(pi, np.float64)
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    path = np.zeros(int(offsets[-1] - offsets[0]), np.int32)
    obj = lib().cvo_cp_superseq_f64(a.shape[0], b.shape[1], _p(pi), _p(a), _p(b), offsets.shape[0] - 1,
                                    _p(offsets), _p(obs), _p(path))
    return path, obj
