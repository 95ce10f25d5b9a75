"""HMM fitting on MI355X (cv_hmm_fit_mle / cv_hmm_fit_train).

Replaces HMM::maximum_likelihood_estimation (hmm/hmm.rs:30-62) and HMM::train, the
tag-clamped Baum-Welch of hmm.rs:69-190.  Both start from the CURRENT parameters in
probability space (the reference draws them at random in HMM::new, hmm.rs:22-28, so the
caller supplies them) and return the fitted parameters log-mapped the way the reference's
log() does (0 -> -inf, else ln(x)/ln(10)), i.e. ready for cviterbi.HMM.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def _p(x):
    return x.ctypes.data_as(ctypes.c_void_p)


def _prep(pi, a, b, offsets, obs, tags):
    pi = np.array(pi, np.float64, copy=True)
    a = np.array(a, np.float64, copy=True)
    b = np.array(b, np.float64, copy=True)
    n = pi.shape[0]
    b = b.reshape(n, -1)
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    tags = np.ascontiguousarray(tags, np.int32)
    return pi, a, b, offsets, obs, tags


def fit_mle(pi, a, b, offsets, obs, tags, device=0):
    """Supervised fit (every tag >= 0).  Returns log-mapped (pi, a, b[N, V])."""
    pi, a, b, offsets, obs, tags = _prep(pi, a, b, offsets, obs, tags)
    n, v = b.shape
    L.check(L.lib().cv_hmm_fit_mle(n, v, len(offsets) - 1, _p(offsets), _p(obs), _p(tags), int(device), _p(pi),
                                   _p(a), _p(b)))
    return pi, a, b


def fit_train(pi, a, b, offsets, obs, tags, max_iter=1000, tol=0.001, device=0):
    """Tag-clamped Baum-Welch (tags -1 = unknown); defaults = main.rs:95.  Returns
    log-mapped (pi, a, b[N, V]) and the number of iterations run."""
    pi, a, b, offsets, obs, tags = _prep(pi, a, b, offsets, obs, tags)
    n, v = b.shape
    it = ctypes.c_int32(0)
    L.check(L.lib().cv_hmm_fit_train(n, v, len(offsets) - 1, _p(offsets), _p(obs), _p(tags), int(max_iter),
                                     float(tol), int(device), _p(pi), _p(a), _p(b), ctypes.byref(it)))
    return pi, a, b, it.value
