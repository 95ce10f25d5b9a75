"""numpy restatement of the reference's HMM fitting.

TEST INFRASTRUCTURE ONLY: the checker for cv_hmm_mle / cv_hmm_train (GPU), imported by
tests/ only.  Parity "unpinned" against the Rust binary (it cannot be built here; the
reference ships no tests or fixtures for fitting); pinned by closed-form cases in
tests/test_fit.py.

All arithmetic is f64 in probability space, like the reference; `log_map` is the
reference's final `log()` (hmm.rs:192-205): x == 0 -> -inf, else x.log(10.0), which Rust
computes as ln(x) / ln(10) -- NOT log10(x) (they differ in the last bit).

  mle    hmm.rs:30-62   counts ADDED to the current (initial) probabilities, rows divided
                        by (seen - end) / #sequences / seen; a row with seen == end -> 0.
  train  hmm.rs:69-190  tag-clamped Baum-Welch with per-row normalisation.  Note the
                        reference's forward step multiplies alpha_{t-1} by the emission of
                        o_t BEFORE the transition (hmm.rs:94: (alpha[t-1] * b(o_t)) . A),
                        and the backward step uses b(o_{t+1}) (hmm.rs:114-116); restated
                        as written.  normalize(v) = v / sum(v), or uniform 1/len when the
                        sum is 0 (hmm.rs:274-282, 306-317).
"""
from __future__ import annotations

import math

import numpy as np


def log_map(x):
    """hmm.rs:192-205: 0 -> -inf, else ln(x)/ln(10) elementwise (Rust f64::log(10.0))."""
    x = np.asarray(x, np.float64)
    out = np.full(x.shape, -np.inf)
    nz = x != 0.0
    out[nz] = np.log(x[nz]) / math.log(10.0)
    return out


def _normalize(v):
    s = v.sum()
    return v / s if s != 0.0 else np.full(v.shape, 1.0 / v.size)


def mle(pi0, a0, b0, offsets, obs, tags):
    """hmm.rs:30-62.  pi0[N], a0[N,N], b0[N,V]: the CURRENT probabilities (HMM::new draws
    them at random, hmm.rs:22-28); obs/tags flattened per CSR offsets, every tag >= 0.
    Returns log-mapped (pi, a, b)."""
    pi = np.array(pi0, np.float64, copy=True)
    a = np.array(a0, np.float64, copy=True)
    b = np.array(b0, np.float64, copy=True)
    n = a.shape[0]
    seen = np.zeros(n)
    end = np.zeros(n)
    nseq = len(offsets) - 1
    for s in range(nseq):
        lo, hi = int(offsets[s]), int(offsets[s + 1])
        tg = tags[lo:hi]
        ob = obs[lo:hi]
        pi[tg[0]] += 1.0
        for t in range(hi - lo - 1):
            b[tg[t], ob[t]] += 1.0
            a[tg[t], tg[t + 1]] += 1.0
            seen[tg[t]] += 1.0
        b[tg[-1], ob[-1]] += 1.0
        seen[tg[-1]] += 1.0
        end[tg[-1]] += 1.0
    for st in range(n):
        if seen[st] != end[st]:
            a[st] /= seen[st] - end[st]
        else:
            a[st] = 0.0
        pi[st] /= float(nseq)
        b[st] /= seen[st]
    return log_map(pi), log_map(a), log_map(b)


def _alpha(pi, a, b, ob, tg):
    n = a.shape[0]
    T = len(ob)
    al = np.zeros((T, n))
    if tg[0] >= 0:
        al[0, tg[0]] = 1.0
    else:
        al[0] = _normalize(pi * b[:, ob[0]])
    for t in range(1, T):
        if tg[t] >= 0:
            al[t, tg[t]] = 1.0
        else:
            al[t] = _normalize((al[t - 1] * b[:, ob[t]]) @ a)  # hmm.rs:93-94, as written
    return al


def _beta(a, b, ob, tg):
    n = a.shape[0]
    T = len(ob)
    be = np.zeros((T, n))
    if tg[T - 1] >= 0:
        be[T - 1, tg[T - 1]] = 1.0
    else:
        be[T - 1] = 1.0
    for t in range(T - 2, -1, -1):
        if tg[t] >= 0:
            be[t, tg[t]] = 1.0
        else:
            be[t] = _normalize((be[t + 1] * b[:, ob[t + 1]]) @ a.T)  # hmm.rs:114-116
    return be


def train_step(pi, a, b, offsets, obs, tags):
    """One EM iteration of hmm.rs:73-178 in probability space; tags -1 = untagged.
    Returns (new_pi, new_a, new_b, d) with d = sum |new - old| (hmm.rs:172-175)."""
    n = a.shape[0]
    V = b.shape[1]
    r = len(offsets) - 1
    new_pi = np.zeros(n)
    a_den = np.zeros(n)
    xi_sum = np.zeros((n, n))
    new_b = np.zeros((n, V))
    b_den = np.zeros(n)
    for s in range(r):
        lo, hi = int(offsets[s]), int(offsets[s + 1])
        ob = np.asarray(obs[lo:hi], np.int64)
        tg = np.asarray(tags[lo:hi], np.int64)
        al = _alpha(pi, a, b, ob, tg)
        be = _beta(a, b, ob, tg)
        g = np.array([_normalize(al[t] * be[t]) for t in range(len(ob))])  # hmm.rs:124-131
        for t in range(len(ob) - 1):  # hmm.rs:133-143
            m = (b[:, ob[t + 1]] * be[t + 1])[None, :] * al[t][:, None]
            xi_sum += _normalize((m * a).ravel()).reshape(n, n)
        new_pi += g[0]
        a_den += g[:-1].sum(axis=0)
        for t in range(len(ob)):
            new_b[:, ob[t]] += g[t]
        b_den += g.sum(axis=0)
    new_pi /= float(r)
    new_a = xi_sum / a_den[:, None]
    new_b = new_b / b_den[:, None]
    d = np.abs(new_pi - pi).sum() + np.abs(new_a - a).sum() + np.abs(new_b - b).sum()
    return new_pi, new_a, new_b, d


def train(pi0, a0, b0, offsets, obs, tags, max_iter, tol):
    """hmm.rs:69-190: iterate train_step until d <= tol (after the update) or max_iter;
    returns log-mapped (pi, a, b) and the number of iterations run."""
    pi, a, b = (np.array(x, np.float64, copy=True) for x in (pi0, a0, b0))
    it = 0
    for it in range(1, max_iter + 1):
        pi, a, b, d = train_step(pi, a, b, offsets, obs, tags)
        if d <= tol:
            break
    return log_map(pi), log_map(a), log_map(b), it
