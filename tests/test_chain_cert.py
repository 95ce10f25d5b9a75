"""CPU: the parallel CPSolver chain's certificate (DESIGN.md §3 "the parallel chain") checked
against the oracle's serial chain (cvo_cp_superseq_f64, the restatement of cp.rs:63-93 over
utils.rs:24-38) -- independently of the GPU.

For random, tie-heavy and scaled log10 models: every sequence is decoded on its own with the
row-A0 f64 recurrence (numpy, the forward's own association), the certificate rho / gF is
computed exactly as cp_cert_f64 computes it, and the host's test (rho > U at the chain's running
maximum M, the boundary test with the next sequence's score) is applied at the M the ORACLE's
chain reaches.  Whenever it certifies sequence k, the oracle's chain must take the row-A0 path
inside sequence k, and its running maximum after k must be the CP fold of that path from M --
both bit for bit; with M and the path's values in one binade, also M + q 2^(e-52) (the
quantised fold of cp_quant_f64).  Uncertified sequences are what the GPU re-runs through the
serial chain kernel."""
import zlib

import numpy as np
import pytest

import c_oracle as O
from cviterbi import synth


def _a0_rows(pi, a, b, obs):
    d = pi + b[:, obs[0]]
    rows = [d]
    for t in range(1, len(obs)):
        d = (d[:, None] + a).max(axis=0) + b[:, obs[t]]
        rows.append(d)
    return np.array(rows)


def _top2(x):
    m1 = x.max()
    arg = int(np.flatnonzero(x == m1)[0])
    rest = np.delete(x, arg)
    return arg, m1, (rest.max() if rest.size else -np.inf)


def _cert(pi, a, b, obs):
    """(path, rho, gF, score) of cp_cert_f64 on the row-A0 decode of one sequence."""
    rows = _a0_rows(pi, a, b, obs)
    T = len(obs)
    arg, m1, m2 = _top2(rows[-1])
    path = [arg]
    u0 = (abs(m1) + 16.0) * 2.0 ** -51
    gF = (m1 - m2) - 4.0 * T * u0
    rho = gF / (3 * T + 2)
    ok = m1 > -np.inf
    cur = arg
    for t in range(T - 1, 0, -1):
        x = rows[t - 1] + a[:, cur]
        p, x1, x2 = _top2(x)
        ok = ok and x1 > -np.inf
        rho = min(rho, ((x1 - x2) - (4 * t + 1) * u0) / (3 * t + 1))
        path.append(p)
        cur = p
    path = np.array(path[::-1])
    if not (ok and rho > 0):
        return path, -1.0, -1.0, m1
    return path, rho * (1 - 2.0 ** -50), gF * (1 - 2.0 ** -50), m1


def _fold(pi, a, b, obs, path, M):
    d = M + (pi[path[0]] + b[path[0], obs[0]])
    for t in range(1, len(obs)):
        d = d + (a[path[t - 1], path[t]] + b[path[t], obs[t]])
    return d


def _quant_fold(pi, a, b, obs, path, M):
    """M + q 2^(e-52) when M and every value share M's binade and no arc is a tie, else None."""
    e = int(np.floor(np.log2(abs(M)))) if M != 0 else None
    if e is None or abs(M) < 2.0 ** 12:
        return None
    g = 2.0 ** (e - 52)
    q = 0
    for t in range(len(obs)):
        w = pi[path[0]] + b[path[0], obs[0]] if t == 0 else a[path[t - 1], path[t]] + b[path[t], obs[t]]
        xs = w / g
        if xs - np.floor(xs) == 0.5:
            return None
        q += int(np.rint(xs))
    Mn = M + q * g
    return Mn if int(np.floor(np.log2(abs(Mn)))) == e else None


@pytest.mark.parametrize("kind,n,scale,jump", [("random", 16, 1.0, 0), ("random", 40, 1.0, 0), ("random", 16, 1e4, 0),
                                               ("random", 24, 1e8, 0), ("random", 16, 1e11, 0), ("dyadic", 12, 1.0, 0),
                                               ("dyadic", 12, 1e6, 0), ("random", 16, 1.0, 30), ("random", 32, 1.0, 38),
                                               ("random", 16, 1.0, 44)])
def test_chain_certificate_vs_oracle_chain(kind, n, scale, jump):
    """jump > 0: a first one-element sequence emits a symbol of log10-probability -2^jump, so
    every later sequence runs at |M| ~ 2^jump, where the chain's ulp (2^(jump-52)) reaches the
    path margins: some certificates fail, and the ones that hold are tested under heavy rounding."""
    rng = np.random.default_rng(zlib.crc32(repr((kind, n, scale, jump)).encode()))
    v = 9
    if kind == "dyadic":  # exact ties: certificates must fail there, never hold wrongly
        pi = np.round(rng.uniform(-2, 0, n) * 4) / 4
        a = np.round(rng.uniform(-2, 0, (n, n)) * 4) / 4
        b = np.round(rng.uniform(-2, 0, (n, v)) * 4) / 4
    else:
        pi, a, b = synth.random_hmm(n, v, seed=n)
    pi, a, b = pi * scale, a * scale, b * scale
    pimax = float(np.max(np.abs(pi[np.isfinite(pi)])))
    lengths = rng.integers(1, 30, size=36)
    obs = rng.integers(0, v, size=int(lengths.sum())).astype(np.int32)
    if jump:
        b = np.concatenate([b, np.full((n, 1), -2.0 ** jump)], axis=1)
        lengths = np.concatenate([[1], lengths])
        obs = np.concatenate([[v], obs]).astype(np.int32)
    off = synth.offsets_from_lengths(lengths)
    full_path, _ = O.cp_superseq_f64(pi, a, b, off, obs)
    nseq = len(lengths)
    info = [_cert(pi, a, b, obs[off[k]:off[k + 1]]) for k in range(nseq)]
    certified = quant = 0
    M = 0.0
    for k in range(nseq):
        lo, hi = off[k], off[k + 1]
        ob = obs[lo:hi]
        path, rho, gF, S = info[k]
        U = 2.0 ** -52 * (abs(M) + abs(S) + 16.0)
        ok = rho > U
        Mn = _fold(pi, a, b, ob, path, M) if ok else None
        if ok and k + 1 < nseq:
            U1 = 2.0 ** -52 * (abs(Mn) + abs(info[k + 1][3]) + pimax + 16.0)
            ok = gF - 3.0 * len(ob) * U > 2.0 * U1
        # the oracle chain's running maximum after sequence k (prefix chain 0..k)
        _, Mk = O.cp_superseq_f64(pi, a, b, off[:k + 2], obs[:hi])
        if ok:
            certified += 1
            assert np.array_equal(full_path[lo:hi], path), f"seq {k}: certified path differs from the chain's"
            assert Mn == Mk, f"seq {k}: fold {Mn!r} != chain {Mk!r}"
            qf = _quant_fold(pi, a, b, ob, path, M)
            if qf is not None:
                quant += 1
                assert qf == Mk, f"seq {k}: quantised fold {qf!r} != chain {Mk!r}"
        M = Mk
    if kind == "random" and scale <= 1e4 and not jump:
        assert certified >= nseq - 2
    if kind == "random" and (scale >= 1e4 or jump):
        assert quant > 0
    if jump >= 44:
        assert certified < nseq - 1, "no certificate failed at a 2^%d running total" % jump
