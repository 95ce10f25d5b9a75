"""CPU: the certified suffix trace's argument (kernels/trellis64.hip suffix_trace_f64, DESIGN.md
§3) checked against the oracle, no GPU involved.  A numpy restatement of the reversed suffix
pass (the kernel's association: r_x(j) = max_k (r_{x+1}(k) + a[j][k]) + b[j][o_x]) and of the
forward read-off with the margin test w2 (1 - rho) + 2 rho |d| < w_P (1 + rho),
rho = (4L + 8) 2^-52: whenever every step certifies, the path after t1 and the forward fold
(d + a) + b from delta_{t1}(s*) must equal the oracle's forced decode (viterbi.rs:13-18 with
the constrained element forced) bit for bit.  Random log10 models certify nearly always;
dyadic models (exact ties) must fail somewhere -- and never certify a wrong path."""
import numpy as np
import pytest

import c_oracle as O
from cviterbi import synth

NINF = -np.inf


def _forward_row(pi, a, b, obs, t1):
    """delta_{t1} of the unforced row-A0 recurrence (cp.rs:66-68, viterbi.rs:15-17)."""
    d = pi + b[:, obs[0]]
    for t in range(1, t1 + 1):
        d = np.max(d[:, None] + a, axis=0) + b[:, obs[t]]
    return d


def _suffix_rows(a, b, seg):
    """Rows of the reversed suffix pass for the elements x = 1 .. len(seg) - 1 of seg = obs[t1:]."""
    r = {len(seg) - 1: 0.0 + b[:, seg[-1]]}  # pi0 + e
    for x in range(len(seg) - 2, 0, -1):
        r[x] = np.max(r[x + 1][None, :] + a, axis=1) + b[:, seg[x]]
    return r


def _trace(a, b, seg, d, s0):
    L = len(seg) - 1
    rho = (4 * L + 8) * 2.0 ** -52
    r = _suffix_rows(a, b, seg)
    cur, path = s0, []
    for x in range(1, L + 1):
        w = r[x] + a[cur, :]
        idx = int(np.argmax(w))  # first index of the maximum
        M = w[idx]
        w2 = np.max(np.delete(w, idx)) if len(w) > 1 else NINF
        if not (M > NINF and w2 * (1 - rho) + 2 * rho * abs(d) < M * (1 + rho)):
            return None
        d = (d + a[cur, idx]) + b[idx, seg[x]]
        cur = idx
        path.append(idx)
    return np.array(path, np.int32), d


def _run(pi, a, b, nseq, tmax, seed):
    rng = np.random.default_rng(seed)
    n, v = b.shape
    lens = rng.integers(1, tmax, size=nseq)
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    t1s = np.array([rng.integers(0, T) for T in lens])
    states = rng.integers(0, n, size=nseq)
    forced = np.full(len(obs), -1, np.int32)
    forced[off[:-1] + t1s] = states
    rp, rs, rst = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, forced=forced)
    certified = mismatched = 0
    for k in range(nseq):
        o = obs[off[k]:off[k + 1]]
        t1, s0 = int(t1s[k]), int(states[k])
        D = _forward_row(pi, a, b, o, t1)[s0]
        if not D > NINF:
            continue
        got = _trace(a, b, o[t1:], D, s0)
        if got is None:
            continue
        certified += 1
        path, score = got
        ok = rst[k] == 0 and np.array_equal(path, rp[off[k] + t1 + 1:off[k + 1]]) and rp[off[k] + t1] == s0 \
            and np.float64(score).view(np.int64) == np.float64(rs[k]).view(np.int64)
        mismatched += not ok
    return certified, mismatched


@pytest.mark.parametrize("n,seed", [(8, 1), (16, 2), (33, 3)])
def test_trace_certified_paths_equal_forced_decode(n, seed):
    pi, a, b = synth.random_hmm(n, 12, seed=seed)
    certified, mismatched = _run(pi, a, b, nseq=120, tmax=40, seed=seed)
    assert mismatched == 0
    assert certified >= 100  # continuous models: near ties at the 1e-10 level are rare


@pytest.mark.parametrize("quant", [2, 4])
def test_trace_dyadic_ties_never_certify_wrong(quant):
    pi, a, b = synth.random_hmm(6, 5, seed=40 + quant)
    pi, a, b = (np.where(np.isfinite(x), np.round(x * quant) / quant, x) for x in (pi, a, b))
    certified, mismatched = _run(pi, a, b, nseq=150, tmax=30, seed=quant)
    assert mismatched == 0
    assert certified < 150  # exact ties on the paths make some traces fall back
