"""Probe (CPU, numpy): path margins at config 4, and whether a normalised f32 forward pass can
CERTIFY its path as the f64 decode's own (VERDICT r3 "next" items 1 and 4).

For the first B config-4 sequences (N=256, T=512):
  * the f64 row-A0 decode (viterbi.rs:13-18 association, pi init cp.rs:66-68): path P64, and per
    sequence the on-path gap min_t (x_P - x_2) of the candidates x_i = d[i] + a[i, P_t] (and the
    final-row gap) -- the path margin; its magnitude |score|;
  * an f32 forward with the row max of the previous step subtracted every step (values stay in
    [-~20, 0]), its path P32 (first-index backtrack on its own rows), its on-path gaps and a
    RIGOROUS uniform error bound e_t (below); P32 is certified when every gap beats the bound.
    Certified paths must equal P64 (asserted).

Error bound (all finite model entries <= 0, so every value below is <= 0 and the candidates near
the top of a column have |a|, |d| <= |m|): exact shifted values E_t = delta_t - sum(c) (real
arithmetic on the f64 inputs); e_t >= max_j |d32_t[j] - E_t[j]| over finite j:
  e_0 = u max_j(|pi|+|b|+|d0|) * 1.01
  e_t = e_{t-1} (1 + 4u) + 1.01 u max_j (3|m_j| + 2|b_j| + |r_j| + |d_t[j]|)
with u = 2^-24, m_j = max_i fl(d[i] + a32[i,j]), r_j = fl(m_j + b32_j), d_t[j] = fl(r_j - c_t).
Exact gap at step t >= gap32_t - 2 e_{t-1} - 4.04 u (|s_P| + |s_2|); final >= gap32 - 2 e_{T-1}.
Certificate: every lower bound > 2 * gamma64 * |score| (f64 decode's own error, gamma64 =
(2T+2) 2^-53 * 1.01), so P32 is the strict optimum of the exact AND the f64 problem.

Usage: python tools/probe_margin.py [B] [chunk]
"""
import sys
import time

import numpy as np

sys.path.insert(0, "consistent-viterbi_amd")
from cviterbi import synth  # noqa: E402

U32 = 2.0 ** -24
U64 = 2.0 ** -53


def decode64(pi, a, b, obs):
    """obs [S, T]; returns path [S, T], gaps [S] (min over steps incl. final), score [S]."""
    S, T = obs.shape
    N = a.shape[0]
    d = pi[None, :] + b[:, obs[:, 0]].T  # [S, N]
    rows = np.empty((T, S, N))
    rows[0] = d
    for t in range(1, T):
        cand = d[:, :, None] + a[None, :, :]  # [S, i, j]
        m = cand.max(axis=1)
        d = m + b[:, obs[:, t]].T
        rows[t] = d
    path = np.empty((S, T), np.int64)
    last = rows[T - 1]
    cur = last.argmax(axis=1)
    srt = np.sort(last, axis=1)
    gap = srt[:, -1] - srt[:, -2]
    score = last[np.arange(S), cur]
    path[:, T - 1] = cur
    for t in range(T - 1, 0, -1):
        x = rows[t - 1] + a[:, cur].T  # [S, i]
        p = x.argmax(axis=1)
        xs = np.sort(x, axis=1)
        gap = np.minimum(gap, xs[:, -1] - xs[:, -2])
        path[:, t - 1] = p
        cur = p
    return path, gap, score


def decode32n(pi, a, b, obs):
    """Normalised f32 forward + backtrack; returns path, cert lower bound on the exact margin
    (min over steps), per-step error bound at the end, and the raw gap."""
    S, T = obs.shape
    N = a.shape[0]
    f = np.float32
    a32, b32, pi32 = a.astype(f), b.astype(f), pi.astype(f)
    d = pi32[None, :] + b32[:, obs[:, 0]].T
    fin = np.isfinite(d)
    e = np.zeros((T, S))
    e[0] = U32 * 1.01 * np.where(fin, np.abs(pi)[None, :] + np.abs(b[:, obs[:, 0]].T) + np.abs(d), 0).max(axis=1)
    rows = np.empty((T, S, N), f)
    rows[0] = d
    for t in range(1, T):
        c = d.max(axis=1)  # row max of the previous step (exact in f32)
        cand = d[:, :, None] + a32[None, :, :]
        m = cand.max(axis=1)
        bt = b32[:, obs[:, t]].T
        r = m + bt
        dn = r - c[:, None]
        fin = np.isfinite(dn)
        loc = np.where(fin, 3 * np.abs(m).astype(np.float64) + 2 * np.abs(bt) + np.abs(r) + np.abs(dn), 0).max(axis=1)
        e[t] = e[t - 1] * (1 + 4 * U32) + 1.01 * U32 * loc
        d = dn
        rows[t] = d
    path = np.empty((S, T), np.int64)
    last = rows[T - 1].astype(np.float64)
    cur = last.argmax(axis=1)
    srt = np.sort(last, axis=1)
    lb = (srt[:, -1] - srt[:, -2]) - 2 * e[T - 1]
    raw = srt[:, -1] - srt[:, -2]
    path[:, T - 1] = cur
    for t in range(T - 1, 0, -1):
        x = (rows[t - 1] + a32[:, cur].T).astype(np.float64)  # the forward's own f32 sums
        p = x.argmax(axis=1)
        xs = np.sort(x, axis=1)
        g = xs[:, -1] - xs[:, -2]
        raw = np.minimum(raw, g)
        lb = np.minimum(lb, g - 2 * e[t - 1] - 4.04 * U32 * (np.abs(xs[:, -1]) + np.abs(xs[:, -2])))
        path[:, t - 1] = p
        cur = p
    return path, lb, e[T - 1], raw


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    c = synth.config("c4", B)
    pi, a, b = c["pi"], c["a"], c["b"]
    T = 512
    obs = c["obs"].reshape(B, T)
    gaps, scores, lbs, eT, raw32, same, cert_ok = [], [], [], [], [], [], []
    t0 = time.time()
    for s0 in range(0, B, chunk):
        o = obs[s0:s0 + chunk]
        p64, g64, sc = decode64(pi, a, b, o)
        p32, lb, e_end, raw = decode32n(pi, a, b, o)
        gam = (2 * T + 2) * U64 * 1.01
        cert = lb > 2 * gam * np.abs(sc)
        eq = (p32 == p64).all(axis=1)
        assert np.all(eq[cert]), "a certified f32 path differs from the f64 path"
        gaps.append(g64); scores.append(sc); lbs.append(lb); eT.append(e_end); raw32.append(raw)
        same.append(eq); cert_ok.append(cert)
        print(f"{s0 + len(o)}/{B} seqs, {time.time() - t0:.0f} s: certified {np.concatenate(cert_ok).mean():.4f}"
              f", f32 path == f64 {np.concatenate(same).mean():.4f}", flush=True)
    g = np.concatenate(gaps); sc = np.concatenate(scores); lb = np.concatenate(lbs)
    e = np.concatenate(eT); eq = np.concatenate(same); cert = np.concatenate(cert_ok)
    print(f"\nB={B} N=256 T=512 (config 4, first {B} sequences)")
    print(f"f64 path margin (min on-path gap incl. final): quantiles 1/5/10/50% ="
          f" {np.quantile(g, [0.01, 0.05, 0.10, 0.5])}")
    for x in (1e-9, 1e-7, 1e-5, 1e-4, 1e-3, 1e-2):
        print(f"  P(margin < {x:g}) = {np.mean(g < x):.4f}")
    print(f"|score| median {np.median(np.abs(sc)):.1f}")
    print(f"normalised f32: error bound e_T median {np.median(e):.3e}, max {e.max():.3e}")
    print(f"normalised f32: path == f64 path {eq.mean():.4f}; CERTIFIED {cert.mean():.4f}"
          f" ({cert.sum()} of {B})")
    # CP super-sequence chain: sequence k carries |M_{k-1}| ~ k * median|score|; the certificate
    # needs margin > ~ c T u (2|M| + |score|); report the fraction failing at the chain positions of
    # a config-4-sized chain (65,536 sequences) with c = 8
    med = np.median(np.abs(sc))
    for k in (1, 1024, 16384, 65535):
        need = 8 * (T + 2) * U64 * (2 * k * med + np.abs(sc))
        print(f"  chain position {k}: margin below the f64 chain bound for {np.mean(g <= need):.5f}")


if __name__ == "__main__":
    main()
