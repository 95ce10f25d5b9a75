"""Seeded synthetic workloads for the configs of BASELINE.json.

The reference ships no usable data for configs 2-5 (trucks data missing, POS
corpora need the network), so these are synthetic by design:
  config 2  N=45,  V=50,000 Zipf(1.1)-shaped emissions, T~U[1,128], B=4,096, seed 2
  config 3  N=64,  V=256, T~U[32,1024], B=16,384, seed 3
  config 4  N=256, V=1,024 (bdims [32,32]), T=512, B=65,536, seed 20261015
  config 5  config 4 + one constrained position in half the sequences, K=7 components
Rows of A, B and pi are Dirichlet(alpha) samples turned into log10 probabilities
with exact zeros mapped to -inf (reference hmm/hmm.rs:192-205 `log`).
"""
from __future__ import annotations

import numpy as np


def log10_probs(p: np.ndarray) -> np.ndarray:
    """hmm.rs:192-205: x == 0 -> -inf else log10(x)."""
    out = np.full(p.shape, -np.inf)
    nz = p != 0
    out[nz] = np.log10(p[nz])
    return out


def dirichlet_rows(rng, rows, cols, alpha=1.0):
    g = rng.gamma(alpha, 1.0, size=(rows, cols))
    s = g.sum(axis=1, keepdims=True)
    s[s == 0] = 1.0
    return g / s


def random_hmm(n, v, seed=0, alpha=1.0, zipf=None, zero_frac=0.0):
    """Returns (pi[N], a[N,N], b[N,V]) as log10 f64 arrays."""
    rng = np.random.default_rng(seed)
    a = dirichlet_rows(rng, n, n, alpha)
    if zipf is not None:
        ranks = np.arange(1, v + 1, dtype=np.float64)
        base = ranks ** (-zipf)
        b = np.empty((n, v))
        for s in range(n):
            w = base[rng.permutation(v)] * rng.gamma(1.0, 1.0, size=v)
            b[s] = w / w.sum()
    else:
        b = dirichlet_rows(rng, n, v, alpha)
    pi = dirichlet_rows(rng, 1, n, alpha)[0]
    if zero_frac > 0:
        for m in (a, b):
            mask = rng.random(m.shape) < zero_frac
            m[mask] = 0.0
        pi[rng.random(n) < zero_frac] = 0.0
    return log10_probs(pi), log10_probs(a), log10_probs(b)


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    """splitmix64 stream (uint64), vectorised; elements [start, start+count)."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def iid_obs(v, total, seed, start=0):
    """obs iid uniform in [0, v) from splitmix64; any slice
    [start, start+total) of the stream can be generated independently (per-rank shards)."""
    return (splitmix64(seed, total, start) % np.uint64(v)).astype(np.int32)


def uniform_lengths(rng, lo, hi, nseq):
    return rng.integers(lo, hi + 1, size=nseq).astype(np.int64)


def offsets_from_lengths(lengths):
    off = np.zeros(len(lengths) + 1, np.int64)
    np.cumsum(lengths, out=off[1:])
    return off


def config(name: str, nseq: int | None = None):
    """Returns dict(pi, a, b, offsets, obs, bdims) for config "c2" | "c3" | "c4" (optionally fewer seqs)."""
    if name == "c4":
        n, v, T, B, seed = 256, 1024, 512, 65536, 20261015
        B = nseq or B
        pi, a, b = random_hmm(n, v, seed=seed)
        off = np.arange(B + 1, dtype=np.int64) * T
        obs = iid_obs(v, B * T, seed)
        return dict(pi=pi, a=a, b=b, offsets=off, obs=obs, bdims=(32, 32))
    if name == "c2":
        n, v, B, seed = 45, 50000, 4096, 2
        B = nseq or B
        pi, a, b = random_hmm(n, v, seed=seed, zipf=1.1)
        rng = np.random.default_rng(seed + 1)
        off = offsets_from_lengths(uniform_lengths(rng, 1, 128, B))
        obs = iid_obs(v, int(off[-1]), seed)
        return dict(pi=pi, a=a, b=b, offsets=off, obs=obs, bdims=(v, 1))
    if name == "c3":
        n, v, B, seed = 64, 256, 16384, 3
        B = nseq or B
        pi, a, b = random_hmm(n, v, seed=seed)
        rng = np.random.default_rng(seed + 1)
        off = offsets_from_lengths(uniform_lengths(rng, 32, 1024, B))
        obs = iid_obs(v, int(off[-1]), seed)
        return dict(pi=pi, a=a, b=b, offsets=off, obs=obs, bdims=(v, 1))
    if name == "c5":
        c = config("c4", nseq)
        c["component"] = constraint_components(c["offsets"], seed=20261016)
        return c
    raise ValueError(name)


def constraint_components(offsets, seed, ncomp=7, prob=0.5):
    """Config 5: each sequence gets, with probability `prob`, ONE constrained
    position at a uniform t, with a component uniform in [0, ncomp) -- the reference's POS
    pipeline puts one tagged position per sentence.  Returns component[sum T] (-1 = free)."""
    offsets = np.asarray(offsets, np.int64)
    rng = np.random.default_rng(seed)
    comp = np.full(int(offsets[-1]), -1, np.int32)
    for k in range(len(offsets) - 1):
        T = int(offsets[k + 1] - offsets[k])
        if T > 0 and rng.random() < prob:
            comp[offsets[k] + rng.integers(0, T)] = rng.integers(0, ncomp)
    return comp
