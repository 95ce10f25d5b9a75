"""Baum-Welch diagnostics against the oracle (one EM iteration, max |log10 diff| of pi, a, b):
the GEMM path forced at small N (CV_BW_GEMM_PATH=1) without tiny arcs, and the tiny-arc
model (a 1e-306 and / or a subnormal forced arc) -- python tools/debug/bw_tiny_diag.py"""
import os
import sys

R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [os.path.join(R, "consistent-viterbi_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")]
import numpy as np  # noqa: E402

import cviterbi as cv  # noqa: E402
import fit_oracle as FO  # noqa: E402
from test_fit import _corpus, _probs  # noqa: E402


def diff(got, ref):
    out = []
    for g, r in zip(got, ref):
        fin = np.isfinite(r) & np.isfinite(g)
        same_inf = np.array_equal(np.isinf(g), np.isinf(r))
        out.append(f"{np.max(np.abs(g[fin] - r[fin])) if fin.any() else 0:.2e}{'' if same_inf else ' INF-MISMATCH'}")
    return " ".join(out)


def case(n, arcs, iters):
    v = 23
    rng = np.random.default_rng(7000 + n)
    pi0, a0, b0 = _probs(n, v, seed=7000 + n)
    p, q, p2, q2 = 1, 3, 5, 2
    tagged = []
    if "normal" in arcs or "tags" in arcs:
        if "normal" in arcs:
            a0[p, q] = 1e-306
        tagged += [np.tile([p, q], 30)] * 20
    if "sub" in arcs or "tags" in arcs:
        if "sub" in arcs:
            a0[p2, q2] = 5e-320
        tagged += [np.tile([p2, q2], 30)] * 20
    a0 /= a0.sum(axis=1, keepdims=True)
    free = [rng.integers(0, n, size=int(rng.integers(5, 40))) for _ in range(30)]
    seqs = tagged + free
    lengths = np.array([len(x) for x in seqs])
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum(lengths, out=off[1:])
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    tags = np.full(int(off[-1]), -1, np.int32)
    for k in range(len(tagged)):
        tags[off[k]:off[k + 1]] = tagged[k]
    got = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=iters, tol=0.0)[:3]
    ref = FO.train(pi0, a0, b0, off, obs, tags, iters, 0.0)[:3]
    return diff(got, ref)


for n in (20, 100, 300):
    for iters in (1, 2):
        print(f"N={n} iters={iters} tiny normal+sub: {case(n, ('normal', 'sub'), iters)}", flush=True)
        print(f"N={n} iters={iters} tiny normal:     {case(n, ('normal',), iters)}", flush=True)
        print(f"N={n} iters={iters} tiny sub:        {case(n, ('sub',), iters)}", flush=True)
        print(f"N={n} iters={iters} none:            {case(n, (), iters)}", flush=True)
        print(f"N={n} iters={iters} tags, no tiny:   {case(n, ('tags',), iters)}", flush=True)
        os.environ["CV_BW_GEMM_PATH"] = "1"
        print(f"N={n} iters={iters} none, GEMM path: {case(n, (), iters)}", flush=True)
        print(f"N={n} iters={iters} tags, GEMM path: {case(n, ('tags',), iters)}", flush=True)
        del os.environ["CV_BW_GEMM_PATH"]
