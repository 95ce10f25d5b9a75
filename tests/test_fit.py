"""HMM fitting: cv_hmm_fit_mle / cv_hmm_fit_train against the numpy
restatement of hmm.rs:30-62 / 69-190 (oracle/fit_oracle.py).

CPU: the oracle against closed forms -- MLE by hand on a tiny corpus, and a fully tagged
corpus, where one Baum-Welch iteration must reproduce the MLE counts (alpha, beta and
gamma are one-hot, each xi_t is a single 1 at (tag_t, tag_t+1)).
GPU: MLE to ~1 ulp (same host arithmetic; numpy's vectorised log may differ from glibc's by
an ulp); Baum-Welch within 1e-9 (log10) after several iterations (f64 sums in another
order -- the reference's own order is BLAS-internal, hmm.rs:94 `.dot`)."""
import numpy as np
import pytest

import fit_oracle as FO


def _corpus(n, v, nseq, tmax, tag_frac, seed):
    rng = np.random.default_rng(seed)
    lengths = rng.integers(1, tmax + 1, size=nseq)
    off = np.zeros(nseq + 1, np.int64)
    np.cumsum(lengths, out=off[1:])
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    tags = rng.integers(0, n, size=int(off[-1])).astype(np.int32)
    if tag_frac < 1.0:
        tags = np.where(rng.random(len(tags)) < tag_frac, tags, -1).astype(np.int32)
    return off, obs, tags


def _probs(n, v, seed):
    rng = np.random.default_rng(seed + 100)
    a = rng.random((n, n))
    a /= a.sum(axis=1, keepdims=True)
    b = rng.random((n, v))
    b /= b.sum(axis=1, keepdims=True)
    pi = rng.random(n)
    pi /= pi.sum()
    return pi, a, b


def test_mle_oracle_by_hand():
    # two sequences: states 0 1 1 / 1 0 ; obs 2 0 1 / 1 1 ; zero initial parameters
    off = np.array([0, 3, 5])
    obs = np.array([2, 0, 1, 1, 1])
    tags = np.array([0, 1, 1, 1, 0])
    pi, a, b = FO.mle(np.zeros(2), np.zeros((2, 2)), np.zeros((2, 3)), off, obs, tags)
    # transitions 0->1, 1->1, 1->0; seen = [2, 3], end = [1, 1] -> rows divided by [1, 2]
    np.testing.assert_array_equal(a, FO.log_map(np.array([[0.0, 1.0], [0.5, 0.5]])))
    np.testing.assert_array_equal(pi, FO.log_map(np.array([0.5, 0.5])))
    np.testing.assert_array_equal(b, FO.log_map(np.array([[0, 1, 1], [1, 2, 0]]) / np.array([[2.0], [3.0]])))
    assert a[0, 0] == -np.inf and b[1, 2] == -np.inf


def test_log_map_is_ln_over_ln10():
    x = np.array([0.0, 1.0, 0.001, 0.3, 1e-300])
    got = FO.log_map(x)
    assert got[0] == -np.inf and got[1] == 0.0
    for xi, gi in zip(x[2:], got[2:]):
        assert gi == np.log(xi) / np.log(10.0)  # Rust f64::log(10.0), not log10


def test_train_fully_tagged_equals_counts():
    n, v = 4, 6
    off, obs, tags = _corpus(n, v, 9, 12, 1.0, seed=5)
    pi0, a0, b0 = _probs(n, v, seed=5)
    pi1, a1, b1, _ = FO.train_step(pi0, a0, b0, off, obs, tags)
    lp, la, lb = FO.mle(np.zeros(n), np.zeros((n, n)), np.zeros((n, v)), off, obs, tags)
    seen_from = np.zeros(n)
    for s in range(len(off) - 1):
        for t in range(off[s], off[s + 1] - 1):
            seen_from[tags[t]] += 1
    ok = seen_from > 0  # rows of A with at least one outgoing transition
    np.testing.assert_allclose(FO.log_map(a1[ok]), la[ok], rtol=1e-12)
    np.testing.assert_allclose(FO.log_map(pi1), lp, rtol=1e-12)
    np.testing.assert_allclose(FO.log_map(b1), lb, rtol=1e-12)


def test_train_step_rows_are_distributions():
    n, v = 5, 7
    off, obs, tags = _corpus(n, v, 11, 15, 0.3, seed=9)
    pi, a, b = _probs(n, v, seed=9)
    for _ in range(3):
        pi, a, b, d = FO.train_step(pi, a, b, off, obs, tags)
        assert d >= 0
    np.testing.assert_allclose(a.sum(axis=1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(b.sum(axis=1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(pi.sum(), 1.0, rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("n,v", [(2, 3), (12, 30), (45, 200)])
def test_gpu_mle_matches_oracle(gpu, n, v):
    import cviterbi as cv

    off, obs, tags = _corpus(n, v, 40, 25, 1.0, seed=n)
    pi0, a0, b0 = _probs(n, v, seed=n)
    got = cv.fit_mle(pi0, a0, b0, off, obs, tags)
    ref = FO.mle(pi0, a0, b0, off, obs, tags)
    for g, r, what in zip(got, ref, ("pi", "a", "b")):
        assert np.array_equal(np.isinf(g), np.isinf(r)), what
        fin = np.isfinite(r)
        np.testing.assert_allclose(g[fin], r[fin], rtol=1e-15, atol=0, err_msg=what)


@pytest.mark.gpu
# N <= 64 runs the one-wave kernels (padded to 16/32/48/64 states), N > 64 the workgroup
# kernels; T > 64 crosses the 64-step observation blocks of the wave kernels
@pytest.mark.parametrize("n,v,frac,tmax", [(3, 5, 0.0, 30), (12, 30, 0.3, 150), (20, 30, 0.5, 200),
                                           (45, 60, 0.2, 130), (64, 40, 0.1, 70), (65, 40, 0.1, 40),
                                           (128, 40, 0.1, 30), (129, 40, 0.1, 30), (200, 50, 0.2, 40),
                                           (256, 40, 0.1, 24)])
def test_gpu_train_matches_oracle(gpu, n, v, frac, tmax):
    import cviterbi as cv

    off, obs, tags = _corpus(n, v, 27, tmax, frac, seed=100 + n)  # 27: a partly filled last block
    pi0, a0, b0 = _probs(n, v, seed=100 + n)
    iters = 3
    gp, ga, gb, it = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=iters, tol=0.0)
    assert it == iters
    rp, ra, rb, rit = FO.train(pi0, a0, b0, off, obs, tags, iters, 0.0)
    assert rit == iters
    for g, r, what in zip((gp, ga, gb), (rp, ra, rb), ("pi", "a", "b")):
        assert np.array_equal(np.isinf(g), np.isinf(r)), what
        fin = np.isfinite(r)
        np.testing.assert_allclose(g[fin], r[fin], rtol=0, atol=1e-9, err_msg=what)


@pytest.mark.gpu
# 64 < N <= 256 runs 32 sequences per workgroup (bw_fwd_mm / bw_bwd_mm): several workgroups,
# ragged lengths inside each (longest first), one-element sequences, tagged first/last
# elements, fully tagged sequences and a padded state count per kernel width (128/192/256);
# N > 256: the strided per-sequence kernels (2 and 3 states per thread)
@pytest.mark.parametrize("n,nseq,tmax,frac", [(65, 150, 40, 0.2), (100, 200, 60, 0.3), (128, 130, 33, 0.0),
                                              (150, 97, 50, 0.5), (192, 70, 45, 0.1), (255, 140, 30, 0.2),
                                              (256, 260, 40, 0.15), (257, 40, 20, 0.2), (300, 50, 25, 0.1),
                                              (520, 24, 16, 0.3)])
def test_gpu_train_groups_match_oracle(gpu, n, nseq, tmax, frac):
    import cviterbi as cv

    v = 37
    off, obs, tags = _corpus(n, v, nseq, tmax, frac, seed=500 + n)
    lengths = np.diff(off)
    # a fully tagged sequence and one with only its ends tagged
    k = int(np.argmax(lengths))
    tags[off[k]:off[k + 1]] = np.arange(lengths[k]) % n
    k2 = (k + 1) % nseq
    tags[off[k2]:off[k2 + 1]] = -1
    tags[off[k2]] = 3
    tags[off[k2 + 1] - 1] = n - 1
    pi0, a0, b0 = _probs(n, v, seed=500 + n)
    iters = 2
    gp, ga, gb, it = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=iters, tol=0.0)
    assert it == iters
    rp, ra, rb, _ = FO.train(pi0, a0, b0, off, obs, tags, iters, 0.0)
    for g, r, what in zip((gp, ga, gb), (rp, ra, rb), ("pi", "a", "b")):
        assert np.array_equal(np.isinf(g), np.isinf(r)), what
        fin = np.isfinite(r)
        np.testing.assert_allclose(g[fin], r[fin], rtol=0, atol=1e-9, err_msg=what)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [20, 100, 200, 300])  # wave, matrix-core and strided kernels
def test_gpu_train_subnormal_xi_denominator(gpu, n):
    """Emission probabilities below DBL_MIN for one observation make xi's normaliser c_t
    subnormal: the reference normalises xi entry by entry (hmm.rs:135-141) and stays finite;
    the kernels' factor alpha_t / c_t would overflow (inf * 0 = NaN in the sums) without the
    balanced power-of-two scaling (fit.hip xi_scale).  Two iterations against the oracle, to
    1e-3: the oracle's (the reference's) entry products alpha u a fall ~1e-315 and below, deep
    in the subnormal range where few bits remain, so it is itself only that accurate here."""
    import cviterbi as cv

    v = 12
    off, obs, tags = _corpus(n, v, 20, 30, 0.1, seed=300 + n)
    pi0, a0, b0 = _probs(n, v, seed=300 + n)
    b0[:, 3] = 1e-311 * (1.0 + np.arange(n) / n)  # subnormal
    assert np.count_nonzero(obs == 3) > 5
    gp, ga, gb, it = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=2, tol=0.0)
    rp, ra, rb, _ = FO.train(pi0, a0, b0, off, obs, tags, 2, 0.0)
    for g, r, what in zip((gp, ga, gb), (rp, ra, rb), ("pi", "a", "b")):
        assert not np.isnan(g).any(), what
        assert np.array_equal(np.isinf(g), np.isinf(r)), what
        fin = np.isfinite(r)
        np.testing.assert_allclose(g[fin], r[fin], rtol=0, atol=1e-3, err_msg=what)


@pytest.mark.gpu
def test_gpu_train_converges_like_oracle(gpu):
    import cviterbi as cv

    off, obs, tags = _corpus(6, 9, 30, 20, 0.5, seed=77)
    pi0, a0, b0 = _probs(6, 9, seed=77)
    gp, ga, gb, it = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=200, tol=1e-6)
    rp, ra, rb, rit = FO.train(pi0, a0, b0, off, obs, tags, 200, 1e-6)
    assert it == rit < 200
    np.testing.assert_allclose(ga, ra, rtol=0, atol=1e-8)


@pytest.mark.gpu
def test_gpu_fit_limits(gpu):
    import cviterbi as cv

    off, obs, tags = _corpus(300, 4, 3, 5, 0.5, seed=1)
    pi0, a0, b0 = _probs(300, 4, seed=1)
    with pytest.raises(cv.CVError):  # MLE needs every element tagged
        cv.fit_mle(pi0, a0, b0, off, obs, tags)


@pytest.mark.gpu
@pytest.mark.parametrize("n,nseq,tmax,forced", [(300, 50, 25, True), (520, 2100, 6, True), (4097, 5, 4, False)])
def test_gpu_train_global_scratch_match_oracle(gpu, monkeypatch, n, nseq, tmax, forced):
    """Baum-Welch beyond the LDS-resident vectors (N > 4,096: the strided kernels' step vector and
    gamma sums in global scratch, kBwScratchSeqs sequences per launch, the pi / a M-step over
    1,024 blocks) -- at N = 4,097 itself, and at N = 300 / 520 with tuning key bw_global = 1 (2,100
    sequences: two scratch batches) -- two EM iterations against the oracle (hmm.rs:69-190)."""
    import cviterbi as cv

    if forced:
        monkeypatch.setenv("CV_BW_GLOBAL", "1")
    v = 11
    off, obs, tags = _corpus(n, v, nseq, tmax, 0.25, seed=700 + n)
    pi0, a0, b0 = _probs(n, v, seed=700 + n)
    gp, ga, gb, it = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=2, tol=0.0)
    assert it == 2
    rp, ra, rb, _ = FO.train(pi0, a0, b0, off, obs, tags, 2, 0.0)
    for g, r, what in zip((gp, ga, gb), (rp, ra, rb), ("pi", "a", "b")):
        assert np.array_equal(np.isinf(g), np.isinf(r)), what
        fin = np.isfinite(r)
        np.testing.assert_allclose(g[fin], r[fin], rtol=0, atol=1e-9, err_msg=what)


@pytest.mark.gpu
# N = 20: the one-wave kernels on A 2^K; 100: the matrix-core kernels; 300: the strided ones
@pytest.mark.parametrize("n", [20, 100, 300])
def test_gpu_train_tiny_arcs_forced(gpu, n):
    """Arcs far below DBL_MIN's square root that tags force through: a 1e-306 arc
    p -> q and a subnormal 5e-320 arc p2 -> q2, each taken ~1,200 times by fully tagged
    sequences, so every step's xi is one-hot there and the factored sum sum_t r_t u_{t+1}
    (~1 / a per step) leaves the f64 range, and the subnormal arc's step normaliser c_t = fl(a u)
    keeps ~13 bits.  The E-step on A 2^K -- on whichever kernels N picks (since round 5 no
    path is selected for tiny arcs) -- keeps those counts exact: two EM iterations against the
    oracle (per-entry xi, hmm.rs:133-143)."""
    import cviterbi as cv

    v = 23
    rng = np.random.default_rng(7000 + n)
    pi0, a0, b0 = _probs(n, v, seed=7000 + n)
    p, q, p2, q2 = 1, 3, 5, 2
    a0[p, q] = 1e-306
    a0[p2, q2] = 5e-320
    a0 /= a0.sum(axis=1, keepdims=True)
    assert 0 < a0[p2, q2] < 2.3e-308  # still subnormal after the renormalisation
    tagged = [np.tile([p, q], 30), np.tile([p2, q2], 30)] * 20  # 1,200 forced steps per arc
    free = [rng.integers(0, n, size=int(rng.integers(5, 40))) for _ in range(30)]
    seqs = tagged + free
    lengths = np.array([len(x) for x in seqs])
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum(lengths, out=off[1:])
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    tags = np.full(int(off[-1]), -1, np.int32)
    for k in range(len(tagged)):
        tags[off[k]:off[k + 1]] = tagged[k]
    iters = 2
    gp, ga, gb, it = cv.fit_train(pi0, a0, b0, off, obs, tags, max_iter=iters, tol=0.0)
    assert it == iters
    rp, ra, rb, _ = FO.train(pi0, a0, b0, off, obs, tags, iters, 0.0)
    for g, r, what in zip((gp, ga, gb), (rp, ra, rb), ("pi", "a", "b")):
        assert np.array_equal(np.isinf(g), np.isinf(r)), what
        fin = np.isfinite(r)
        np.testing.assert_allclose(g[fin], r[fin], rtol=0, atol=1e-9, err_msg=what)
