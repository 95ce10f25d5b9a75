"""GPU: full-size BASELINE configs checked by size-independent properties (the oracle cannot
decode 33.5M-element batches in seconds), plus oracle samples.

* config 2 (N=45, 4,096 sequences, T <= 128) and config 3 (N=64, 16,384 sequences,
  T in [32, 1024]) -- the whole batches, not subsets: the exact-f64 decode equals the generic
  f64 kernel (an independent implementation with inline first-argmax) on every sequence, every
  f64 score is the f64 fold along its own path (what the reference recurrence computes,
  viterbi.rs:13-18 in f64), the f32 trellis is bit-exact vs the f32 oracle on the full
  config 2 and on a config-3 sample.
* config 5 (config 4 + one constrained position in half of 65,536 sequences, K = 7) in f64
  (the reference's precision) and f32: every constrained element takes its component's state,
  every status is clean, every score is the f64 re-score of its path (f64: the decode's own
  score, bit for bit), and sampled sequences equal the oracle's forced decode given the chosen
  component states.
"""
import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu


def _same(got, ref, what):
    for x, y, name in zip(got, ref, ("path", "score", "status")):
        bad = np.nonzero(np.asarray(x) != np.asarray(y))[0]
        assert bad.size == 0, f"{what}: {name} differs at {bad[:8]}"


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_full_config_f64_vs_generic_and_rescore(gpu, name):
    c = synth.config(name)
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    gen = cv.decode_batch(h, off, obs, dtype="f64", kernel="generic", rescore_f64=False)
    _same(got, gen, f"{name}: t64 vs generic f64")
    path, score, status = got
    assert np.all(status == 0)
    np.testing.assert_array_equal(score, O.rescore_batch_f64(pi, a, b, off, obs, path))


def test_full_config2_f32_vs_oracle(gpu):
    c = synth.config("c2")
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f32", rescore_f64=False)
    _same(got, O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32, nthreads=8), "c2 f32 full")


def test_config3_f32_sample_vs_oracle(gpu):
    c = synth.config("c3")
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    path, score, status = cv.decode_batch(h, off, obs, dtype="f32", rescore_f64=True)
    assert np.all(status == 0)
    # the f32 paths' scores are their f64 re-scores
    np.testing.assert_array_equal(score, O.rescore_batch_f64(pi, a, b, off, obs, path))
    for k in np.linspace(0, len(off) - 2, 96).astype(int):
        lo, hi = off[k], off[k + 1]
        rp, _, rst = O.decode_batch(pi, a, b, np.array([0, hi - lo]), obs[lo:hi], O.VITERBI, np.float32)
        assert rst[0] == status[k] and np.array_equal(rp, path[lo:hi]), f"seq {k}"


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_full_config5_properties(gpu, dtype):
    c = synth.config("c5")
    pi, a, b, off, obs, comp = c["pi"], c["a"], c["b"], c["offsets"], c["obs"], c["component"]
    h = cv.HMM(pi, a, b.reshape(256, 32, 32))
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, 7, dtype=dtype)
    assert np.all(status == 0)
    assert np.all(states >= 0)
    e = np.nonzero(comp >= 0)[0]
    assert np.array_equal(path[e], states[comp[e]]), "a constrained element left its component's state"
    # scores: f64 -- the decode's own max, which is the f64 fold along the path; f32 -- the
    # f64 re-score of the f32 path
    np.testing.assert_array_equal(score, O.rescore_batch_f64(pi, a, b, off, obs, path))
    assert obj == pytest.approx(float(np.sum(score)), rel=1e-12)
    # sampled sequences: the oracle's forced decode given the chosen component states
    dt = np.float64 if dtype == "f64" else np.float32
    forced = np.full(len(obs), -1, np.int32)
    forced[e] = states[comp[e]]
    seqs = np.unique(np.searchsorted(off, e, side="right") - 1)
    for k in np.concatenate([seqs[:: max(1, len(seqs) // 12)], [0, 1, 2]]):
        lo, hi = off[k], off[k + 1]
        rp, rs, rst = O.decode_batch(pi, a, b, np.array([0, hi - lo]), obs[lo:hi], O.VITERBI, dt,
                                     forced=forced[lo:hi])
        assert rst[0] == status[k] and np.array_equal(rp, path[lo:hi]), f"seq {k}"
        if dtype == "f64":
            assert rs[0] == score[k]


def test_full_config5_state_terms_sample(gpu):
    """The component STATES of full config 5 rest on the exact unary sums U_c(s) of ~32,768
    constrained sequences' max-marginals (csp.hpp).  This checks those terms independently: the
    GPU's exact partials of the full batch select the decode's states, and for a sample of 192
    constrained sequences (every component) the GPU's partial words equal the oracle's own
    max-marginals (oracle/c_oracle.py max_marginal, f64: forward row to t1 + reversed suffix
    pass, dp.rs:153-165 semantics) turned into exact integers (units of 2^-64), state by state."""
    from concurrent.futures import ThreadPoolExecutor

    c = synth.config("c5")
    pi, a, b, off, obs, comp = c["pi"], c["a"], c["b"], c["offsets"], c["obs"], c["component"]
    n, K = 256, 7
    h = cv.HMM(pi, a, b.reshape(n, 32, 32))
    _, _, status, states, _ = cv.decode_constrained(h, off, obs, comp, K, dtype="f64")
    assert np.all(status == 0) and np.all(states >= 0)
    full = cv.constrained_partials(h, off, obs, comp, K)
    sel, _ = cv.constrained_select(n, K, full)
    assert np.array_equal(sel, states), "the full partials select other states than the decode"
    # sample: constrained sequences spread over the batch
    e = np.nonzero(comp >= 0)[0]
    seqs = np.searchsorted(off, e, side="right") - 1
    pick = np.linspace(0, len(e) - 1, 192).astype(int)
    ks, ts = seqs[pick], e[pick]
    lens = off[ks + 1] - off[ks]
    so = synth.offsets_from_lengths(lens)
    sobs = np.concatenate([obs[off[k]:off[k + 1]] for k in ks]).astype(np.int32)
    scomp = np.concatenate([comp[off[k]:off[k + 1]] for k in ks]).astype(np.int32)
    gw = cv.constrained_partials(h, so, sobs, scomp, K)
    # oracle max-marginals of the sample (C restatement, threads: ctypes releases the GIL)
    with ThreadPoolExecutor(8) as ex:
        mus = list(ex.map(lambda q: O.max_marginal(pi, a, b, obs[off[ks[q]]:off[ks[q] + 1]],
                                                   int(ts[q] - off[ks[q]]), np.float64), range(len(ks))))
    words = 5 * n + 1
    for cc in range(K):
        mine = [q for q in range(len(ks)) if comp[ts[q]] == cc]
        assert mine, f"component {cc} not sampled"
        blk = gw[cc * words:(cc + 1) * words].astype(object)
        got = [int(blk[4 * s]) + (int(blk[4 * s + 1]) << 32) + (int(blk[4 * s + 2]) << 64) + (int(blk[4 * s + 3]) << 96)
               for s in range(n)]
        ninf = [int(x) for x in blk[4 * n:5 * n]]
        want, want_inf = [0] * n, [0] * n
        for q in mine:
            for s in range(n):
                x = float(mus[q][s])
                if x == -np.inf:
                    want_inf[s] += 1
                else:
                    want[s] += int(np.rint(x * 2.0 ** 64))
        assert int(blk[5 * n]) == len(mine)
        assert ninf == want_inf, f"component {cc}: -inf counts"
        bad = [s for s in range(n) if got[s] != want[s]]
        assert not bad, f"component {cc}: exact sums differ at states {bad[:8]}"
