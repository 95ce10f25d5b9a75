"""CPU: the oracle itself -- hand-derived known answers, exhaustive enumeration, the
numpy vs C restatements, and the committed golden fixtures.

Parity status: the reference (Rust) cannot be built or imported here and has no tests
or fixtures of its own, so the oracle is "parity unpinned" against
the binary; these tests pin it to the reference's stated semantics instead.
"""
import itertools
import math

import numpy as np
import pytest

import c_oracle as C
import np_oracle as NO
from conftest import load_golden
from cviterbi import synth

L10 = np.log10
MODES = {"viterbi": C.VITERBI, "cp": C.CP, "dp": C.DP, "decode": C.DECODE}


def _kat_model():
    pi = L10([0.6, 0.4])
    a = L10([[0.7, 0.3], [0.4, 0.6]])
    b = L10([[0.9, 0.1], [0.2, 0.8]])
    return pi, a, b


def test_kat_two_state_viterbi():
    """Worked by hand in probability space: d0=[.54,.08]; t1 (o=1): [.0378 (psi 0), .1296 (psi 0)];
    t2 (o=1): [.005184 (psi 1), .062208 (psi 1)] -> end 1, path [0,1,1], score log10(.062208)."""
    pi, a, b = _kat_model()
    obs = np.array([0, 1, 1], np.int32)
    for dt in (np.float64, np.float32):
        p, s, st = C.decode_batch(pi, a, b, [0, 3], obs, C.VITERBI, dt)
        assert st[0] == 0 and p.tolist() == [0, 1, 1]
        assert s[0] == pytest.approx(math.log10(0.062208), abs=1e-5 if dt == np.float32 else 1e-12)
        for m in (C.CP, C.DP):
            p2, s2, _ = C.decode_batch(pi, a, b, [0, 3], obs, m, dt)
            assert p2.tolist() == [0, 1, 1]


def test_kat_decode_compat_row0_zero():
    """viterbi::decode leaves row 0 at 0.0 (viterbi.rs:6,9): d0=[1,1] in probability;
    t1: [.07 (psi 0), .48 (psi 1)]; t2: [.0192 (psi 1), .2304 (psi 1)] -> path [1,1,1]."""
    pi, a, b = _kat_model()
    obs = np.array([0, 1, 1], np.int32)
    p, s, _ = C.decode_batch(pi, a, b, [0, 3], obs, C.DECODE, np.float64)
    assert p.tolist() == [1, 1, 1]
    assert s[0] == pytest.approx(math.log10(0.2304), abs=1e-12)


def test_kat_all_ties_first_index():
    pi = L10([0.5, 0.5])
    a = np.full((2, 2), L10(0.5))
    b = np.full((2, 3), L10(0.5))
    obs = np.array([0, 2, 1, 1, 0], np.int32)
    for m in MODES.values():
        for dt in (np.float32, np.float64):
            p, _, _ = C.decode_batch(pi, a, b, [0, 5], obs, m, dt)
            assert p.tolist() == [0, 0, 0, 0, 0]


def test_kat_single_step_and_empty():
    pi = L10([0.2, 0.5, 0.3])
    a = L10(np.full((3, 3), 1 / 3))
    b = L10([[0.5, 0.5], [0.1, 0.9], [0.9, 0.1]])
    p, s, st = C.decode_batch(pi, a, b, [0, 0, 1, 1], np.array([0], np.int32), C.VITERBI, np.float64)
    # seq 0 empty, seq 1 = [o=0]: d0 = [.1, .05, .27] -> state 2, seq 2 empty
    assert st.tolist() == [2, 0, 2] and p.tolist() == [2]
    assert s[1] == pytest.approx(math.log10(0.27), abs=1e-12) and s[0] == 0.0 and s[2] == 0.0


def test_kat_infeasible():
    pi = L10([0.5, 0.5])
    a = np.array([[0.0, -np.inf], [-np.inf, 0.0]])  # log10(1) / log10(0)
    b = np.array([[0.0, -np.inf], [-np.inf, 0.0]])  # state 0 emits only 0, state 1 only 1
    obs = np.array([0, 1], np.int32)  # would need a 0 -> 1 transition: impossible
    for m in MODES.values():
        if m == C.DECODE:
            continue
        p, s, st = C.decode_batch(pi, a, b, [0, 2], obs, m, np.float64)
        assert st[0] == 1 and s[0] == -np.inf and p.tolist() == [0, 0]


def test_kat_decode_infeasible_backtracks_from_argmax0():
    """viterbi::decode on an infeasible sequence (viterbi.rs:19-30): the last row is all -inf,
    argmax gives 0 (first index), and the backtrack follows bt, which is 0 where the emission
    is -inf but a real first argmax elsewhere.  Worked by hand (log10 values):
      row 0 = [0, 0] (viterbi.rs:6, 9)
      t1 (o=0): to 0: max(0 + -1, 0 + -0.25) -> psi 1, -0.25 + -0.5 = -0.75
                to 1: max(0 + -0.5, 0 + -2) -> psi 0, -0.5 + -1 = -1.5
      t2 (o=2): emission -inf in both states -> row -inf, bt 0
      end = argmax([-inf, -inf]) = 0; path[1] = bt[2][0] = 0; path[0] = bt[1][0] = 1
    so the reference returns [1, 0, 0] -- not the all-zero path of an infeasible CP/DP decode."""
    pi = np.array([-0.3, -0.3])
    a = np.array([[-1.0, -0.5], [-0.25, -2.0]])
    b = np.array([[-0.5, -1.0, -np.inf], [-1.0, -0.5, -np.inf]])
    obs = np.array([0, 0, 2], np.int32)
    for dt in (np.float64, np.float32):
        p, s, st = C.decode_batch(pi, a, b, [0, 3], obs, C.DECODE, dt)
        assert st[0] == 1 and s[0] == -np.inf and p.tolist() == [1, 0, 0]
        p2, s2, st2 = NO.decode(pi, a, b, obs, NO.DECODE, dt)
        assert st2 == 1 and p2.tolist() == [1, 0, 0]
    # an emission that is -inf mid-sequence resets bt to 0 there: obs [0, 2, 0] -> t1 row
    # -inf with bt 0, t2 row -inf (all predecessors -inf: first argmax 0) -> [0, 0, 0]
    p, _, st = C.decode_batch(pi, a, b, [0, 3], np.array([0, 2, 0], np.int32), C.DECODE, np.float64)
    assert st[0] == 1 and p.tolist() == [0, 0, 0]


@pytest.mark.parametrize("seed", range(40))
def test_c_matches_numpy_restatement(seed):
    n = [1, 2, 3, 5, 8, 13][seed % 6]
    v = 1 + seed % 7
    pi, a, b = synth.random_hmm(n, v, seed=seed, zero_frac=[0.0, 0.1, 0.4][seed % 3])
    rng = np.random.default_rng(seed)
    off = synth.offsets_from_lengths(rng.integers(0, 12, size=5))
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    for name, m in MODES.items():
        for dt in (np.float32, np.float64):
            cp, cs, cst = C.decode_batch(pi, a, b, off, obs, m, dt)
            npp, ns, nst = NO.decode_batch(pi, a, b, off, obs, m, dt)
            assert np.array_equal(cst, nst) and np.array_equal(cp, npp) and np.array_equal(cs, ns), (name, dt)


@pytest.mark.parametrize("seed", range(30))
def test_dp_equals_exhaustive_enumeration(seed):
    n = 2 + seed % 3
    T = 1 + seed % 6
    pi, a, b = synth.random_hmm(n, 4, seed=seed, zero_frac=0.2 if seed % 2 else 0.0)
    obs = np.random.default_rng(seed).integers(0, 4, size=T).astype(np.int32)
    for dt in (np.float32, np.float64):
        p, s, st = C.decode_batch(pi, a, b, [0, T], obs, C.VITERBI, dt)
        bp, bs, bst, nopt = NO.brute_force(pi, a, b, obs, dt)
        assert st[0] == bst
        if bst == 0:
            assert s[0] == float(bs)
            if nopt == 1:
                assert np.array_equal(p, bp)


def test_exhaustive_dyadic_ties():
    """Dyadic values: exact arithmetic, many optimal paths; the DP's first-index backtrack
    equals the optimal path with the lexicographically smallest reversed state sequence."""
    rng = np.random.default_rng(5)
    for trial in range(25):
        n, T = 3, 5
        q = lambda s: -rng.integers(0, 5, size=s) / 2.0  # noqa: E731
        pi, a, b = q(n), q((n, n)), q((n, 3))
        obs = rng.integers(0, 3, size=T).astype(np.int32)
        for dt in (np.float32, np.float64):
            p, s, _ = C.decode_batch(pi, a, b, [0, T], obs, C.VITERBI, dt)
            bp, bs, _, nopt = NO.brute_force(pi, a, b, obs, dt)
            assert s[0] == bs and np.array_equal(p, bp), (trial, nopt)


@pytest.mark.parametrize("name", ["golden_small.npz", "golden_ties.npz", "golden_inf.npz", "golden_ar_house_a.npz"])
def test_golden_fixtures_c_oracle(name):
    g = load_golden(name)
    for key, dt in (("f32", np.float32), ("f64", np.float64)):
        for mname, m in MODES.items():
            p, s, st = C.decode_batch(g["pi"], g["a"], g["b"], g["offsets"], g["obs"], m, dt)
            assert np.array_equal(st, g[f"{key}_{mname}_status"])
            assert np.array_equal(p, g[f"{key}_{mname}_path"])
            assert np.array_equal(s, g[f"{key}_{mname}_score"])


def test_rescore_matches_decode_f64():
    """The f64 row-A0 re-score of the f64 decoded path equals the f64 decode score."""
    pi, a, b = synth.random_hmm(16, 9, seed=2)
    rng = np.random.default_rng(2)
    off = synth.offsets_from_lengths(rng.integers(1, 40, size=10))
    obs = rng.integers(0, 9, size=int(off[-1])).astype(np.int32)
    p, s, _ = C.decode_batch(pi, a, b, off, obs, C.VITERBI, np.float64)
    for k in range(10):
        lo, hi = off[k], off[k + 1]
        assert C.rescore_f64(pi, a, b, obs[lo:hi], p[lo:hi]) == s[k]


def test_cp_superseq_vs_per_sequence():
    """utils.rs:24-38 boundary semantics: the CP super-sequence objective is the sum of the
    per-sequence optima (up to the rounding of the running offset)."""
    pi, a, b = synth.random_hmm(6, 5, seed=8)
    rng = np.random.default_rng(8)
    off = synth.offsets_from_lengths(rng.integers(1, 15, size=7))
    obs = rng.integers(0, 5, size=int(off[-1])).astype(np.int32)
    path, obj = C.cp_superseq_f64(pi, a, b, off, obs)
    p, s, _ = C.decode_batch(pi, a, b, off, obs, C.CP, np.float64)
    assert obj == pytest.approx(float(np.sum(s)), rel=1e-12)
    assert np.array_equal(path, p)


# ---- consistency-constrained decode spec (np_oracle.constrained_decode) -------------------
def _constrained_case(seed, n=3, v=4, nseq=6, tmax=6, ncomp=2, p=0.7, maxpos=1):
    pi, a, b = synth.random_hmm(n, v, seed=seed)
    rng = np.random.default_rng(seed)
    lengths = rng.integers(1, tmax, size=nseq)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    comp = np.full(len(obs), -1, np.int32)
    for k in range(nseq):
        if rng.random() < p:
            m = int(rng.integers(1, maxpos + 1))
            for t in rng.choice(lengths[k], size=min(m, lengths[k]), replace=False):
                comp[off[k] + t] = rng.integers(0, ncomp)
    return pi, a, b, off, obs, comp


@pytest.mark.parametrize("seed", range(25))
def test_constrained_spec_is_exact_optimum(seed):
    """With one constrained position per sequence the components decouple, so summing the
    max-marginals per component and forcing the best state gives the exhaustive optimum
    over all component-state assignments (f64; equal objective, tolerance 1e-12 rel)."""
    pi, a, b, off, obs, comp = _constrained_case(seed)
    states, forced = NO.constrained_decode(pi, a, b, off, obs, comp, np.float64)
    p, s, st = C.decode_batch(pi, a, b, off, obs, C.VITERBI, np.float64, forced=forced)
    best, bobj = NO.constrained_brute(pi, a, b, off, obs, comp, np.float64)
    obj = float(np.sum(np.where(st == 0, s, -np.inf)))
    assert obj == pytest.approx(bobj, rel=1e-12)
    for e in np.nonzero(comp >= 0)[0]:
        assert p[e] == states[int(comp[e])]  # every constrained element takes its component's state


@pytest.mark.parametrize("seed", range(30))
def test_constrained_multi_position_spec_is_exact_optimum(seed):
    """Several constrained positions per sequence (pairwise component terms, segment
    tables): the spec's exact search reaches the exhaustive optimum over all component-state
    assignments (f64 objective within 1e-12 rel), with 2-3 components linked in groups."""
    pi, a, b, off, obs, comp = _constrained_case(seed, n=3, v=4, nseq=5, tmax=8, ncomp=3, p=0.9, maxpos=3)
    states, forced = NO.constrained_decode(pi, a, b, off, obs, comp, np.float64)
    p, s, st = C.decode_batch(pi, a, b, off, obs, C.VITERBI, np.float64, forced=forced)
    _, bobj = NO.constrained_brute(pi, a, b, off, obs, comp, np.float64)
    obj = float(np.sum(np.where(st == 0, s, -np.inf)))
    if bobj == -np.inf:
        assert obj == -np.inf
    else:
        assert obj == pytest.approx(bobj, rel=1e-12)
    for e in np.nonzero(comp >= 0)[0]:
        assert p[e] == states[int(comp[e])]


def test_segment_table_matches_forced_decode():
    """M[s, s'] (start in s with score 0, run to s') == the forced-decode score of the segment
    with both ends forced minus nothing: checked against decode_forced with a zero-emission
    first element (pi = 0 at s), f64."""
    pi, a, b = synth.random_hmm(4, 5, seed=4)
    obs = np.array([1, 3, 0, 4, 2], np.int32)
    M = NO.segment_table(a, b, obs, np.float64)
    for s in range(4):
        for s2 in range(4):
            best = -np.inf
            for mid in itertools.product(range(4), repeat=len(obs) - 2):
                path = (s,) + mid + (s2,)
                v = sum(a[path[t - 1], path[t]] + b[path[t], obs[t]] for t in range(1, len(obs)))
                best = max(best, v)
            assert M[s, s2] == pytest.approx(best, abs=1e-12)


@pytest.mark.parametrize("seed", range(8))
def test_constrained_spec_numpy_vs_c(seed):
    pi, a, b, off, obs, comp = _constrained_case(seed, n=6, v=5, nseq=9, tmax=12, ncomp=3)
    for dt in (np.float32, np.float64):
        s1, f1 = NO.constrained_decode(pi, a, b, off, obs, comp, dt)
        s2, f2 = C.constrained_forced(pi, a, b, off, obs, comp, dt)
        assert s1 == s2


def test_forced_decode_c_vs_numpy():
    pi, a, b = synth.random_hmm(7, 5, seed=3, zero_frac=0.1)
    rng = np.random.default_rng(3)
    off = synth.offsets_from_lengths(rng.integers(1, 15, size=10))
    obs = rng.integers(0, 5, size=int(off[-1])).astype(np.int32)
    forced = np.where(rng.random(len(obs)) < 0.2, rng.integers(0, 7, size=len(obs)), -1).astype(np.int32)
    for dt in (np.float32, np.float64):
        p, s, st = C.decode_batch(pi, a, b, off, obs, C.VITERBI, dt, forced=forced)
        for k in range(10):
            lo, hi = off[k], off[k + 1]
            q, sc, sst = NO.decode_forced(pi, a, b, obs[lo:hi], forced[lo:hi], dt)
            assert sst == st[k]
            if sst == 0:
                assert np.array_equal(q, p[lo:hi]) and float(sc) == s[k]
                assert all(p[lo + t] == forced[lo + t] for t in range(hi - lo) if forced[lo + t] >= 0)
