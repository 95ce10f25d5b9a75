"""CFN export (cfn.rs:11-205): cv_solver_write_cfn against the Python
restatement oracle/cfn_oracle.py, byte for byte.

CPU: the oracle's longest path against brute-force enumeration of state sequences (an
independent statement of cfn.rs:11-34), and Rust `{}` float formatting on known cases.
GPU: the file the library writes equals the oracle's text for random super-sequences with
sequence crossings, repeated components, -inf transitions/emissions and every component
active; error statuses where the reference would panic."""
import itertools
import math

import numpy as np
import pytest

import cfn_oracle as CO
from cviterbi import cli, synth

RUST = [(0.1, "0.1"), (1.0, "1"), (-0.0, "-0"), (0.0, "0"), (1e-7, "0.0000001"), (1e21, "1000000000000000000000"),
        (123.456, "123.456"), (-1.5e-5, "-0.000015"), (-12.25, "-12.25"), (2.0 ** 60, "1152921504606847000"),
        (-math.inf, "-inf"), (math.inf, "inf"), (float("nan"), "NaN"), (5e-324, "0." + "0" * 323 + "5")]


@pytest.mark.parametrize("x,s", RUST)
def test_rust_float_display(x, s):
    assert CO.rust_display(x) == s
    assert cli.rust_f64(x) == s


def _brute_longest(pi, a, b, value, comp, first, t_from, n_from, t_to, n_to):
    """max over every state sequence on (t_from, t_to] of the left-to-right f64 sum
    ((score + transition) + emission per step) with constrained elements forced."""
    N = len(pi)
    best = -math.inf
    steps = list(range(t_from + 1, t_to + 1))
    for states in itertools.product(range(N), repeat=len(steps)):
        prev, score, ok = n_from, 0.0, True
        for t, s in zip(steps, states):
            if comp[t] >= 0 and s != (n_from if t < t_to else n_to):
                ok = False
                break
            score = score + (pi[s] if first[t] else a[prev][s]) + b[s][value[t]]
            prev = s
        if ok:
            best = max(best, score)
    return best


def test_oracle_longest_path_vs_enumeration():
    pi, a, b = synth.random_hmm(3, 4, seed=3)
    pi, a, b = pi.tolist(), a.tolist(), b.tolist()
    a[1][2] = -math.inf
    value = [0, 3, 1, 2, 0, 1]
    first = [1, 0, 0, 1, 0, 0]
    comp = [0, -1, 0, -1, -1, 1]
    for n1 in range(3):
        for n2 in range(3):
            got = CO.longest_path(pi, a, b, value, comp, first, 0, n1, 5, n2)
            ref = _brute_longest(pi, a, b, value, comp, first, 0, n1, 5, n2)
            # f64 rounding is monotone, so the DP's greedy max equals the best path sum exactly
            assert got == ref, (n1, n2)


def _problem(n, v, nseq, ncomp, seed, neg=False):
    import cviterbi as cv

    pi, a, b = synth.random_hmm(n, v, seed=seed)
    if neg:
        a[0, n - 1] = -np.inf
        b[n - 1, 0] = -np.inf
    rng = np.random.default_rng(seed)
    seqs = [[(int(x), 0) for x in rng.integers(0, v, size=int(t))] for t in rng.integers(1, 9, size=nseq)]
    tags = [[(int(rng.integers(0, ncomp)) if rng.random() < 0.3 else None) for _ in s] for s in seqs]
    free = [(i, t) for i, s in enumerate(seqs) for t in range(len(s)) if tags[i][t] is None]
    for c, j in zip(range(ncomp), rng.permutation(len(free))):  # every component at least once
        i, t = free[j]
        tags[i][t] = c
    h = cv.HMM(pi, a, b.reshape(n, v, 1), bdims=(v, 1))
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags(tags), h)
    ss.recompute_constraints(1.0)
    return pi, a, b, h, ss


def _oracle_text(pi, a, b, ss):
    comp = np.where(ss.active == 1, ss.component, -1).tolist()
    return CO.write_cfn_text(pi.tolist(), a.tolist(), b.tolist(), ss.value.tolist(), comp, (ss.t == 0).astype(int).tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("n,v,nseq,ncomp,neg", [(2, 3, 4, 2, False), (3, 5, 6, 3, True), (7, 6, 8, 3, False),
                                                (16, 9, 5, 4, True)])
def test_gpu_cfn_matches_oracle(gpu, tmp_path, n, v, nseq, ncomp, neg):
    import cviterbi as cv

    pi, a, b, h, ss = _problem(n, v, nseq, ncomp, seed=10 * n + nseq, neg=neg)
    if ss.number_constraints() != ncomp:
        pytest.skip("sampling left a component without active positions")
    s = cv.GpuSolver(h, ss, "gpu")
    path = tmp_path / "problem.cfn"
    ms = s.write_cfn(path)
    assert ms >= 0
    got = path.read_text()
    ref = _oracle_text(pi, a, b, ss)
    assert got == ref


@pytest.mark.gpu
def test_gpu_cfn_errors(gpu, tmp_path):
    import cviterbi as cv

    pi, a, b = synth.random_hmm(3, 4, seed=1)
    h = cv.HMM(pi, a, b.reshape(3, 4, 1), bdims=(4, 1))
    seqs = [[(0, 0), (1, 0)], [(2, 0)]]
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags([[None, None], [None]]), h)
    with pytest.raises(cv.CVError):  # no constraint: the reference unwraps an empty list
        cv.GpuSolver(h, ss, "gpu").write_cfn(tmp_path / "x.cfn")
    # component 1 active, component 0 without active position: cost tables sized by the
    # number of active components, indexed by component id (out of bounds in the reference)
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags([[0, 1], [None]]), h)
    ss.active[ss.component == 0] = 0
    with pytest.raises(cv.CVError):
        cv.GpuSolver(h, ss, "gpu").write_cfn(tmp_path / "y.cfn")
