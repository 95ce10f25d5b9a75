"""CPU: host-side mirror of the reference's solver interface -- loaders (src/utils.rs),
Constraints (constraints.rs), SuperSequence (viterbi_solver/utils.rs), output format
(main.rs:129-133)."""
import numpy as np
import pytest

import cviterbi as cv
from cviterbi import synth


@pytest.fixture
def hmm():
    pi, a, b = synth.random_hmm(4, 6, seed=1, zero_frac=0.2)
    return cv.HMM(pi, a, b.reshape(4, 3, 2))


def test_load_sequences_and_tags(tmp_path):
    (tmp_path / "sequences").write_text("0 1 0\n0 2 1\n1 0 1\n1 1\n1 2 0\n3 1 1\n")
    (tmp_path / "tags").write_text("0 2\n0 -1\n1 0\n1 1\n1 -1\n3 3\n")
    seqs = cv.load_sequences(tmp_path / "sequences", D=2)
    assert seqs == [[(1, 0), (2, 1)], [(0, 1), (1, 0), (2, 0)], [(1, 1)]]  # missing dim -> 0
    tags = cv.load_tags(tmp_path / "tags")
    assert tags == [[2, None], [0, 1, None], [3]]


def test_constraints_from_tags_and_file(tmp_path):
    c = cv.Constraints.from_tags([[None, 4], [4, 7, None], [7]])
    assert c.components == [{(0, 1), (1, 0)}, {(1, 1), (2, 0)}]
    (tmp_path / "c").write_text("0 1\n1 2\n\n3 3\n\n2 0\n2 5\n4 4\n")
    c2 = cv.Constraints.from_file(tmp_path / "c")
    assert c2.components == [{(0, 1), (1, 2)}, {(2, 0), (2, 5), (4, 4)}]  # singleton dropped


def test_supersequence_elements(hmm):
    seqs = [[(0, 1), (1, 0), (2, 1)], [(1, 1)], [(2, 0), (0, 0)]]
    cons = cv.Constraints.from_tags([[None, 5, None], [5], [None, 6]])
    ss = cv.SuperSequence(seqs, cons, hmm)
    assert len(ss) == 6
    assert ss.seq.tolist() == [0, 0, 0, 1, 2, 2] and ss.t.tolist() == [0, 1, 2, 0, 0, 1]
    assert ss.value.tolist() == [1, 2, 5, 3, 4, 0]
    assert ss.component.tolist() == [-1, 0, -1, 0, -1, 1]
    assert ss.last.tolist() == [0, 0, 0, 1, 0, 1]  # last active element of each component
    assert ss.number_constraints() == 2
    offs, obs, ids = ss.sequence_blocks()
    assert offs.tolist() == [0, 3, 4, 6] and ids.tolist() == [0, 1, 2]


def test_reorder_follows_reference_key(hmm):
    """utils.rs:105-136: sort by (last element constrained?, mean #emittable states, id)."""
    seqs = [[(0, 0), (1, 1)], [(2, 1)], [(1, 0), (0, 1), (2, 0)]]
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags([[None, 1], [None], [None, None, None]]), hmm)
    order = ss.get_sequences_ordering()
    fin = lambda o: np.isfinite(hmm.emit_probs(o)).sum()  # noqa: E731
    keys = []
    for sid, s in enumerate(seqs):
        vals = [hmm.flat(v) for v in s]
        keys.append((1 if sid == 0 else 0, sum(fin(v) for v in vals) / len(vals), sid))
    assert order == [k[2] for k in sorted(keys)]
    ss.recompute_constraints(1.0)
    assert ss.seq.tolist()[:len(seqs[order[0]])] == [order[0]] * len(seqs[order[0]])
    sol = np.arange(len(ss))
    per = ss.parse_solution(sol)
    assert [len(x) for x in per] == [2, 1, 3]


def test_stdrng_chacha_core_known_answer():
    """The ChaCha core of the restated rand 0.8 StdRng reproduces the published all-zero
    key / all-zero nonce ChaCha20 keystream block (djb layout, 64-bit counter)."""
    from cviterbi.stdrng import chacha_blocks

    blk = chacha_blocks([0] * 8, 0, 1, rounds=20)[0].astype("<u4").tobytes().hex()
    assert blk == ("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                   "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")


def test_recompute_constraints_draws(hmm):
    """utils.rs:168-177: one gen::<f64>() per element WITH a component, in element order,
    stream continuing across calls; prop=1 activates all, prop=0 (practically) none."""
    from cviterbi.stdrng import StdRng

    seqs = [[(0, 0), (1, 1), (2, 0)], [(1, 1), (0, 1)], [(2, 1)]]
    tags = [[1, None, 2], [None, 1], [2]]
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags(tags), hmm)
    ss.recompute_constraints(0.5)
    ref = StdRng(3019).gen_f64(8)
    # draws of the first call happen in the ORIGINAL element order (before reorder)
    orig_comp = [0, -1, 1, -1, 0, 1]
    act = [ref[i] <= 0.5 for i in range(4)]
    k = 0
    exp = {}
    for e, c in enumerate(orig_comp):
        if c != -1:
            exp[e] = act[k]
            k += 1
    got = {}
    for e in range(len(ss)):
        seq, t = int(ss.seq[e]), int(ss.t[e])
        oe = [0, 3, 5][seq] + t
        if orig_comp[oe] != -1:
            got[oe] = bool(ss.active[e])
    assert got == exp
    ss.recompute_constraints(1.0)
    assert ss.active.tolist() == (ss.component != -1).astype(int).tolist()


def test_write_output_format(tmp_path, hmm):
    class Fake(cv.Solver):
        def get_solution(self):
            return np.array([3, 1, 2])

        def get_objective(self):
            return -4.5

    ss = cv.SuperSequence([[(0, 0), (1, 1)], [(2, 0)]], None, hmm)
    p = tmp_path / "0_0"
    cv.write_output(p, Fake(), ss, elapsed_ms=12, explored_nodes=0)
    assert p.read_text() == "-4.5 0\n12\n0 3\n0 1\n1 2\n"
