"""CPU: the exact component-state search behind the constrained decode (csp.cpp via the
host-only C-ABI calls cv_constrained_pairs / cv_constrained_select) against the oracle's
brute force (oracle/np_oracle.py constrained_solve) on random exact-integer terms with
ties, -inf entries, several connected groups and limb carries."""
import itertools

import numpy as np
import pytest

import np_oracle as NO
from cviterbi.decode import constrained_pairs, constrained_select, partial_words

M32 = (1 << 32) - 1


def pack(U, P, n, ncomp, pairs):
    """Test-side packing of include/cviterbi.h's CV_PARTIAL_WORDS layout."""
    part = np.zeros(partial_words(n, ncomp, len(pairs)), np.int64)
    uw, pw = 5 * n + 1, 5 * n * n + 1

    def put(base, idx, x, nent):
        if x is None:
            part[base + 4 * nent + idx] += 1
        else:
            part[base + 4 * idx:base + 4 * idx + 4] += [x & M32, (x >> 32) & M32, (x >> 64) & M32, x >> 96]

    for c, vec in U.items():
        part[c * uw + 5 * n] += 1
        for s, x in enumerate(vec):
            put(c * uw, s, x, n)
    for p, (c1, c2) in enumerate(pairs):
        if (c1, c2) not in P:
            continue
        base = ncomp * uw + p * pw
        part[base + 5 * n * n] += 1
        for s1 in range(n):
            for s2 in range(n):
                put(base, s1 * n + s2, P[(c1, c2)][s1][s2], n * n)
    return part


def rand_terms(rng, n, comps, pair_list, ninf=0.1, scale=1 << 70, coarse=False):
    def val():
        if rng.random() < ninf:
            return None
        if coarse:  # many exact ties
            return int(rng.integers(-3, 3)) << 60
        return int(rng.integers(-(1 << 62), 1 << 62)) * int(rng.integers(1, scale >> 62)) - (1 << 80)

    U = {c: [val() for _ in range(n)] for c in comps}
    P = {pr: [[val() for _ in range(n)] for _ in range(n)] for pr in pair_list}
    return U, P


@pytest.mark.parametrize("seed", range(40))
def test_select_matches_brute_force(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 6))
    ncomp = int(rng.integers(2, 7))
    comps = sorted(set(rng.choice(ncomp, size=int(rng.integers(1, ncomp + 1)), replace=False).tolist()))
    all_pairs = [(c1, c2) for c1, c2 in itertools.combinations(comps, 2)]
    k = int(rng.integers(0, len(all_pairs) + 1)) if all_pairs else 0
    pair_list = sorted(all_pairs[i] for i in rng.choice(len(all_pairs), size=k, replace=False)) if k else []
    while any(n ** len(g) > 20000 for g in [comps]):  # keep brute force small
        comps = comps[:-1]
        pair_list = [p for p in pair_list if p[0] in comps and p[1] in comps]
    U, P = rand_terms(rng, n, comps, pair_list, ninf=[0.0, 0.1, 0.4][seed % 3], coarse=seed % 2 == 1)
    want = NO.constrained_solve(U, P, n)
    pairs = np.array(pair_list, np.int32).reshape(-1, 2)
    got, explored = constrained_select(n, ncomp, pack(U, P, n, ncomp, pair_list), pairs)
    for c in range(ncomp):
        assert got[c] == want.get(c, -1), (c, got.tolist(), want)
    assert explored >= n * len(comps) or all(v == -1 for v in want.values())


def test_select_chain_of_seven_components():
    """A 7-component chain at n = 8 (8^7 = 2.1M assignments): branch and bound must reach
    the optimum of a planted solution with strong pairwise agreement terms."""
    rng = np.random.default_rng(7)
    n, comps = 8, list(range(7))
    plant = rng.integers(0, n, size=7)
    U = {c: [int(rng.integers(0, 1 << 40)) for _ in range(n)] for c in comps}
    P = {}
    for c in range(6):
        P[(c, c + 1)] = [[(1 << 50) if (s1 == plant[c] and s2 == plant[c + 1]) else int(rng.integers(0, 1 << 40))
                          for s2 in range(n)] for s1 in range(n)]
    got, _ = constrained_select(n, 7, pack(U, P, n, 7, sorted(P)), np.array(sorted(P), np.int32))
    assert got.tolist() == plant.tolist()


def test_pairs_from_components():
    off = np.array([0, 4, 7, 9], np.int64)
    comp = np.array([2, -1, 0, 2,   1, 1, -1,   3, 0], np.int32)
    pairs = constrained_pairs(off, comp, 4)
    # seq 0: 2 -> 0 -> 2 gives (0,2) twice; seq 1: 1 -> 1 (same component, no pair); seq 2: 3 -> 0
    assert pairs.tolist() == [[0, 2], [0, 3]]
