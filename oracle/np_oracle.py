"""numpy restatement of the reference Viterbi decode path + exhaustive enumerator.

TEST INFRASTRUCTURE ONLY: used in this container to cross-check the C oracle
(oracle/cv_oracle.c) and to generate the committed golden fixtures under
tests/golden/.  Never imported by the product package.

Parity status: "parity unpinned" against the reference binary (a Rust crate that
cannot be built or run here, with no tests or fixtures of its own; SURVEY.md §4,
§8c).  Pinned instead by exhaustive enumeration (`brute_force`) and hand-derived
known answers (tests/test_oracle_kat.py).

Semantics follow SURVEY.md §8a (file:line into /root/reference/src):
  VITERBI (row A0)  d0 = pi + b[:,o0] (hmm/hmm.rs:215-218, viterbi_solver/cp.rs:66-68);
                    s = d[:,None] + a; psi = first argmax; d' = max(s) + b[:,o]
                    (viterbi_solver/viterbi.rs:13-18).
  CP                psi as above; d'[j] = d[psi] + (a[psi,j] + b[j,o])
                    (cp.rs:70-78 via utils.rs:24-30 -> hmm.rs:220-222).
  DP                c = (a + b[None,:,o]) + d[:,None] over finite entries; first max
                    (dp.rs:127-177, ascending-index iteration instead of HashMap order).
  DECODE            viterbi.rs:5-32: row 0 = 0.0, -inf emission -> -inf, bt 0; an infeasible
                    sequence still backtracks from argmax 0 (viterbi.rs:24-30).
"""
from __future__ import annotations

import itertools

import numpy as np

VITERBI, CP, DP, DECODE = 0, 1, 2, 3
SEQ_OK, SEQ_INFEASIBLE, SEQ_EMPTY = 0, 1, 2


def decode(pi, a, b, obs, assoc=VITERBI, dtype=np.float64):
    """Decode one sequence. pi[N], a[N,N] (from,to), b[N,V]; returns (path, score, status)."""
    pi = np.asarray(pi, dtype=dtype)
    a = np.asarray(a, dtype=dtype)
    b = np.asarray(b, dtype=dtype)
    obs = np.asarray(obs, dtype=np.int64)
    n = a.shape[0]
    T = obs.shape[0]
    if T == 0:
        return np.zeros(0, np.int32), dtype(0), SEQ_EMPTY
    ninf = dtype(-np.inf)
    e0 = b[:, obs[0]]
    if assoc == DECODE:
        prev = np.zeros(n, dtype)
    elif assoc == DP:
        prev = np.where(e0 > ninf, pi + e0, ninf).astype(dtype)
    else:
        prev = (pi + e0).astype(dtype)
    bt = np.zeros((T, n), np.int32)
    cols = np.arange(n)
    for t in range(1, T):
        e = b[:, obs[t]]
        if assoc == DP:
            arc = a + e[None, :]
            c = arc + prev[:, None]
            c = np.where(np.isfinite(prev)[:, None] & (arc > ninf), c, ninf)
            arg = np.argmax(c, axis=0)
            cur = c[arg, cols]
            cur = np.where(e > ninf, cur, ninf)
            arg = np.where(e > ninf, arg, 0)
        else:
            s = prev[:, None] + a
            arg = np.argmax(s, axis=0)  # first maximal index, like ndarray-stats argmax
            m = s[arg, cols]
            if assoc == CP:
                cur = prev[arg] + (a[arg, cols] + e)
            else:
                cur = m + e
            if assoc == DECODE:
                dead = ~(e > ninf)
                cur = np.where(dead, ninf, cur)
                arg = np.where(dead, 0, arg)
        bt[t] = arg
        prev = cur.astype(dtype)
    end = int(np.argmax(prev))
    best = prev[end]
    path = np.zeros(T, np.int32)
    if not best > ninf and assoc != DECODE:
        return path, ninf, SEQ_INFEASIBLE
    # viterbi.rs:24-30 backtracks from argmax 0 of an all -inf last row too (bt left 0 where
    # the emission is -inf); the other solvers panic there (cp.rs:87, dp.rs:184-186)
    cs = end
    for t in range(T - 1, -1, -1):
        path[t] = cs
        cs = bt[t, cs]
    if not best > ninf:
        return path, ninf, SEQ_INFEASIBLE
    return path, best, SEQ_OK


def decode_batch(pi, a, b, offsets, obs, assoc=VITERBI, dtype=np.float64):
    nseq = len(offsets) - 1
    path = np.zeros(int(offsets[-1]), np.int32)
    score = np.zeros(nseq, np.float64)
    status = np.zeros(nseq, np.uint8)
    for s in range(nseq):
        lo, hi = int(offsets[s]), int(offsets[s + 1])
        p, sc, st = decode(pi, a, b, obs[lo:hi], assoc, dtype)
        path[lo:hi] = p
        score[s] = float(sc)
        status[s] = st
    return path, score, status


def path_score(pi, a, b, obs, path, dtype=np.float64):
    """Row-A0 float score of a fixed path: d=(d + a[p,q]) + b[q,o], sequential rounding."""
    pi = np.asarray(pi, dtype)
    a = np.asarray(a, dtype)
    b = np.asarray(b, dtype)
    d = pi[path[0]] + b[path[0], obs[0]]
    for t in range(1, len(obs)):
        d = d + a[path[t - 1], path[t]]
        d = d + b[path[t], obs[t]]
    return d


def brute_force(pi, a, b, obs, dtype=np.float64):
    """Exhaustive Viterbi: max float score over all N^T paths (row-A0 per-path rounding).

    Float addition is monotone, so the DP's delta equals this maximum exactly.  The DP
    backtrack's tie rule (first argmax at the end, then first argmax of each
    predecessor sum) selects, among optimal paths, the one whose REVERSED state
    sequence is lexicographically smallest -- exactly so whenever the arithmetic is
    exact (dyadic test values); with rounded arithmetic two paths whose pre-emission
    sums differ can still round to one total, so callers compare paths only when
    `n_opt == 1` or the values are dyadic.  Returns (path, score, status, n_opt).
    """
    pi = np.asarray(pi, dtype)
    a = np.asarray(a, dtype)
    b = np.asarray(b, dtype)
    n = a.shape[0]
    T = len(obs)
    paths = np.array(list(itertools.product(range(n), repeat=T)), dtype=np.int64)
    d = pi[paths[:, 0]] + b[paths[:, 0], obs[0]]
    for t in range(1, T):
        d = d + a[paths[:, t - 1], paths[:, t]]
        d = d + b[paths[:, t], obs[t]]
    best = d.max()
    if not best > -np.inf:
        return np.zeros(T, np.int32), dtype(-np.inf), SEQ_INFEASIBLE, 0
    cand = paths[d == best]
    # np.lexsort(keys) sorts by keys[-1] first; cand.T rows are t=0..T-1, so the primary
    # key is t=T-1, then T-2, ...: lexicographic order of the reversed sequence.
    order = np.lexsort(cand.T)
    return cand[order[0]].astype(np.int32), best, SEQ_OK, int(cand.shape[0])


# ---------------------------------------------------------------------------------------
# Consistency-constrained decode (intended semantics of
# opti.rs:101-111 / dp.rs:157-164): every ACTIVE position of a component decodes to one
# common state; maximise the total log-likelihood.  Spec used by the GPU path when each
# sequence has at most one active constrained position (the components then decouple):
#   mu_k(s)  = delta_{t_k}(s) + beta_{t_k}(s)           (max-marginal at the position)
#     delta  : row-A0 forward over elements 0..t_k            (dtype)
#     g      : the same recurrence run BACKWARD with a^T and pi = 0 over T-1..t_k+1,
#              g_t[i] = max_j(g_{t+1}[j] + a[i,j]) + b[i,o_t]  (dtype)
#     beta   : max_j(g_{t_k+1}[j] + a[i,j]), 0 when t_k = T-1  (dtype)
#   U_c(s)   = sum over the component's sequences of round(mu_k(s) * 2^64) as exact
#              integers (order- and rank-count independent); -inf terms exclude s
#   s_c      = first argmax of U_c; then a forced decode with s_c at every active position.
# Several positions per sequence add alpha / segment-table / beta terms and pairwise terms
# between components (constrained_terms below); the search is then exact over the
# component groups they link (constrained_solve).
def forward_last_row(pi, a, b, obs, dtype):
    pi = np.asarray(pi, dtype)
    a = np.asarray(a, dtype)
    b = np.asarray(b, dtype)
    d = (pi + b[:, obs[0]]).astype(dtype)
    for t in range(1, len(obs)):
        d = ((d[:, None] + a).max(axis=0) + b[:, obs[t]]).astype(dtype)
    return d


def exact_units(x):
    """mu (float) -> exact integer in units of 2^-64 (None for -inf)."""
    x = float(x)
    if x == -np.inf:
        return None
    return int(np.rint(x * 2.0 ** 64))


def max_marginal(pi, a, b, obs, tk, dtype):
    a_ = np.asarray(a, dtype)
    d = forward_last_row(pi, a, b, obs[:tk + 1], dtype)
    T = len(obs)
    if tk == T - 1:
        beta = np.zeros(a_.shape[0], dtype)
    else:
        g = forward_last_row(np.zeros(a_.shape[0]), np.asarray(a).T, b, obs[tk + 1:][::-1], dtype)
        beta = (g[None, :] + a_).max(axis=1).astype(dtype)  # beta[i] = max_j g[j] + a[i,j]
    return (d + beta).astype(dtype)


def suffix_beta(a, b, obs_after, dtype):
    """beta[i] = best continuation score after a position in state i over the elements
    obs_after (0 when empty): g from the reversed pass on a^T, then max_j(g[j] + a[i,j])."""
    a_ = np.asarray(a, dtype)
    if len(obs_after) == 0:
        return np.zeros(a_.shape[0], dtype)
    g = forward_last_row(np.zeros(a_.shape[0]), np.asarray(a).T, b, obs_after[::-1], dtype)
    return (g[None, :] + a_).max(axis=1).astype(dtype)


def segment_table(a, b, obs_seg, dtype):
    """M[s, s'] = best score from state s at obs_seg[0] (score 0, no emission there) to
    state s' at obs_seg[-1], row-A0 recurrence in dtype (the kernel's `start` mode)."""
    a = np.asarray(a, dtype)
    b = np.asarray(b, dtype)
    n = a.shape[0]
    D = np.full((n, n), -np.inf, dtype)
    np.fill_diagonal(D, 0)
    for t in range(1, len(obs_seg)):
        D = ((D[:, :, None] + a[None, :, :]).max(axis=1) + b[None, :, obs_seg[t]]).astype(dtype)
    return D


def _acc(vec, vals):
    """vec (list of int|None) += exact units of vals; None (-inf) is sticky."""
    for s, x in enumerate(vals):
        u = exact_units(x)
        vec[s] = None if (u is None or vec[s] is None) else vec[s] + u


def constrained_terms(pi, a, b, offsets, obs, component, dtype=np.float32, mm=None):
    """Exact unary U[c][s] and pairwise P[(c1,c2)][s1][s2] terms (c1 < c2) of the
    constrained objective (csp.hpp): per sequence with constrained positions t_1 < .. < t_m,
      m == 1: U[c_1] += mu = dtype(delta_{t_1} + beta)
      m >= 2: U[c_1] += alpha = delta_{t_1}; U[c_m] += beta; per segment k: M_k into
              P[(c_k, c_k+1)] (oriented by component id) or its diagonal into U[c_k] when
              c_k == c_k+1.
    mm (optional) replaces max_marginal (e.g. a C-accelerated one)."""
    offsets = np.asarray(offsets, np.int64)
    obs = np.asarray(obs, np.int64)
    component = np.asarray(component, np.int64)
    n = np.asarray(a).shape[0]
    mm = mm or max_marginal
    U, P = {}, {}
    for k in range(len(offsets) - 1):
        lo, hi = int(offsets[k]), int(offsets[k + 1])
        pos = [int(t) for t in np.nonzero(component[lo:hi] >= 0)[0]]
        if not pos:
            continue
        o = obs[lo:hi]
        cs = [int(component[lo + t]) for t in pos]
        for c in cs:
            U.setdefault(c, [0] * n)
        if len(pos) == 1:
            _acc(U[cs[0]], mm(pi, a, b, o, pos[0], dtype))
            continue
        _acc(U[cs[0]], forward_last_row(pi, a, b, o[:pos[0] + 1], dtype))
        _acc(U[cs[-1]], suffix_beta(a, b, o[pos[-1] + 1:], dtype))
        for j in range(len(pos) - 1):
            M = segment_table(a, b, o[pos[j]:pos[j + 1] + 1], dtype)
            c1, c2 = cs[j], cs[j + 1]
            if c1 == c2:
                _acc(U[c1], np.diag(M))
                continue
            if c1 > c2:
                c1, c2, M = c2, c1, M.T
            tab = P.setdefault((c1, c2), [[0] * n for _ in range(n)])
            for s1 in range(n):
                _acc(tab[s1], M[s1])
    return U, P


def constrained_solve(U, P, n, limit=200000):
    """Exact maximisation of sum U + sum P, brute force per connected group of components
    (ascending ids); ties -> lexicographically smallest state vector; -1 for a group with
    no feasible assignment.  Returns {component: state}."""
    parent = {c: c for c in U}

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x

    for c1, c2 in P:
        parent[find(c1)] = find(c2)
    groups = {}
    for c in sorted(U):
        groups.setdefault(find(c), []).append(c)
    out = {}
    for comps in groups.values():
        assert n ** len(comps) <= limit, "oracle brute force is for small cases"
        pairs = [(i, j, P[(ci, cj)]) for i, ci in enumerate(comps) for j, cj in enumerate(comps)
                 if (ci, cj) in P]
        best, best_v = None, None
        for st in itertools.product(range(n), repeat=len(comps)):  # lexicographic order
            v = 0
            for i, c in enumerate(comps):
                x = U[c][st[i]]
                if x is None:
                    v = None
                    break
                v += x
            if v is None:
                continue
            for i, j, tab in pairs:
                x = tab[st[i]][st[j]]
                if x is None:
                    v = None
                    break
                v += x
            if v is not None and (best_v is None or v > best_v):
                best, best_v = st, v
        for i, c in enumerate(comps):
            out[c] = -1 if best is None else best[i]
    return out


def constrained_decode(pi, a, b, offsets, obs, component, dtype=np.float32, mm=None):
    """The constrained-decode spec: exact terms, exact search.  Returns (comp_state dict,
    forced[sum T]) -- forced uses 0 for a component without a feasible state (its
    sequences are then reported infeasible)."""
    U, P = constrained_terms(pi, a, b, offsets, obs, component, dtype, mm)
    comp_state = constrained_solve(U, P, np.asarray(a).shape[0])
    component = np.asarray(component, np.int64)
    forced = np.full(len(component), -1, np.int32)
    for e in np.nonzero(component >= 0)[0]:
        forced[e] = max(comp_state[int(component[e])], 0)
    return comp_state, forced


def constrained_brute(pi, a, b, offsets, obs, component, dtype=np.float64):
    """Exhaustive over component-state assignments: returns (assignment, objective)
    maximising the sum of per-sequence forced-decode scores (dtype decode, f64 sum)."""
    comps = sorted(set(int(c) for c in component if c >= 0))
    n = np.asarray(a).shape[0]
    best, best_obj = None, -np.inf
    for assign in itertools.product(range(n), repeat=len(comps)):
        st = dict(zip(comps, assign))
        total = 0.0
        for k in range(len(offsets) - 1):
            lo, hi = offsets[k], offsets[k + 1]
            f = np.array([st[int(c)] if c >= 0 else -1 for c in component[lo:hi]], np.int32)
            _, sc, status = decode_forced(pi, a, b, obs[lo:hi], f, dtype)
            total += float(sc) if status == SEQ_OK else -np.inf
        if total > best_obj:
            best, best_obj = st, total
    return best, best_obj


def decode_forced(pi, a, b, obs, forced, dtype=np.float64):
    """Row-A0 decode with forced states (-1 = free)."""
    pi = np.asarray(pi, dtype)
    a = np.asarray(a, dtype)
    b = np.asarray(b, dtype)
    n, T = a.shape[0], len(obs)
    if T == 0:
        return np.zeros(0, np.int32), dtype(0), SEQ_EMPTY
    ninf = dtype(-np.inf)
    prev = (pi + b[:, obs[0]]).astype(dtype)
    if forced[0] >= 0:
        prev = np.where(np.arange(n) == forced[0], prev, ninf)
    bt = np.zeros((T, n), np.int32)
    cols = np.arange(n)
    for t in range(1, T):
        s = prev[:, None] + a
        arg = np.argmax(s, axis=0)
        cur = (s[arg, cols] + b[:, obs[t]]).astype(dtype)
        if forced[t] >= 0:
            cur = np.where(cols == forced[t], cur, ninf)
        bt[t] = arg
        prev = cur
    end = int(np.argmax(prev))
    if not prev[end] > ninf:
        return np.zeros(T, np.int32), ninf, SEQ_INFEASIBLE
    path = np.zeros(T, np.int32)
    cs = end
    for t in range(T - 1, -1, -1):
        path[t] = cs
        cs = bt[t, cs]
    return path, prev[end], SEQ_OK
