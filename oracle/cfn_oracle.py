"""Pure-Python restatement of the reference's CFN export (viterbi_solver/cfn.rs:11-205).

TEST INFRASTRUCTURE ONLY: the checker for cv_solver_write_cfn, imported by tests/ only.
Parity unpinned against the Rust binary (it cannot be built here; main.rs:108 leaves the
CFN branch disabled and the reference ships no CFN fixture); pinned by the structure and
float-format cases in tests/test_cfn.py.  Small problems only (plain Python loops).

The super-sequence is given element-wise: value[e] (flat observation index), comp[e] (the
active constraint component, -1 = none: MetaElements::is_constrained), first[e] (t == 0:
MetaElements::transitions returns the constant pi vector, utils.rs:32-38).  pi[N], a[N][N],
b[N][V] are log10 (the HMM as decoded).  All arithmetic is Python float (IEEE f64), in the
reference's order: (row + transitions) elementwise, max, then + emission.
"""
from __future__ import annotations

import math
from decimal import Decimal

NEG = -math.inf


def rust_display(x: float) -> str:
    """Rust `format!("{}", f64)`: shortest round-trip digits, positional, inf / -inf / NaN."""
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    s = format(Decimal(repr(float(x))), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


def _trans(pi, a, first, i, n):
    return pi[n] if first else a[i][n]


def _step(pi, a, b, row, value, first, states):
    """One element: for each n in `states`, max_i(row[i] + trans_i(n)) + b[n][value]."""
    N = len(pi)
    out = [NEG] * N
    for n in states:
        m = NEG
        for i in range(N):
            x = row[i] + _trans(pi, a, first, i, n)
            if x > m:
                m = x
        out[n] = m + b[n][value]
    return out


def longest_path(pi, a, b, value, comp, first, t_from, n_from, t_to, n_to):
    """cfn.rs:11-34."""
    N = len(pi)
    row = [NEG] * N
    row[n_from] = 0.0
    for t in range(t_from + 1, t_to + 1):
        if comp[t] >= 0:
            n = n_from if t < t_to else n_to
            row = _step(pi, a, b, row, value[t], first[t], [n])
        else:
            row = _step(pi, a, b, row, value[t], first[t], range(N))
    return max(row)


def unary_start(pi, a, b, value, comp, first, t_limit):
    """cfn.rs:36-53 (init_probs = pi + b[:, value[0]], hmm.rs:215-218)."""
    N = len(pi)
    row = [pi[n] + b[n][value[0]] for n in range(N)]
    for t in range(1, t_limit + 1):
        row = _step(pi, a, b, row, value[t], first[t], range(N))
    return row


def unary_end(pi, a, b, value, comp, first, t_start):
    """cfn.rs:55-80."""
    N = len(pi)
    L = len(value)
    if t_start == L - 1:
        return [0.0] * N
    out = []
    for n in range(N):
        row = [NEG] * N
        row[n] = 0.0
        for t in range(t_start + 1, L):
            if comp[t] >= 0:
                row = _step(pi, a, b, row, value[t], first[t], [n])
            else:
                row = _step(pi, a, b, row, value[t], first[t], range(N))
        out.append(max(row))
    return out


def write_cfn_text(pi, a, b, value, comp, first) -> str:
    """cfn.rs:82-205: the text of the .cfn file."""
    N = len(pi)
    L = len(value)
    bnd = []
    last = None
    for t in range(L):
        if comp[t] >= 0:
            c = comp[t]
            if last is None or c != last:
                bnd.append((t, c))
            last = c
    k = len({c for c in comp if c >= 0})  # number_constraints (utils.rs:200-202)
    tables = [[[[0.0] * N for _ in range(N)] for _ in range(k)] for _ in range(k)]
    for i in range(len(bnd) - 1):
        tf, cf = bnd[i]
        tt, ct = bnd[i + 1]
        for n1 in range(N):
            for n2 in range(N):
                cost = longest_path(pi, a, b, value, comp, first, tf, n1, tt, n2)
                if cost != NEG:
                    x = tables[cf][ct][n1][n2]
                    tables[cf][ct][n1][n2] = cost if x == 0.0 else x + cost
                    y = tables[ct][cf][n2][n1]
                    tables[ct][cf][n2][n1] = cost if y == 0.0 else y + cost
    unary = [[0.0] * N for _ in range(k)]
    f_time, f_cid = bnd[0]
    l_time, l_cid = bnd[-1]
    start = unary_start(pi, a, b, value, comp, first, f_time)
    unary[f_cid] = [u + s for u, s in zip(unary[f_cid], start)]
    end = unary_end(pi, a, b, value, comp, first, l_time)
    unary[l_cid] = [u + e for u, e in zip(unary[l_cid], end)]
    lb = -1.0
    for k1 in range(k):
        for k2 in range(k1 + 1, k):
            lb += min(min(r) for r in tables[k1][k2])
    for kk in range(k):
        unary[kk] = [lb if u == NEG else u for u in unary[kk]]

    def vec(v):
        return "[" + "".join(f"{rust_display(x)}{']' if q == len(v) - 1 else ','} " for q, x in enumerate(v))

    out = "{\n\tproblem: { name: consistent_viterbi, mustbe: >" + rust_display(lb) + "},\n"
    out += "\tvariables: {"
    dom = "[" + ",".join(f"s{i}" for i in range(N)) + "]"
    for i in range(k):
        out += f"n{i}: {dom}{',' if i != k - 1 else '},' + chr(10)}"
    out += "\tfunctions: {\n"
    for i in range(k):
        out += f"\t\tf{i}: {{ scope: [n{i}], costs: " + vec(unary[i]) + "}, \n"
        for j in range(i + 1, k):
            flat = [x for r in tables[i][j] for x in r]
            if sum(flat) != 0.0:
                out += f"\t\tf{i}_{j}: {{ scope: [n{i}, n{j}], costs: " + vec(flat) + "},\n"
    out += "\t}\n}"
    return out
