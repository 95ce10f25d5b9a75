"""Command line mirror of the reference's `main` (src/main.rs:25-136) on the GPU solver.

    python -m cviterbi.cli -i INPUT -o OUTPUT -n NSTATES -b NOBS [NOBS ...] -p PROP
                           [-t [-s]] [--cfn] [--kind gpu-cp] [--seed S]

Reads INPUT/sequences, INPUT/tags, INPUT/test_tags (main.rs:80-87) and either INPUT/hmm.json
(main.rs:100-103) or, with -t, fits the HMM on the GPU from a random start (HMM::new,
hmm.rs:22-28, seeded here with --seed where the reference uses thread_rng): -s = supervised
MLE (hmm.rs:30-62), otherwise tag-clamped Baum-Welch with max_iter 1000, tol 0.001
(main.rs:92-96); the fitted model is written to INPUT/hmm.json (main.rs:97).  Builds the
super-sequence with the test tags as consistency constraints (Constraints::from_tags,
main.rs:87; SuperSequence::from + recompute_constraints(prop), main.rs:106-115) and writes
OUTPUT/{prop}_0 like main.rs:111-133: "{objective} {explored_nodes}\\n{elapsed_ms}\\n" then
"{seq} {state}" per element.  --cfn takes the reference's run_cfn branch (main.rs:116-118):
OUTPUT/problem_{prop}_0.cfn (cfn.rs:82-205) and the compile time in OUTPUT/{prop}_0.
The solver defaults to what main.rs:120 runs, CPSolver: kind "gpu-cp" -- without active
constraints the exact chained super-sequence decode in f64 (cv_decode_superseq_cp: the same
path and objective bits as cp.rs), with them the consistency-constrained decode in f64.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from decimal import Decimal

import numpy as np

from .fit import fit_mle, fit_train
from .hmm import HMM
from .solver import Constraints, GpuSolver, SuperSequence, load_sequences, load_tags, write_output


def rust_f64(x: float) -> str:
    """Rust's `{}` (Display) of an f64: the shortest decimal that reads back to the same
    double, positional (never an exponent); "inf", "-inf", "NaN"."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "inf" if x > 0 else "-inf"
    s = format(Decimal(repr(x)), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


def _random_start(n, bdims, rng):
    """HMM::new (hmm.rs:22-28): uniform [0,1) draws, rows of A / each state's emission array
    / pi normalised to sum 1 (hmm.rs:274-317)."""
    a = rng.random((n, n))
    a /= a.sum(axis=1, keepdims=True)
    b = rng.random((n, int(np.prod(bdims))))
    b /= b.sum(axis=1, keepdims=True)
    pi = rng.random(n)
    pi /= pi.sum()
    return pi, a, b


def _flatten(seqs, tags, bdims):
    """Sequences of [usize; 2] and tags (None = unknown) -> CSR offsets, flat obs, tags (-1)."""
    lens = np.array([len(s) for s in seqs], np.int64)
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    el = np.array([v for s in seqs for v in s], np.int64).reshape(-1, len(bdims))
    obs = np.zeros(len(el), np.int64)
    for d, n in enumerate(bdims):
        obs = obs * int(n) + el[:, d]
    tg = np.array([-1 if t is None else t for ts in tags for t in ts], np.int32)
    if len(tg) != len(obs):
        raise SystemExit(f"tags hold {len(tg)} elements, sequences {len(obs)}")
    return off, obs.astype(np.int32), tg


def main(argv=None):
    p = argparse.ArgumentParser(prog="cviterbi", description="Hidden Markov Model with consistency constraints")
    p.add_argument("-i", "--input", required=True)
    p.add_argument("-o", "--output", default=".")
    p.add_argument("-n", "--nstates", type=int, required=True)
    p.add_argument("-b", "--nobs", type=int, nargs="+")
    p.add_argument("-p", "--prop", type=float, required=True)
    p.add_argument("-t", "--train", action="store_true", help="learn the HMM from the data")
    p.add_argument("-s", "--supervised", action="store_true", help="with -t: supervised MLE")
    p.add_argument("--cfn", action="store_true", help="write the CFN instead of solving (main.rs run_cfn)")
    p.add_argument("--seed", type=int, default=None, help="random start of -t (reference: thread_rng)")
    p.add_argument("--kind", default="gpu-cp",
                   help="solver kind: gpu-cp (default: CPSolver, main.rs:120, f64), gpu-cp-seq, gpu-f64, gpu-dp, "
                        "gpu (f32 trellis)")
    p.add_argument("--device", type=int, default=0)
    a = p.parse_args(argv)
    print("Loading data")
    seqs = load_sequences(os.path.join(a.input, "sequences"), D=2)
    tags = load_tags(os.path.join(a.input, "tags"))
    control = load_tags(os.path.join(a.input, "test_tags"))
    cons = Constraints.from_tags(control)
    if a.train:
        if not a.nobs or len(a.nobs) < 2:
            p.error("-t needs -b NOBS0 NOBS1 (main.rs:91)")
        bdims = (a.nobs[0], a.nobs[1])
        pi0, a0, b0 = _random_start(a.nstates, bdims, np.random.default_rng(a.seed))
        off, obs, tg = _flatten(seqs, tags, bdims)
        if a.supervised:
            lp, la, lb = fit_mle(pi0, a0, b0, off, obs, tg, device=a.device)
        else:
            lp, la, lb, _ = fit_train(pi0, a0, b0, off, obs, tg, max_iter=1000, tol=0.001, device=a.device)
        hmm = HMM(lp, la, lb, bdims=bdims, device=a.device)
        hmm.write(os.path.join(a.input, "hmm.json"))
    else:
        hmm = HMM.from_json(os.path.join(a.input, "hmm.json"), device=a.device)
    if hmm.nstates() != a.nstates:
        p.error(f"hmm.json has {hmm.nstates()} states, -n says {a.nstates}")
    ss = SuperSequence(seqs, cons, hmm)
    ss.recompute_constraints(a.prop)
    os.makedirs(a.output, exist_ok=True)
    out = os.path.join(a.output, f"{rust_f64(a.prop)}_0")
    if a.prop not in (0.0, 1.0):
        ss.recompute_constraints(a.prop)  # main.rs:113-115
    solver = GpuSolver(hmm, ss, a.kind)
    if a.cfn:  # main.rs:116-118
        ms = solver.write_cfn(os.path.join(a.output, f"problem_{rust_f64(a.prop)}_0.cfn"))
        with open(out, "w") as f:
            f.write(f"{ms}\n")
        return 0
    print(f"[{solver.get_name()} EXP {rust_f64(a.prop)}] Run 1/1")
    t0 = time.perf_counter()
    solver.solve()
    ms = int((time.perf_counter() - t0) * 1000)
    write_output(out, solver, ss, ms, solver.get_explored_nodes())
    return 0


if __name__ == "__main__":
    sys.exit(main())
