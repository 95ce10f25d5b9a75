"""Command line mirror of the reference's `main` (src/main.rs:25-136) on the GPU solver.

    python -m cviterbi.cli -i INPUT -o OUTPUT -n NSTATES -b NOBS [NOBS ...] -p PROP [--kind gpu]

Reads INPUT/sequences, INPUT/tags, INPUT/test_tags and INPUT/hmm.json (main.rs:71-102),
builds the super-sequence with the test tags as consistency constraints
(Constraints::from_tags, main.rs:87; SuperSequence::from + recompute_constraints(prop),
main.rs:106-115), solves, and writes OUTPUT/{prop}_0 exactly like main.rs:111-133:
"{objective} {explored_nodes}\\n{elapsed_ms}\\n" then "{seq} {state}" per element.
`-t/--train` (Baum-Welch / MLE fitting, hmm.rs:22-190) is out of scope and rejected.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

from .hmm import HMM
from .solver import Constraints, GpuSolver, SuperSequence, load_sequences, load_tags, write_output


def rust_f64(x: float) -> str:
    """Rust's `{}` formatting of an f64 for the values main.rs prints (prop, objective)."""
    if x == int(x) and abs(x) < 1e16:
        return str(int(x))
    return repr(float(x))


def main(argv=None):
    p = argparse.ArgumentParser(prog="cviterbi", description="Hidden Markov Model with consistency constraints")
    p.add_argument("-i", "--input", required=True)
    p.add_argument("-o", "--output", default=".")
    p.add_argument("-n", "--nstates", type=int, required=True)
    p.add_argument("-b", "--nobs", type=int, nargs="+")
    p.add_argument("-p", "--prop", type=float, required=True)
    p.add_argument("-t", "--train", action="store_true")
    p.add_argument("-s", "--supervised", action="store_true")
    p.add_argument("--kind", default="gpu", help="solver kind (gpu, gpu-f64, gpu-cp, gpu-dp)")
    p.add_argument("--device", type=int, default=0)
    a = p.parse_args(argv)
    if a.train:
        p.error("HMM fitting (-t) is out of scope: provide INPUT/hmm.json")
    print("Loading data")
    seqs = load_sequences(os.path.join(a.input, "sequences"), D=2)
    load_tags(os.path.join(a.input, "tags"))  # main.rs:84 (used only for training)
    control = load_tags(os.path.join(a.input, "test_tags"))
    cons = Constraints.from_tags(control)
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
    print(f"[{solver.get_name()} EXP {rust_f64(a.prop)}] Run 1/1")
    t0 = time.perf_counter()
    solver.solve()
    ms = int((time.perf_counter() - t0) * 1000)
    write_output(out, solver, ss, ms, solver.get_explored_nodes())
    return 0


if __name__ == "__main__":
    sys.exit(main())
