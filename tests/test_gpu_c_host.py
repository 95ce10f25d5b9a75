"""A compiled C host program (examples/solver_main.c) drives the Solver ABI the way the Rust
binding of INTEGRATION.md would (HMM::from_json -> CPSolver::new as "gpu-cp" -> solve ->
get_objective / get_solution / get_explored_nodes, main.rs:120-133).  Its output must equal
the CP super-sequence restatement (oracle cvo_cp_superseq_f64, cp.rs:63-93 over
utils.rs:62-103) without constraints, the ctypes GpuSolver on the same super-sequence with
active constraints, and every element of a constrained component must share one state."""
import os
import subprocess

import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "solver_main")


def _write_input(path, off, obs, comp, active):
    with open(path, "w") as f:
        f.write(f"{len(off) - 1}\n")
        for arr in (off, obs, comp, active):
            f.write(" ".join(str(int(x)) for x in arr) + "\n")


def _run(hmm_json, inp, kind="gpu-cp"):
    out = subprocess.run([EXE, str(hmm_json), str(inp), kind], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    obj = float(lines[0].split()[1])
    explored = int(lines[1].split()[1])
    name = lines[2].split(maxsplit=1)[1]
    sol = np.array([int(l.split()[1]) for l in lines[3:]], np.int32)
    return obj, explored, name, sol


def _case(seed):
    pi, a, b = synth.random_hmm(12, 20, seed=seed)
    rng = np.random.default_rng(seed)
    off = synth.offsets_from_lengths(rng.integers(3, 30, size=40))
    obs = rng.integers(0, 20, size=int(off[-1])).astype(np.int32)
    return pi, a, b, off, obs


def test_c_host_unconstrained_matches_cp_superseq(gpu, tmp_path):
    assert os.path.exists(EXE), "examples/solver_main not built (__graft_entry__.build())"
    pi, a, b, off, obs = _case(5)
    cv.HMM(pi, a, b).write(tmp_path / "hmm.json")
    ne = int(off[-1])
    _write_input(tmp_path / "in.txt", off, obs, np.full(ne, -1), np.zeros(ne))
    obj, explored, name, sol = _run(tmp_path / "hmm.json", tmp_path / "in.txt")
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert np.array_equal(sol, rp)
    assert obj == robj
    assert name and explored >= 0


def test_c_host_constrained_matches_ctypes_solver(gpu, tmp_path):
    pi, a, b, off, obs = _case(6)
    cv.HMM(pi, a, b).write(tmp_path / "hmm.json")
    ne = int(off[-1])
    rng = np.random.default_rng(7)
    comp = np.full(ne, -1, np.int32)
    pos = rng.choice(ne, size=12, replace=False)
    comp[pos] = rng.integers(0, 3, size=12)
    active = (comp >= 0).astype(np.uint8)
    _write_input(tmp_path / "in.txt", off, obs, comp, active)
    obj, explored, name, sol = _run(tmp_path / "hmm.json", tmp_path / "in.txt")
    # the same super-sequence through the shipped ctypes binding
    import ctypes

    from cviterbi import _lib as L

    h = cv.HMM.from_json(tmp_path / "hmm.json")
    o64, ob32 = np.ascontiguousarray(off, np.int64), np.ascontiguousarray(obs, np.int32)
    desc = L.SuperSeqDesc(len(off) - 1, o64.ctypes.data, ob32.ctypes.data, None, comp.ctypes.data, active.ctypes.data)
    s = ctypes.c_void_p()
    L.check(L.lib().cv_solver_create(b"gpu-cp", h.handle, ctypes.byref(desc), ctypes.byref(s)))
    try:
        L.check(L.lib().cv_solver_solve(s))
        ptr = ctypes.POINTER(ctypes.c_int32)()
        n = ctypes.c_int64()
        L.check(L.lib().cv_solver_get_solution(s, ctypes.byref(ptr), ctypes.byref(n)))
        ref = np.ctypeslib.as_array(ptr, shape=(n.value,)).copy()
        v = ctypes.c_double()
        L.check(L.lib().cv_solver_get_objective(s, ctypes.byref(v)))
    finally:
        L.lib().cv_solver_destroy(s)
    assert np.array_equal(sol, ref) and obj == v.value
    for c in range(3):  # every active element of a component decodes to one state
        st = set(sol[(comp == c) & (active == 1)].tolist())
        assert len(st) <= 1, (c, st)
