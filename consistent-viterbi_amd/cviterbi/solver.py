"""Solver, SuperSequence, Constraints and the text loaders -- the reference's
viterbi_solver host interface, with the decode itself on MI355X.

Mirrors (file:line into /root/reference/src):
  trait Solver                      viterbi_solver.rs:11-16
  SuperSequence / MetaElements      viterbi_solver/utils.rs:9-211
  Constraints::from_tags/from_file  viterbi_solver/constraints.rs:12-69
  load_sequences / load_tags        utils.rs:7-60
  main's output file                main.rs:111-133
Decoding goes through cv_solver_* (libcviterbi).  Active consistency constraints use
cv_decode_constrained (exact for any number of active constrained elements per
sequence: unary + pairwise component terms and an exact search).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .hmm import HMM
from .stdrng import StdRng


def _p(x):
    return x.ctypes.data_as(ctypes.c_void_p)


# ---- text loaders (src/utils.rs) -----------------------------------------------------
def load_sequences(path, D=2):
    """utils::load_sequences::<D> (utils.rs:7-34): lines "seq_id v0 [v1 ...]"; a new
    sequence starts when seq_id changes; missing components are 0."""
    seqs, cur, last = [], [], None
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            s = [int(x) for x in line.split(" ")]
            if last is not None and s[0] != last:
                seqs.append(cur)
                cur = []
            last = s[0]
            el = [0] * D
            for i, v in enumerate(s[1:]):
                el[i] = v
            cur.append(tuple(el))
    seqs.append(cur)
    return seqs


def load_tags(path):
    """utils::load_tags (utils.rs:36-60): lines "seq_id tag", tag -1 -> None."""
    out, cur, last = [], [], None
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            s = line.split(" ")
            sid = int(s[0])
            if last is not None and sid != last:
                out.append(cur)
                cur = []
            cur.append(None if s[1] == "-1" else int(s[1]))
            last = sid
    out.append(cur)
    return out


# ---- constraints.rs --------------------------------------------------------------------
@dataclass
class Constraints:
    components: list = field(default_factory=list)  # list[set[(seq_id, t)]]

    @classmethod
    def from_tags(cls, truth):
        """constraints.rs:40-69: one component per distinct tag value, in first-seen order."""
        values, comps = [], []
        for sid, tags in enumerate(truth):
            for t, tag in enumerate(tags):
                if tag is None:
                    continue
                if tag in values:
                    comps[values.index(tag)].add((sid, t))
                else:
                    values.append(tag)
                    comps.append({(sid, t)})
        return cls(comps)

    @classmethod
    def from_file(cls, path):
        """constraints.rs:12-38: blank-line separated groups of "seq_id t"; singletons dropped."""
        comps, comp = [], set()
        with open(path) as f:
            for line in f:
                line = line.rstrip("\n")
                if line == "":
                    if len(comp) > 1:
                        comps.append(comp)
                    comp = set()
                else:
                    a, b = line.split()[:2]
                    comp.add((int(a), int(b)))
        if len(comp) > 1:
            comps.append(comp)
        return cls(comps)


# ---- utils.rs: SuperSequence -------------------------------------------------------------
class SuperSequence:
    """All sequences concatenated into one element array (utils.rs:62-103).

    Element fields (MetaElements, utils.rs:9-16): seq, t, value (flat obs index),
    constraint_component (-1 = none), active_cstr, last_of_constraint.
    """

    def __init__(self, sequences, constraints: Constraints | None, hmm: HMM):
        self.hmm = hmm
        self.constraints = constraints or Constraints()
        self.orig_sizes = [len(s) for s in sequences]
        n = sum(self.orig_sizes)
        self.seq = np.zeros(n, np.int64)
        self.t = np.zeros(n, np.int64)
        self.value = np.zeros(n, np.int32)
        self.component = np.full(n, -1, np.int32)
        self.active = np.zeros(n, np.uint8)
        self.last = np.zeros(n, np.uint8)
        lookup = {}
        for cid, comp in enumerate(self.constraints.components):
            for key in comp:
                lookup.setdefault(key, cid)  # first component containing (seq,t) (utils.rs:70-75)
        k = 0
        for sid, s in enumerate(sequences):
            for t, v in enumerate(s):
                self.seq[k], self.t[k], self.value[k] = sid, t, hmm.flat(v)
                c = lookup.get((sid, t), -1)
                self.component[k] = c
                self.active[k] = c != -1
                k += 1
        self.start = np.concatenate([[0], np.cumsum(self.orig_sizes)[:-1]]).astype(np.int64) if sequences else \
            np.zeros(0, np.int64)
        self._mark_last()
        self.rng = StdRng(3019)  # utils.rs:101 StdRng::seed_from_u64(3019)

    def _mark_last(self):
        """utils.rs:104-115 / 168-179: last active element of each component, scanning backwards."""
        self.last[:] = 0
        seen = set()
        self.nb_active_cstr = 0
        for k in range(len(self.seq) - 1, -1, -1):
            if self.active[k]:
                c = int(self.component[k])
                if c not in seen:
                    seen.add(c)
                    self.nb_active_cstr += 1
                    self.last[k] = 1

    def get_sequences_ordering(self):
        """utils.rs:105-136.  Note the reference keeps only the LAST element's constraint
        flag per sequence (`is_constrained` is overwritten in the loop); reproduced."""
        keys = []
        finite = np.isfinite(np.stack([self.hmm.emit_probs(int(v)) for v in self.value])) if len(self.value) else None
        for sid, size in enumerate(self.orig_sizes):
            st = int(self.start[sid])
            is_c = bool(self.active[st + size - 1]) if size else False
            possible = float(finite[st:st + size].sum()) if size else 0.0
            avg = possible / size if size else float("nan")
            keys.append((1 if is_c else 0, avg, sid))
        keys.sort()
        return [k[2] for k in keys]

    def reorder(self):
        """utils.rs:138-165: rebuild the element array in get_sequences_ordering order."""
        order = self.get_sequences_ordering()
        idx = np.concatenate([np.arange(self.start[s], self.start[s] + self.orig_sizes[s]) for s in order]) \
            if order else np.zeros(0, np.int64)
        for name in ("seq", "t", "value", "component", "active"):
            setattr(self, name, getattr(self, name)[idx])
        new_start = np.zeros(len(self.orig_sizes), np.int64)
        pos = 0
        for s in order:
            new_start[s] = pos
            pos += self.orig_sizes[s]
        self.start = new_start
        self._mark_last()

    def recompute_constraints(self, proportion: float):
        """utils.rs:168-177: in element order, an element with a component is active iff
        rng.gen::<f64>() <= proportion (one draw per such element, short-circuit: none for
        free elements), then reorder().  The RNG stream persists across calls, as in
        main.rs:107 + 113-115 (see stdrng.py for the restated StdRng)."""
        has = self.component != -1
        draws = self.rng.gen_f64(int(has.sum()))
        act = np.zeros(len(self.component), np.uint8)
        act[has] = (draws <= proportion).astype(np.uint8)
        self.active = act
        self.reorder()

    def __len__(self):
        return len(self.seq)

    def number_constraints(self):
        return self.nb_active_cstr

    def sequence_blocks(self):
        """(offsets[B+1], obs, seq_ids) of the element array: sequences are contiguous."""
        order = np.argsort(self.start, kind="stable")
        offsets = np.zeros(len(order) + 1, np.int64)
        for i, s in enumerate(order):
            offsets[i + 1] = offsets[i] + self.orig_sizes[s]
        return offsets, self.value, order.astype(np.int64)

    def parse_solution(self, solution):
        """utils.rs:183-190: element-order solution -> per original sequence arrays."""
        out = [np.zeros(s, np.int64) for s in self.orig_sizes]
        for k in range(len(self.seq)):
            out[int(self.seq[k])][int(self.t[k])] = solution[k]
        return out


# ---- viterbi_solver.rs: trait Solver -------------------------------------------------------
class Solver:
    """trait Solver (viterbi_solver.rs:11-16)."""

    def solve(self):
        raise NotImplementedError

    def get_solution(self):
        raise NotImplementedError

    def get_objective(self) -> float:
        raise NotImplementedError

    def get_name(self) -> str:
        raise NotImplementedError


class GpuSolver(Solver):
    """Solver backed by cv_solver_* (kinds: gpu-cp = CPSolver, the default, what main.rs:120
    runs; gpu-cp-seq, gpu-f64, gpu-dp, gpu; include/cviterbi.h)."""

    def __init__(self, hmm: HMM, sequence: SuperSequence, kind: str = "gpu-cp"):
        self.hmm = hmm
        self.sequence = sequence
        offsets, obs, seq_ids = sequence.sequence_blocks()
        self._keep = (offsets, np.ascontiguousarray(obs, np.int32), seq_ids,
                      np.ascontiguousarray(sequence.component, np.int32),
                      np.ascontiguousarray(sequence.active, np.uint8))
        o, ob, si, comp, act = self._keep
        desc = L.SuperSeqDesc(len(offsets) - 1, o.ctypes.data, ob.ctypes.data, si.ctypes.data, comp.ctypes.data,
                              act.ctypes.data)
        s = ctypes.c_void_p()
        L.check(L.lib().cv_solver_create(kind.encode(), hmm.handle, ctypes.byref(desc), ctypes.byref(s)))
        self._s = s

    def __del__(self):
        s = getattr(self, "_s", None)
        if s:
            L.lib().cv_solver_destroy(s)
            self._s = None

    def solve(self):
        L.check(L.lib().cv_solver_solve(self._s))

    def get_solution(self):
        ptr = ctypes.POINTER(ctypes.c_int32)()
        n = ctypes.c_int64()
        L.check(L.lib().cv_solver_get_solution(self._s, ctypes.byref(ptr), ctypes.byref(n)))
        return np.ctypeslib.as_array(ptr, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int32)

    def get_objective(self) -> float:
        v = ctypes.c_double()
        L.check(L.lib().cv_solver_get_objective(self._s, ctypes.byref(v)))
        return v.value

    def get_name(self) -> str:
        return L.lib().cv_solver_get_name(self._s).decode()

    def write_cfn(self, path) -> int:
        """write_cfn (cfn.rs:82-205) of this solver's super-sequence to `path`; returns the
        table compilation time in ms (what main.rs:117 records)."""
        ms = ctypes.c_uint64()
        L.check(L.lib().cv_solver_write_cfn(self._s, str(path).encode(), ctypes.byref(ms)))
        return ms.value

    def get_explored_nodes(self) -> int:
        v = ctypes.c_uint64()
        L.check(L.lib().cv_solver_get_explored_nodes(self._s, ctypes.byref(v)))
        return v.value


def write_output(path, solver: Solver, sequence: SuperSequence, elapsed_ms: int, explored_nodes: int = 0):
    """main.rs:129-133: "objective explored\\nms\\n" then "seq state" per element."""
    from .cli import rust_f64

    sol = solver.get_solution()
    with open(path, "w") as f:
        f.write(f"{rust_f64(solver.get_objective())} {explored_nodes}\n{elapsed_ms}\n")
        for k in range(len(sol)):
            f.write(f"{int(sequence.seq[k])} {int(sol[k])}\n")
