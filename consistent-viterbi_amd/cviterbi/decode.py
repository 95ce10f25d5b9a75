"""Batch Viterbi decode on MI355X (cv_decode_batch / cv_decode_batch_device).

Replaces, per sequence, the dense forward + backtrack of the reference's solvers:
CPSolver::init_viterbi + backtrack (viterbi_solver/cp.rs:63-93), viterbi::decode
(viterbi.rs:5-32) and DPSolver::solve (dp.rs:94-209); see include/cviterbi.h.

dtype defaults to "f64": the reference's own arithmetic (hmm.rs:10-18 stores f64), paths
and scores bit-identical to the f64 recurrence.  dtype="f32" selects the f32 trellis (about
twice as fast; paths differ from the f64 ones on a few % of long sequences, scores are the
f64 re-score of the f32 path when rescore_f64 is set).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .hmm import HMM

_DT = {"f32": L.DTYPE_F32, "f64": L.DTYPE_F64, np.float32: L.DTYPE_F32, np.float64: L.DTYPE_F64}
_ASSOC = {"viterbi": L.ASSOC_VITERBI, "cp": L.ASSOC_CP, "dp": L.ASSOC_DP, "decode": L.ASSOC_DECODE}
_KERNEL = {"auto": L.KERNEL_AUTO, "trellis": L.KERNEL_TRELLIS, "generic": L.KERNEL_GENERIC,
           "trellis_f64": L.KERNEL_TRELLIS_F64}


def _p(x):
    return x.ctypes.data_as(ctypes.c_void_p)


def make_opts(dtype="f64", assoc="viterbi", kernel="auto", rescore_f64=True, stream=None, workspace_bytes=0,
              variant=None, serial=False):
    """variant: None/"valu" (f32 trellis: two equal-length sequences per workgroup where
    N % 64 == 0, default; for N <= 64 one wave per sequence with the backtrack fused),
    "nowave" (the workgroup kernels at N <= 64) or "valu1" (one sequence per workgroup) --
    all bit-identical; serial: no forward/backtrack stream overlap."""
    flags = L.FLAG_SERIAL if serial else 0
    if variant == "valu1":
        flags |= L.FLAG_NO_PAIR | L.FLAG_NO_WAVE
    elif variant == "nowave":
        flags |= L.FLAG_NO_WAVE
    elif variant not in (None, "valu"):
        raise ValueError(f"unknown variant {variant!r}")
    return L.opts(_DT.get(dtype, dtype), _ASSOC.get(assoc, assoc), _KERNEL.get(kernel, kernel), rescore_f64, stream,
                  workspace_bytes, flags)


def decode_batch(hmm: HMM, offsets, obs, dtype="f64", assoc="viterbi", kernel="auto", rescore_f64=True,
                 workspace_bytes=0, variant=None, serial=False, forced=None):
    """Decode CSR sequences (offsets[B+1], flat obs) -> (path int32[sum T], score f64[B], status u8[B]).
    forced[sum T] (optional): -1 free, s >= 0 forces state s at that element."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    nseq = offsets.shape[0] - 1
    total = int(offsets[-1]) if nseq >= 0 else 0
    path = np.zeros(max(total, 0), np.int32)
    score = np.zeros(max(nseq, 0), np.float64)
    status = np.zeros(max(nseq, 0), np.uint8)
    o = make_opts(dtype, assoc, kernel, rescore_f64, None, workspace_bytes, variant, serial)
    if forced is not None:
        forced = np.ascontiguousarray(forced, np.int32)
        o.forced = forced.ctypes.data
    L.check(L.lib().cv_decode_batch(hmm.handle, nseq, _p(offsets), _p(obs), ctypes.byref(o), _p(path), _p(score),
                                    _p(status)))
    return path, score, status


def decode_constrained(hmm: HMM, offsets, obs, component, ncomp=None, rescore_f64=True, dtype="f64"):
    """Consistency-constrained decode (cv_decode_constrained): component[sum T] (-1 = free).
    dtype "f64" (default, the reference's precision: cp.rs:95-126 / dp.rs:147-166 in f64) or
    "f32".  Returns (path, score, status, comp_state[ncomp], objective)."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    component = np.ascontiguousarray(component, np.int32)
    if ncomp is None:
        ncomp = int(component.max()) + 1 if component.size else 0
    nseq = offsets.shape[0] - 1
    path = np.zeros(int(offsets[-1]), np.int32)
    score = np.zeros(nseq, np.float64)
    status = np.zeros(nseq, np.uint8)
    states = np.full(max(ncomp, 1), -1, np.int32)
    obj = ctypes.c_double()
    o = make_opts(dtype, "viterbi", "auto", rescore_f64)
    L.check(L.lib().cv_decode_constrained(hmm.handle, nseq, _p(offsets), _p(obs), _p(component), int(ncomp),
                                          ctypes.byref(o), _p(path), _p(score), _p(status), _p(states),
                                          ctypes.byref(obj)))
    return path, score, status, states[:ncomp], obj.value


def partial_words(nstates: int, ncomp: int, npairs: int) -> int:
    """CV_PARTIAL_WORDS: int64 words of the constrained partials."""
    return int(ncomp) * (5 * int(nstates) + 1) + int(npairs) * (5 * int(nstates) ** 2 + 1)


def constrained_pairs(offsets, component, ncomp):
    """cv_constrained_pairs (host only): int32[npairs, 2] sorted component pairs (c1 < c2)
    that are consecutive constrained elements of a sequence -- compute on the FULL batch."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    component = np.ascontiguousarray(component, np.int32)
    n = ctypes.c_int64()
    nseq = offsets.shape[0] - 1
    L.check(L.lib().cv_constrained_pairs(nseq, _p(offsets), _p(component), int(ncomp), None, 0, ctypes.byref(n)))
    pairs = np.zeros((max(n.value, 1), 2), np.int32)
    L.check(L.lib().cv_constrained_pairs(nseq, _p(offsets), _p(component), int(ncomp), _p(pairs), n.value,
                                         ctypes.byref(n)))
    return pairs[:n.value]


def constrained_partials(hmm: HMM, offsets, obs, component, ncomp, pairs=None, dtype="f64"):
    """cv_constrained_partials: this shard's exact unary + pairwise terms as int64 words
    (partial_words long); partials of disjoint shards add (one all-reduce SUM).  `pairs`
    must come from constrained_pairs on the full batch (default: this batch's own)."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    component = np.ascontiguousarray(component, np.int32)
    if pairs is None:
        pairs = constrained_pairs(offsets, component, ncomp)
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    part = np.zeros(max(partial_words(hmm.nstates(), ncomp, len(pairs)), 1), np.int64)
    o = make_opts(dtype, "viterbi", "auto", True)
    L.check(L.lib().cv_constrained_partials(hmm.handle, offsets.shape[0] - 1, _p(offsets), _p(obs), _p(component),
                                            int(ncomp), len(pairs), _p(pairs) if len(pairs) else None,
                                            ctypes.byref(o), _p(part)))
    return part[:partial_words(hmm.nstates(), ncomp, len(pairs))]


def constrained_select(nstates: int, ncomp: int, partials, pairs=None):
    """cv_constrained_select (host only): (comp_state[ncomp], explored) from reduced partials."""
    partials = np.ascontiguousarray(partials, np.int64)
    pairs = np.zeros((0, 2), np.int32) if pairs is None else np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    if partials.size != partial_words(nstates, ncomp, len(pairs)):
        raise ValueError("partials size does not match (nstates, ncomp, pairs)")
    states = np.full(max(ncomp, 1), -1, np.int32)
    ex = ctypes.c_uint64()
    L.check(L.lib().cv_constrained_select(int(nstates), int(ncomp), len(pairs), _p(pairs) if len(pairs) else None,
                                          _p(partials), _p(states), ctypes.byref(ex)))
    return states[:ncomp], ex.value


def decode_forced_components(hmm: HMM, offsets, obs, component, comp_state, rescore_f64=True, dtype="f64"):
    """cv_decode_forced_components: final decode of a shard given the component states.
    Returns (path, score, status, objective)."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    component = np.ascontiguousarray(component, np.int32)
    cs = np.ascontiguousarray(comp_state, np.int32)
    nseq = offsets.shape[0] - 1
    path = np.zeros(int(offsets[-1]), np.int32)
    score = np.zeros(nseq, np.float64)
    status = np.zeros(nseq, np.uint8)
    obj = ctypes.c_double()
    o = make_opts(dtype, "viterbi", "auto", rescore_f64)
    L.check(L.lib().cv_decode_forced_components(hmm.handle, nseq, _p(offsets), _p(obs), _p(component), len(cs),
                                                _p(cs) if len(cs) else None, ctypes.byref(o), _p(path), _p(score),
                                                _p(status), ctypes.byref(obj)))
    return path, score, status, obj.value


def decode_batch_device(hmm: HMM, offsets_dev, obs_dev, path_dev, score_dev, status_dev, offsets_host=None,
                        dtype="f64", assoc="viterbi", kernel="auto", rescore_f64=True, stream=None,
                        workspace_bytes=0, variant=None, serial=False):
    """Device-pointer decode (ints or objects with data_ptr(), e.g. torch tensors); async on `stream`."""
    def ptr(x):
        if x is None:
            return None
        return x.data_ptr() if hasattr(x, "data_ptr") else int(x)

    nseq = (len(offsets_host) if offsets_host is not None else offsets_dev.numel()) - 1
    oh = None
    if offsets_host is not None:
        oh = np.ascontiguousarray(offsets_host, np.int64)
    o = make_opts(dtype, assoc, kernel, rescore_f64, stream, workspace_bytes, variant, serial)
    L.check(L.lib().cv_decode_batch_device(hmm.handle, nseq, _p(oh) if oh is not None else None, ptr(offsets_dev),
                                           ptr(obs_dev), ctypes.byref(o), ptr(path_dev), ptr(score_dev),
                                           ptr(status_dev)))


EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.c_void_p)


def decode_constrained_exchange(hmm: HMM, offsets, obs, component, ncomp, pairs, exchange=None, rescore_f64=True,
                                dtype="f64"):
    """cv_decode_constrained_exchange: one shard's constrained decode with the exchange step
    made by `exchange(words)` -- a callable that returns the SUM over all shards of the int64
    array `words` (e.g. cviterbi.dist.allreduce_partials); None = a single process.  `pairs`
    = constrained_pairs of the FULL batch.  Returns (path, score, status, comp_state,
    explored, objective) of this shard."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    component = np.ascontiguousarray(component, np.int32)
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    nseq = offsets.shape[0] - 1
    path = np.zeros(max(int(offsets[-1]), 1), np.int32)
    score = np.zeros(max(nseq, 1), np.float64)
    status = np.zeros(max(nseq, 1), np.uint8)
    states = np.full(max(ncomp, 1), -1, np.int32)
    explored, obj = ctypes.c_uint64(), ctypes.c_double()
    err = []

    def cb(words, n, _ctx):
        try:
            w = np.ctypeslib.as_array(words, shape=(n,))
            w[:] = np.asarray(exchange(w.copy()), np.int64).reshape(-1)
            return 0
        except Exception as e:  # reported after the call returns
            err.append(e)
            return 1

    fn = EXCHANGE_FN(cb) if exchange is not None else None  # kept alive for the call
    o = make_opts(dtype, "viterbi", "auto", rescore_f64)
    st = L.lib().cv_decode_constrained_exchange(hmm.handle, nseq, _p(offsets), _p(obs), _p(component), int(ncomp),
                                                len(pairs), _p(pairs) if len(pairs) else None,
                                                ctypes.cast(fn, ctypes.c_void_p) if fn else None, None,
                                                ctypes.byref(o), _p(path), _p(score), _p(status), _p(states),
                                                ctypes.byref(explored), ctypes.byref(obj))
    if err:
        raise err[0]
    L.check(st)
    return (path[:int(offsets[-1])], score[:nseq], status[:nseq], states[:ncomp], explored.value, obj.value)


def decode_constrained_device(hmm: HMM, offsets_host, offsets_dev, obs_dev, component, path_dev, score_dev, status_dev,
                              ncomp=None, rescore_f64=True, stream=None, workspace_bytes=0, dtype="f64"):
    """cv_decode_constrained_device: observations and outputs in HBM (ints or objects with
    data_ptr()), offsets_host/component on the host.  Synchronous.  Returns
    (comp_state[ncomp], objective)."""
    def ptr(x):
        return x.data_ptr() if hasattr(x, "data_ptr") else int(x)

    oh = np.ascontiguousarray(offsets_host, np.int64)
    component = np.ascontiguousarray(component, np.int32)
    if ncomp is None:
        ncomp = int(component.max()) + 1 if component.size else 0
    states = np.full(max(ncomp, 1), -1, np.int32)
    obj = ctypes.c_double()
    o = make_opts(dtype, "viterbi", "auto", rescore_f64, stream, workspace_bytes)
    L.check(L.lib().cv_decode_constrained_device(hmm.handle, oh.shape[0] - 1, _p(oh), ptr(offsets_dev), ptr(obs_dev),
                                                 _p(component), int(ncomp), ctypes.byref(o), ptr(path_dev),
                                                 ptr(score_dev), ptr(status_dev), _p(states), ctypes.byref(obj)))
    return states[:ncomp], obj.value


def decode_superseq_cp(hmm: HMM, offsets, obs):
    """cv_decode_superseq_cp: CPSolver::solve (cp.rs:133-143) exactly -- the sequences decoded
    as ONE chained super-sequence in f64 (utils.rs:62-103), as main.rs:120 runs it.
    Returns (path[sum T] in super-sequence order, objective)."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    obs = np.ascontiguousarray(obs, np.int32)
    path = np.zeros(max(int(offsets[-1] - offsets[0]), 1), np.int32)
    obj = ctypes.c_double()
    L.check(L.lib().cv_decode_superseq_cp(hmm.handle, offsets.shape[0] - 1, _p(offsets), _p(obs), _p(path),
                                          ctypes.byref(obj)))
    return path[:int(offsets[-1] - offsets[0])], obj.value


def last_superseq_stats(hmm: HMM) -> dict:
    """How the last decode_superseq_cp ran (cv_last_superseq_stats): parallel (the certified
    per-sequence decode + host fold) or the serial chain, and how many sequences certified /
    re-ran through the serial chain kernel."""
    out = (ctypes.c_int64 * 9)()
    L.check(L.lib().cv_last_superseq_stats(hmm.handle, out))
    return dict(parallel=bool(out[0]), certified=out[1], rerun=out[2], runs=out[3], quantised=out[4],
                speculated=out[5], spec_batches=out[6], gathered=out[7], path_waits=out[8])


def device_memory() -> dict:
    """Device bytes this process's library holds now and at most (cv_device_memory)."""
    cur, peak = ctypes.c_int64(), ctypes.c_int64()
    L.check(L.lib().cv_device_memory(ctypes.byref(cur), ctypes.byref(peak)))
    return dict(current=cur.value, peak=peak.value)


def _timing_dict(t):
    return dict(fwd_ms=t.fwd_ms, bt_ms=t.bt_ms, total_ms=t.total_ms, launches=t.launches,
                kernel={1: "trellis", 2: "generic", 3: "trellis_f64"}.get(t.kernel, "none"), padded_states=t.padded_states,
                seqs_per_wave=t.mfma_tiles)


def last_suffix_traced(hmm: HMM) -> int:
    """Constrained sequences of the last constrained decode whose forced path came from the
    certified suffix trace (cv_last_suffix_traced) rather than a second forward pass."""
    n = ctypes.c_int64()
    L.check(L.lib().cv_last_suffix_traced(hmm.handle, ctypes.byref(n)))
    return n.value


def last_timing(hmm: HMM) -> dict:
    """Device timings of the last decode call (synchronizes its events)."""
    t = L.Timing()
    L.check(L.lib().cv_last_timing(hmm.handle, ctypes.byref(t)))
    return _timing_dict(t)


def timing_begin(hmm: HMM):
    """Start summing the device timings of every decode call on `hmm` (cv_timing_begin)."""
    L.check(L.lib().cv_timing_begin(hmm.handle))


def timing_end(hmm: HMM) -> dict:
    """Sums since timing_begin (cv_timing_end; synchronizes the events)."""
    t = L.Timing()
    L.check(L.lib().cv_timing_end(hmm.handle, ctypes.byref(t)))
    return _timing_dict(t)


def decode(sequence, hmm: HMM):
    """viterbi::decode (viterbi.rs:5): sequence of [usize; D] (or flat ints) -> path (row 0 = 0.0 semantics)."""
    obs = np.ascontiguousarray([hmm.flat(o) for o in sequence], np.int32)
    path = np.zeros(obs.shape[0], np.int32)
    L.check(L.lib().cv_viterbi_decode(hmm.handle, obs.shape[0], _p(obs), _p(path)))
    return path
