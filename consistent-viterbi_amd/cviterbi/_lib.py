"""ctypes binding of libcviterbi.so (include/cviterbi.h).

This is the same binding a maintainer of the reference would write as a Rust
`extern "C"` block; here it is the Python host layer.  There is no
fallback: if the library or a gfx950 device is missing, calls raise CVError.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CV_LIB_PATH: an A/B variant build (tools/ab_*.sh) loaded instead of the in-tree library, so
# the scripts never overwrite the product .so (a killed A/B run used to leave a variant behind)
LIB_PATH = os.environ.get("CV_LIB_PATH") or os.path.join(_HERE, "libcviterbi.so")

(CV_OK, CV_EINVAL, CV_EDEVICE, CV_ENOMEM, CV_EINFEASIBLE, CV_EIO, CV_EPARSE, CV_EUNSUPPORTED, CV_EINTERNAL,
 CV_ELIMIT) = range(10)
STATUS_NAMES = {0: "CV_OK", 1: "CV_EINVAL", 2: "CV_EDEVICE", 3: "CV_ENOMEM", 4: "CV_EINFEASIBLE", 5: "CV_EIO",
                6: "CV_EPARSE", 7: "CV_EUNSUPPORTED", 8: "CV_EINTERNAL", 9: "CV_ELIMIT"}
SEQ_OK, SEQ_INFEASIBLE, SEQ_EMPTY, SEQ_BADOBS = 0, 1, 2, 3
DTYPE_F32, DTYPE_F64 = 0, 1
ASSOC_VITERBI, ASSOC_CP, ASSOC_DP, ASSOC_DECODE = 0, 1, 2, 3
KERNEL_AUTO, KERNEL_TRELLIS, KERNEL_GENERIC, KERNEL_TRELLIS_F64 = 0, 1, 2, 3
FLAG_NO_PAIR = 0x4
FLAG_NO_WAVE = 0x8
FLAG_NO_T64 = 0x10
FLAG_SERIAL = 0x2


# every symbol include/cviterbi.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "cv_last_error", "cv_version", "cv_abi_version", "cv_device_count", "cv_device_memory", "cv_opts_init",
    "cv_hmm_create", "cv_hmm_from_json", "cv_hmm_write_json", "cv_hmm_destroy", "cv_hmm_nstates", "cv_hmm_nobs",
    "cv_hmm_ndims", "cv_hmm_bdims", "cv_obs_flatten", "cv_hmm_init_prob", "cv_hmm_init_probs",
    "cv_hmm_transition_prob", "cv_hmm_transitions_to", "cv_hmm_emit_prob", "cv_hmm_emit_probs",
    "cv_decode_batch", "cv_decode_batch_device", "cv_last_timing", "cv_timing_begin", "cv_timing_end",
    "cv_decode_constrained", "cv_decode_constrained_device", "cv_last_suffix_traced", "cv_decode_constrained_exchange",
    "cv_constrained_pairs", "cv_constrained_partials", "cv_constrained_select", "cv_decode_forced_components", "cv_viterbi_decode",
    "cv_decode_superseq_cp", "cv_last_superseq_stats",
    "cv_solver_create", "cv_solver_solve", "cv_solver_get_solution", "cv_solver_get_objective",
    "cv_solver_get_name", "cv_solver_get_explored_nodes", "cv_solver_destroy",
    "cv_hmm_fit_mle", "cv_hmm_fit_train", "cv_solver_write_cfn",
    "cv_hmm_set_tuning", "cv_hmm_get_tuning", "cv_tuning_key", "cv_hmm_release_workspaces",
]


class CVError(RuntimeError):
    def __init__(self, status, message):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


class HmmDesc(ctypes.Structure):
    _fields_ = [("nstates", ctypes.c_int32), ("ndims", ctypes.c_int32), ("bdims", ctypes.c_void_p),
                ("pi", ctypes.c_void_p), ("a", ctypes.c_void_p), ("b", ctypes.c_void_p), ("device", ctypes.c_int32)]


class Opts(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("assoc", ctypes.c_int32), ("kernel", ctypes.c_int32),
                ("rescore_f64", ctypes.c_int32), ("stream", ctypes.c_void_p), ("workspace_bytes", ctypes.c_uint64),
                ("flags", ctypes.c_uint32), ("forced", ctypes.c_void_p)]


class Timing(ctypes.Structure):
    _fields_ = [("fwd_ms", ctypes.c_double), ("bt_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("launches", ctypes.c_int64), ("kernel", ctypes.c_int32), ("padded_states", ctypes.c_int32),
                ("mfma_tiles", ctypes.c_int32)]


class SuperSeqDesc(ctypes.Structure):
    _fields_ = [("nseq", ctypes.c_int64), ("offsets", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("seq_id", ctypes.c_void_p), ("component", ctypes.c_void_p), ("active", ctypes.c_void_p)]


_lib = None


def lib():
    """Load libcviterbi.so (raises if it has not been built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CVError(CV_EDEVICE, f"{LIB_PATH} not built (python -c 'import __graft_entry__ as g; g.build()')")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7.  Loading torch
    # first makes our NEEDED libamdhip64.so.7 resolve to that already-loaded copy, so
    # torch-allocated buffers, torch streams and our kernels share one runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64, D, S = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_int
    sig = {
        "cv_last_error": ([], ctypes.c_char_p),
        "cv_version": ([], ctypes.c_char_p),
        "cv_abi_version": ([], I32),
        "cv_device_count": ([], I32),
        "cv_opts_init": ([P], None),
        "cv_hmm_create": ([P, P], S),
        "cv_hmm_from_json": ([ctypes.c_char_p, I32, P], S),
        "cv_hmm_write_json": ([P, ctypes.c_char_p], S),
        "cv_hmm_destroy": ([P], None),
        "cv_hmm_set_tuning": ([P, ctypes.c_char_p, I64], S),
        "cv_hmm_get_tuning": ([P, ctypes.c_char_p, P], S),
        "cv_tuning_key": ([I32], ctypes.c_char_p),
        "cv_hmm_release_workspaces": ([P], S),
        "cv_hmm_nstates": ([P], I32),
        "cv_hmm_nobs": ([P], I64),
        "cv_hmm_ndims": ([P], I32),
        "cv_hmm_bdims": ([P, P], S),
        "cv_obs_flatten": ([P, P, P], S),
        "cv_hmm_init_prob": ([P, I32, I64], D),
        "cv_hmm_init_probs": ([P, I64, P], S),
        "cv_hmm_transition_prob": ([P, I32, I32, I64], D),
        "cv_hmm_transitions_to": ([P, I32, P], S),
        "cv_hmm_emit_prob": ([P, I32, I64], D),
        "cv_hmm_emit_probs": ([P, I64, P], S),
        "cv_decode_batch": ([P, I64, P, P, P, P, P, P], S),
        "cv_decode_batch_device": ([P, I64, P, P, P, P, P, P, P], S),
        "cv_last_timing": ([P, P], S),
        "cv_timing_begin": ([P], S),
        "cv_timing_end": ([P, P], S),
        "cv_last_suffix_traced": ([P, P], S),
        "cv_decode_constrained": ([P, I64, P, P, P, I32, P, P, P, P, P, P], S),
        "cv_decode_constrained_device": ([P, I64, P, P, P, P, I32, P, P, P, P, P, P], S),
        "cv_decode_constrained_exchange": ([P, I64, P, P, P, I32, I64, P, P, P, P, P, P, P, P, P, P], S),
        "cv_constrained_pairs": ([I64, P, P, I32, P, I64, P], S),
        "cv_constrained_partials": ([P, I64, P, P, P, I32, I64, P, P, P], S),
        "cv_constrained_select": ([I32, I32, I64, P, P, P, P], S),
        "cv_decode_forced_components": ([P, I64, P, P, P, I32, P, P, P, P, P, P], S),
        "cv_viterbi_decode": ([P, I64, P, P], S),
        "cv_decode_superseq_cp": ([P, I64, P, P, P, P], S),
        "cv_last_superseq_stats": ([P, P], S),
        "cv_device_memory": ([P, P], S),
        "cv_solver_create": ([ctypes.c_char_p, P, P, P], S),
        "cv_solver_solve": ([P], S),
        "cv_solver_get_solution": ([P, P, P], S),
        "cv_solver_get_objective": ([P, P], S),
        "cv_solver_get_name": ([P], ctypes.c_char_p),
        "cv_solver_get_explored_nodes": ([P, P], S),
        "cv_solver_destroy": ([P], None),
        "cv_solver_write_cfn": ([P, ctypes.c_char_p, P], S),
        "cv_hmm_fit_mle": ([I32, I64, I64, P, P, P, I32, P, P, P], S),
        "cv_hmm_fit_train": ([I32, I64, I64, P, P, P, I32, D, I32, P, P, P, P], S),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(status):
    if status != CV_OK:
        raise CVError(status, lib().cv_last_error().decode())


def opts(dtype=DTYPE_F32, assoc=ASSOC_VITERBI, kernel=KERNEL_AUTO, rescore_f64=True, stream=None,
         workspace_bytes=0, flags=0):
    o = Opts()
    lib().cv_opts_init(ctypes.byref(o))
    o.dtype, o.assoc, o.kernel, o.rescore_f64 = dtype, assoc, kernel, int(bool(rescore_f64))
    o.stream = stream
    o.workspace_bytes = workspace_bytes
    o.flags = flags
    return o
