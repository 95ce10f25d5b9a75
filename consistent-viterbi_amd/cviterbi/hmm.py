"""HMM: Python face of `struct HMM<D>` (reference src/hmm/hmm.rs) over the C ABI.

Same names and argument meaning as the reference: log10 probabilities, `a[from, to]`,
`b[state][obs]` with `obs` a D-tuple (flattened row-major like ndarray) or an already
flat index.  Lookups are served by libcviterbi (cv_hmm_*); model fitting (`new`,
`train`, `maximum_likelihood_estimation`, hmm.rs:22-190) is out of scope (SURVEY.md §2
row 1) -- construct from arrays or from the reference's hmm.json.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def _p(x):
    return x.ctypes.data_as(ctypes.c_void_p)


class HMM:
    def __init__(self, pi, a, b, bdims=None, device=0):
        """pi[N], a[N,N], b[N,*bdims] (or b[N,V] with bdims) as log10 float64 arrays."""
        pi = np.ascontiguousarray(pi, np.float64)
        a = np.ascontiguousarray(a, np.float64)
        b = np.asarray(b, np.float64)
        n = pi.shape[0]
        if bdims is None:
            bdims = b.shape[1:] if b.ndim > 1 else (1,)
        bdims = tuple(int(d) for d in bdims)
        b = np.ascontiguousarray(b.reshape(n, -1))
        bd = np.ascontiguousarray(bdims, np.int64)
        desc = L.HmmDesc(n, len(bdims), bd.ctypes.data, pi.ctypes.data, a.ctypes.data, b.ctypes.data, int(device))
        h = ctypes.c_void_p()
        L.check(L.lib().cv_hmm_create(ctypes.byref(desc), ctypes.byref(h)))
        self._h = h
        self.device = int(device)

    @classmethod
    def from_json(cls, path, device=0):
        """HMM::from_json (hmm.rs:242-245): the reference's serde layout, null = -inf."""
        self = cls.__new__(cls)
        h = ctypes.c_void_p()
        L.check(L.lib().cv_hmm_from_json(str(path).encode(), int(device), ctypes.byref(h)))
        self._h = h
        self.device = int(device)
        return self

    def write(self, path):
        """HMM::write (hmm.rs:236-240)."""
        L.check(L.lib().cv_hmm_write_json(self._h, str(path).encode()))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and L is not None and L.lib is not None:  # module globals may be gone at interpreter exit
            try:
                L.lib().cv_hmm_destroy(h)
            except TypeError:
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    # ---- tuning keys (include/cviterbi.h): per-handle layout / schedule / A-B choices --------
    def set_tuning(self, **keys):
        """cv_hmm_set_tuning for each key=value (bit-identical in results; see cviterbi.h).
        The handle's snapshot was taken from the CV_<KEY> environment at creation; later
        environment changes do not reach it, this does."""
        for k, v in keys.items():
            L.check(L.lib().cv_hmm_set_tuning(self._h, k.encode(), int(v)))

    def release_workspaces(self):
        """cv_hmm_release_workspaces: free the decode workspaces this handle keeps between calls."""
        L.check(L.lib().cv_hmm_release_workspaces(self._h))

    def tuning(self, key) -> int:
        """cv_hmm_get_tuning: the handle's current value of one tuning key."""
        v = ctypes.c_int64()
        L.check(L.lib().cv_hmm_get_tuning(self._h, key.encode(), ctypes.byref(v)))
        return v.value

    def tuned(self, **keys):
        """Context manager: the given tuning keys for the block, the previous values after it."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.tuning(k) for k in keys}
            self.set_tuning(**keys)
            try:
                yield self
            finally:
                self.set_tuning(**old)

        return cm()


    # ---- shape -----------------------------------------------------------------------
    def nstates(self) -> int:
        """HMM::nstates (hmm.rs:207-209)."""
        return L.lib().cv_hmm_nstates(self._h)

    def nobs(self) -> int:
        return L.lib().cv_hmm_nobs(self._h)

    def bdims(self):
        d = L.lib().cv_hmm_ndims(self._h)
        out = np.zeros(d, np.int64)
        L.check(L.lib().cv_hmm_bdims(self._h, _p(out)))
        return tuple(int(x) for x in out)

    def flat(self, obs) -> int:
        """[usize; D] observation -> flat index (row-major over bdims)."""
        if isinstance(obs, (int, np.integer)):
            return int(obs)
        v = np.ascontiguousarray(obs, np.int64)
        out = ctypes.c_int64()
        L.check(L.lib().cv_obs_flatten(self._h, _p(v), ctypes.byref(out)))
        return out.value

    # ---- lookups (hmm.rs:211-234) -------------------------------------------------------
    def init_prob(self, state, obs) -> float:
        return L.lib().cv_hmm_init_prob(self._h, int(state), self.flat(obs))

    def init_probs(self, obs):
        out = np.zeros(self.nstates())
        L.check(L.lib().cv_hmm_init_probs(self._h, self.flat(obs), _p(out)))
        return out

    def transition_prob(self, state_from, state_to, obs) -> float:
        return L.lib().cv_hmm_transition_prob(self._h, int(state_from), int(state_to), self.flat(obs))

    def transitions_to(self, state_to):
        out = np.zeros(self.nstates())
        L.check(L.lib().cv_hmm_transitions_to(self._h, int(state_to), _p(out)))
        return out

    def emit_prob(self, state, obs) -> float:
        return L.lib().cv_hmm_emit_prob(self._h, int(state), self.flat(obs))

    def emit_probs(self, obs):
        out = np.zeros(self.nstates())
        L.check(L.lib().cv_hmm_emit_probs(self._h, self.flat(obs), _p(out)))
        return out


def tuning_keys():
    """Every tuning key the library knows (cv_tuning_key)."""
    out, i = [], 0
    while True:
        k = L.lib().cv_tuning_key(i)
        if not k:
            return out
        out.append(k.decode())
        i += 1
