"""CPU: the C-ABI library loads, exports exactly what include/cviterbi.h declares, and its
host-side entry points (HMM lookups, hmm.json I/O, argument checking) behave like the
reference's hmm.rs -- no compute calls (those need the GPU: tests/test_gpu_parity.py)."""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

import cviterbi as cv
from conftest import ROOT, has_gpu
from cviterbi import _lib as L
from cviterbi import synth

HEADER = os.path.join(ROOT, "include", "cviterbi.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"CV_API\s+[\w\s\*]+?\b(cv_\w+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert declared() == sorted(L.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", L.LIB_PATH], text=True)
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared() if s not in syms]
    assert not missing, missing
    lib = L.lib()
    for s in declared():
        assert getattr(lib, s) is not None
    # nothing else leaks from the C++ side with default visibility
    extra = [s for s in syms if s.startswith("cv_") and s not in declared()]
    assert not extra, extra


def test_version_and_opts_defaults():
    lib = L.lib()
    assert lib.cv_abi_version() == 1
    assert b"gfx950" in lib.cv_version()
    o = L.Opts()
    lib.cv_opts_init(ctypes.byref(o))
    # default dtype = CV_DTYPE_F64: the reference's arithmetic (hmm.rs:10-18)
    assert (o.dtype, o.assoc, o.kernel, o.rescore_f64, o.workspace_bytes) == (1, 0, 0, 1, 0)


def _model():
    pi, a, b = synth.random_hmm(6, 12, seed=21, zero_frac=0.2)
    return pi, a, b


def test_lookups_match_hmm_rs():
    pi, a, b = _model()
    h = cv.HMM(pi, a, b.reshape(6, 3, 4))
    assert h.nstates() == 6 and h.nobs() == 12 and h.bdims() == (3, 4)
    for s in range(6):
        for o in range(12):
            assert h.emit_prob(s, o) == b[s, o]                                   # hmm.rs:228-230
            assert h.init_prob(s, o) == pi[s] + b[s, o]                           # hmm.rs:211-213
            for f in range(6):
                assert h.transition_prob(f, s, o) == a[f, s] + b[s, o]            # hmm.rs:220-222
    for o in range(12):
        np.testing.assert_array_equal(h.init_probs(o), pi + b[:, o])             # hmm.rs:215-218
        np.testing.assert_array_equal(h.emit_probs(o), b[:, o])                  # hmm.rs:232-234
    for t in range(6):
        np.testing.assert_array_equal(h.transitions_to(t), a[:, t])              # hmm.rs:224-226
    # [usize; D] observations flatten row-major like ndarray's b[state][&obs[..]]
    assert h.flat((2, 3)) == 11 and h.flat((1, 0)) == 4
    assert h.emit_prob(2, h.flat((1, 2))) == b.reshape(6, 3, 4)[2, 1, 2]
    with pytest.raises(cv.CVError):
        h.flat((3, 0))


def test_json_roundtrip_and_reference_layout(tmp_path):
    pi, a, b = _model()
    h = cv.HMM(pi, a, b.reshape(6, 3, 4))
    p = tmp_path / "hmm.json"
    h.write(p)
    d = json.loads(p.read_text())
    # serde layout of struct HMM<D> with ndarray 0.15 (hmm.rs:10-18): -inf written as null
    assert d["a"]["dim"] == [6, 6] and d["pi"]["dim"] == [6] and d["b"]["dim"] == [6]
    assert d["b"]["data"][0]["dim"] == [3, 4]
    assert (None in d["a"]["data"]) == bool(np.isneginf(a).any())
    h2 = cv.HMM.from_json(p)
    for o in range(12):
        np.testing.assert_array_equal(h2.emit_probs(o), b[:, o])
        np.testing.assert_array_equal(h2.init_probs(o), pi + b[:, o])
    for t in range(6):
        np.testing.assert_array_equal(h2.transitions_to(t), a[:, t])


def test_json_written_by_serde_style(tmp_path):
    """A hand-written file in the reference's exact serde_json shape, nulls for -inf."""
    txt = ('{"a":{"v":1,"dim":[2,2],"data":[-0.1549019599857432,-0.5228787452803376,null,0.0]},'
           '"b":{"v":1,"dim":[2],"data":[{"v":1,"dim":[3,1],"data":[-0.3010299956639812,-0.3010299956639812,null]},'
           '{"v":1,"dim":[3,1],"data":[null,-0.47712125471966244,-0.17609125905568124]}]},'
           '"pi":{"v":1,"dim":[2],"data":[-0.3010299956639812,-0.3010299956639812]}}')
    p = tmp_path / "hmm.json"
    p.write_text(txt)
    h = cv.HMM.from_json(p)
    assert h.nstates() == 2 and h.bdims() == (3, 1)
    assert h.transition_prob(1, 0, 2) == -np.inf and h.emit_prob(1, 0) == -np.inf
    assert h.transition_prob(0, 1, 1) == -0.5228787452803376 + -0.47712125471966244


@pytest.mark.parametrize("bad,code", [("{", L.CV_EPARSE), ('{"a":1}', L.CV_EPARSE),
                                      ('{"a":{"v":1,"dim":[2,2],"data":[1,2,3]},"b":{"dim":[0],"data":[]},'
                                       '"pi":{"v":1,"dim":[2],"data":[0,0]}}', L.CV_EPARSE),
                                      # dims: overflowing product, fractional, negative, huge
                                      ('{"a":{"v":1,"dim":[99999999999,99999999999],"data":[]}}', L.CV_EPARSE),
                                      ('{"a":{"v":1,"dim":[1.5,2],"data":[1,2,3]}}', L.CV_EPARSE),
                                      ('{"a":{"v":1,"dim":[-1,2],"data":[]}}', L.CV_EPARSE),
                                      ('{"a":{"v":1,"dim":[1e300],"data":[]}}', L.CV_EPARSE),
                                      # non-JSON number forms strtod would accept
                                      ('{"a":{"v":1,"dim":[1,1],"data":[nan]}}', L.CV_EPARSE),
                                      ('{"a":{"v":1,"dim":[1,1],"data":[0x10]}}', L.CV_EPARSE),
                                      ('{"a":{"v":1,"dim":[1,1],"data":[inf]}}', L.CV_EPARSE)])
def test_json_errors(tmp_path, bad, code):
    p = tmp_path / "bad.json"
    p.write_text(bad)
    with pytest.raises(cv.CVError) as e:
        cv.HMM.from_json(p)
    assert e.value.status == code
    with pytest.raises(cv.CVError) as e:
        cv.HMM.from_json(tmp_path / "missing.json")
    assert e.value.status == L.CV_EIO


@pytest.mark.parametrize("val", [np.nan, np.inf])
def test_model_validation(val):
    pi, a, b = _model()
    a = a.copy()
    a[1, 2] = val
    with pytest.raises(cv.CVError) as e:
        cv.HMM(pi, a, b)
    assert e.value.status == L.CV_EINVAL


def test_negative_zero_canonicalised():
    pi, a, b = _model()
    a = a.copy()
    a[0, 0] = -0.0
    h = cv.HMM(pi, a, b)
    v = h.transitions_to(0)[0]
    assert v == 0.0 and not np.signbit(v)


@pytest.mark.skipif(has_gpu(), reason="checks the no-device error path")
def test_decode_without_device_fails_loudly():
    pi, a, b = _model()
    h = cv.HMM(pi, a, b)
    with pytest.raises(cv.CVError) as e:
        cv.decode_batch(h, [0, 3], np.array([1, 2, 3], np.int32), dtype="f32")
    assert e.value.status == L.CV_EDEVICE


def test_argument_errors():
    pi, a, b = _model()
    h = cv.HMM(pi, a, b)
    with pytest.raises(cv.CVError) as e:  # non-monotone offsets
        cv.decode_batch(h, [0, 3, 2], np.array([1, 2, 3], np.int32), dtype="f32")
    assert e.value.status in (L.CV_EINVAL, L.CV_EDEVICE)
    with pytest.raises(cv.CVError) as e:  # obs out of range
        cv.decode_batch(h, [0, 2], np.array([1, 99], np.int32), dtype="f32")
    assert e.value.status in (L.CV_EINVAL, L.CV_EDEVICE)
    with pytest.raises(cv.CVError) as e:
        cv.GpuSolver(h, cv.SuperSequence([[1, 2]], None, h), kind="nope")
    assert e.value.status == L.CV_EINVAL
