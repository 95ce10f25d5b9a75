"""GPU: every BASELINE config in the DEFAULT mode (exact f64, the reference's arithmetic,
hmm.rs:10-18) against the f64 oracle -- the C restatement of the reference recurrence
(viterbi.rs:13-18 association, ndarray-stats first-index argmax), not another HIP kernel.

The GPU side always decodes the config's FULL batch, so the kernels under test are the ones
the bench runs at that size (layout, chunking, longest-first order); the oracle then checks
every sequence where it finishes in seconds (configs 2 and 3: all of them, OpenMP over the
box's CPU share) and a spread sample elsewhere (config 4).  Tolerance: none -- paths,
scores and statuses bit-identical (north_star asks paths bit-exact, scores within 1e-6).

  c1  house-A, N=5, T=50: golden fixture (tests/golden/golden_ar_house_a.npz, made from the
      reference's datasets/ar/house-A.csv) through the default Solver kind (gpu-cp, what
      main.rs:120 runs) and the default batch decode
  c2  N=45, 4,096 sequences, T in [1,128]: all sequences (trellis_wave_f64)
  c3  N=64, 16,384 sequences, T in [32,1024]: all sequences, incl. the 1,024-step ones that
      drive trellis_wave_f64's emission prefetch and the 32-row backtrack ring
  c4  N=256, T=512, 65,536 sequences: 256 sequences spread over the batch + the first/last
  c5  config 4 + K=7 components: see test_gpu_fullsize.py (sampled forced decodes given the
      chosen states) and test_gpu_constrained.py::test_constrained_config5_subset (states by
      the oracle's constrained spec at config-5 shape)
"""
import os

import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from conftest import load_golden
from cviterbi import synth

pytestmark = pytest.mark.gpu


def _threads():
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    return max(1, min(share, 16))


def _same(got, ref, what):
    gp, gs, gst = got
    rp, rs, rst = ref
    bad = np.nonzero(gst != rst)[0]
    assert bad.size == 0, f"{what}: status differs at seqs {bad[:8]}"
    bad = np.nonzero(gs != rs)[0]
    assert bad.size == 0, f"{what}: scores differ at seqs {bad[:8]}: {gs[bad[:4]]} vs {rs[bad[:4]]}"
    bad = np.nonzero(gp != rp)[0]
    assert bad.size == 0, f"{what}: paths differ at elements {bad[:8]}"


def _sub(off, obs, idx):
    """CSR sub-batch of sequences idx (in that order) and the element index of each."""
    lens = off[idx + 1] - off[idx]
    sub_off = synth.offsets_from_lengths(lens)
    el = np.concatenate([np.arange(off[k], off[k + 1]) for k in idx])
    return sub_off, obs[el], el


def test_config1_default_solver_and_decode(gpu):
    g = load_golden("golden_ar_house_a.npz")
    h = cv.HMM(g["pi"], g["a"], g["b"])
    # default batch decode (dtype default f64, row A0)
    got = cv.decode_batch(h, g["offsets"], g["obs"], rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    _same(got, (g["f64_viterbi_path"], g["f64_viterbi_score"], g["f64_viterbi_status"]), "c1 decode")
    ref = O.decode_batch(g["pi"], g["a"], g["b"], g["offsets"], g["obs"], O.VITERBI, np.float64)
    _same(got, ref, "c1 decode vs C oracle")
    # main.rs:120: CPSolver over the super-sequence (one sequence here), the default Solver kind
    seqs = [[(int(x), 0) for x in g["obs"]]]
    ss = cv.SuperSequence(seqs, None, h)
    s = cv.GpuSolver(h, ss)
    s.solve()
    assert s.get_name() == "gpu-cp"
    np.testing.assert_array_equal(s.get_solution(), g["f64_cp_path"])
    assert s.get_objective() == g["f64_cp_score"][0]
    p, obj = O.cp_superseq_f64(g["pi"], g["a"], g["b"], g["offsets"], g["obs"])
    np.testing.assert_array_equal(s.get_solution(), p)
    assert s.get_objective() == obj


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_full_config_default_vs_oracle(gpu, name):
    c = synth.config(name)
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, rescore_f64=False)  # default mode: exact f64
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64", t
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, nthreads=_threads())
    assert np.all(ref[2] == 0)
    _same(got, ref, f"{name} full batch f64 vs oracle")
    if name == "c3":  # the longest sequences are in the batch and were compared
        assert int((off[1:] - off[:-1]).max()) == 1024


def test_config4_default_vs_oracle_sample(gpu):
    c = synth.config("c4")
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b.reshape(256, 32, 32))
    got = cv.decode_batch(h, off, obs, rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    B = len(off) - 1
    idx = np.unique(np.concatenate([np.linspace(0, B - 1, 254).astype(np.int64), [1, B - 2]]))
    sub_off, sub_obs, el = _sub(off, obs, idx)
    ref = O.decode_batch(pi, a, b, sub_off, sub_obs, O.VITERBI, np.float64, nthreads=_threads())
    _same((got[0][el], got[1][idx], got[2][idx]), ref, "c4 sample f64 vs oracle")
