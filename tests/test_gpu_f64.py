"""Exact-f64 trellis kernel (trellis_fwd_f64 + backtrack_f64) against the f64
oracle: the reference's own precision (hmm.rs:10-18 stores f64; viterbi.rs:13-18 row A0).

Bar (BASELINE.json north_star): paths bit-exact and scores bit-exact (tolerance 0 < 1e-6
relative) against the f64 oracle, every status identical; and identical to the generic f64
kernel (inline first-argmax) on batches too large for the oracle to finish in seconds.
"""
import os

import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu
PKG = os.path.dirname(os.path.dirname(os.path.abspath(cv.__file__)))


def _case(n, v, seed, nseq=12, tmax=70, zero_frac=0.0, tmin=1):
    pi, a, b = synth.random_hmm(n, v, seed=seed, zero_frac=zero_frac)
    rng = np.random.default_rng(seed + 100)
    lengths = rng.integers(tmin, tmax + 1, size=nseq)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    return pi, a, b, off, obs


def _assert_same(got, ref, what):
    gp, gs, gst = got
    rp, rs, rst = ref
    assert np.array_equal(gst, rst), f"{what}: status {gst} vs {rst}"
    bad = np.nonzero(gs != rs)[0]
    assert bad.size == 0, f"{what}: scores differ at seqs {bad[:8]}: {gs[bad[:4]]} vs {rs[bad[:4]]}"
    assert np.array_equal(gp, rp), f"{what}: paths differ at {np.nonzero(gp != rp)[0][:8]}"


ASSOC = {"viterbi": O.VITERBI, "cp": O.CP, "dp": O.DP, "decode": O.DECODE}


@pytest.mark.parametrize("n", [1, 2, 5, 33, 45, 63, 64, 65, 100, 128, 129, 192, 200, 255, 256])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp", "decode"])
def test_t64_bit_exact_vs_oracle(gpu, n, assoc):
    """Row A0 (viterbi.rs:13-18), CPSolver's association (cp.rs:70-79: argmax tracked in the
    forward pass, value d[psi] + (a + b)) and viterbi::decode (row 0 = 0.0)."""
    pi, a, b, off, obs = _case(n, 41, seed=700 + n, zero_frac=0.05 if n % 2 else 0.0)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64", t
    assert t["padded_states"] == 64 * ((n + 63) // 64)
    ref = O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], np.float64)
    _assert_same(got, ref, f"t64 {assoc} N={n}")
    if assoc == "viterbi":
        # rescore_f64 changes nothing on the f64 path: the f64 delta already is the reference score
        _assert_same(cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=True), ref, f"t64 rescore N={n}")


@pytest.mark.parametrize("n", [7, 64, 256])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp", "decode"])
def test_t64_ties_and_infeasible(gpu, n, assoc):
    """Quantised log-probs (many exact ties: first index must win), -inf transitions and
    emissions (infeasible sequences), an out-of-range observation, empty and T=1 sequences."""
    rng = np.random.default_rng(n)
    v = 9
    pi = np.round(rng.uniform(-2, 0, n) * 2) / 2
    a = np.round(rng.uniform(-2, 0, (n, n)) * 2) / 2
    b = np.round(rng.uniform(-2, 0, (n, v)) * 2) / 2
    a[rng.random((n, n)) < 0.2] = -np.inf
    b[:, 3] = -np.inf  # observation 3 is impossible in every state: infeasible sequences
    lengths = np.array([0, 1, 2, 17, 40, 0, 5, 33, 1, 60, 12, 12])
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    obs[obs == 3] = 4
    obs[off[3] + 5] = 3   # sequence 3 infeasible
    obs[off[9] + 59] = 3  # sequence 9 infeasible at its last element
    h = cv.HMM(pi, a, b)
    ref = O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], np.float64)
    _assert_same(cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False), ref,
                 f"ties {assoc} N={n}")
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    # out-of-range observation index: rejected (CV_EINVAL) before any kernel runs
    obs_bad = obs.copy()
    obs_bad[off[4] + 2] = v + 5
    for kernel in ("auto", "generic"):
        with pytest.raises(cv.CVError, match="out of range"):
            cv.decode_batch(h, off, obs_bad, dtype="f64", kernel=kernel, rescore_f64=False)


@pytest.mark.parametrize("nseq,uniform", [(8192, False), (8192, True), (12000, True), (4096, False), (2048, False)])
def test_t64_small_batch_layouts_vs_generic(gpu, nseq, uniform):
    """N = 256 batches too small for 8 sequences per wave (8,192 = one GPU of 8-GPU strong
    scaling): 2S sequences over a pair of waves -- the row split (trellis_fwd_f64_rs, four pairs
    per workgroup) for equal lengths, the column split (trellis_fwd_f64<2, 2S, .., W=2>) for
    ragged ones -- the whole batch equals the generic f64 kernel, scores are the f64 fold of
    each path, and the layout reported is the small-batch one."""
    pi, a, b = synth.random_hmm(256, 64, seed=77)
    rng = np.random.default_rng(nseq)
    lengths = np.full(nseq, 44) if uniform else rng.integers(40, 49, size=nseq)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, 64, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["seqs_per_wave"] in (2, 4), t
    _assert_same(got, cv.decode_batch(h, off, obs, dtype="f64", kernel="generic", rescore_f64=False), f"B={nseq}")
    assert np.all(got[2] == 0)
    np.testing.assert_array_equal(got[1], O.rescore_batch_f64(pi, a, b, off, obs, got[0]))


def test_t64_simd_balance_knob_bit_identical(gpu, tmp_path):
    """SIMD balancing (issue priority by remaining work) and the small-batch pair layout are
    scheduling only: a child process with CV_T64_BAL=0 (no balancing) and CV_T64_W2=0 (one wave
    per group) decodes the same single-round batch to the same bits."""
    import subprocess
    import sys

    pi, a, b = synth.random_hmm(256, 64, seed=79)
    rng = np.random.default_rng(79)
    off = synth.offsets_from_lengths(rng.integers(60, 97, size=8192))
    obs = rng.integers(0, 64, size=int(off[-1])).astype(np.int32)
    np.savez(tmp_path / "in.npz", pi=pi, a=a, b=b, off=off, obs=obs)
    got = cv.decode_batch(cv.HMM(pi, a, b), off, obs, dtype="f64", rescore_f64=False)
    code = (
        "import sys, numpy as np; sys.path.insert(0, sys.argv[1]); import cviterbi as cv; "
        "d = np.load(sys.argv[2]); h = cv.HMM(d['pi'], d['a'], d['b']); "
        "p, s, st = cv.decode_batch(h, d['off'], d['obs'], dtype='f64', rescore_f64=False); "
        "np.savez(sys.argv[3], p=p, s=s, st=st)")
    env = dict(os.environ, CV_T64_BAL="0", CV_T64_W2="0")
    subprocess.run([sys.executable, "-c", code, PKG, str(tmp_path / "in.npz"), str(tmp_path / "out.npz")],
                   env=env, check=True, timeout=120)
    ref = np.load(tmp_path / "out.npz")
    _assert_same(got, (ref["p"], ref["s"], ref["st"]), "balance/W2 knobs")


@pytest.mark.parametrize("n", [256, 200, 128])
def test_t64_layout_knob_s6_bit_identical(gpu, tmp_path, n):
    """The 3-waves-per-SIMD layout (6 sequences per wave, CV_T64_S=6) is scheduling only: a
    child process decodes the same ragged batch to the same bits as the default layout."""
    import subprocess
    import sys

    pi, a, b = synth.random_hmm(n, 64, seed=80 + n)
    rng = np.random.default_rng(80 + n)
    off = synth.offsets_from_lengths(rng.integers(1, 97, size=6000))
    obs = rng.integers(0, 64, size=int(off[-1])).astype(np.int32)
    np.savez(tmp_path / "in.npz", pi=pi, a=a, b=b, off=off, obs=obs)
    got = cv.decode_batch(cv.HMM(pi, a, b), off, obs, dtype="f64", rescore_f64=False)
    code = (
        "import sys, numpy as np; sys.path.insert(0, sys.argv[1]); import cviterbi as cv; "
        "d = np.load(sys.argv[2]); h = cv.HMM(d['pi'], d['a'], d['b']); "
        "p, s, st = cv.decode_batch(h, d['off'], d['obs'], dtype='f64', rescore_f64=False); "
        "assert cv.last_timing(h)['seqs_per_wave'] == 6; "
        "np.savez(sys.argv[3], p=p, s=s, st=st)")
    env = dict(os.environ, CV_T64_S="6")
    subprocess.run([sys.executable, "-c", code, PKG, str(tmp_path / "in.npz"), str(tmp_path / "out.npz")],
                   env=env, check=True, timeout=120)
    ref = np.load(tmp_path / "out.npz")
    _assert_same(got, (ref["p"], ref["s"], ref["st"]), f"S=6 layout N={n}")


@pytest.mark.parametrize("n,s", [(256, 8), (200, 8), (192, 8), (256, 4)])
def test_t64_workgroup_units_bit_identical(gpu, tmp_path, n, s):
    """Eight waves per workgroup (S = 8: eight one-wave units, a barrier per step and the SIMD
    pairs' priority trade; S = 4 at N = 256: four pairs of waves) are scheduling only.  Ragged
    lengths 1..96 (units of one workgroup finish at different steps: the trailing barriers) and
    a batch that leaves the last workgroup partly empty: child processes with CV_T64_WG=0 (tuning
    key t64_wg: one unit per workgroup) and the default decode the same bits as this process's
    default layout."""
    import subprocess
    import sys

    pi, a, b = synth.random_hmm(n, 64, seed=90 + n)
    rng = np.random.default_rng(90 + n + s)
    lengths = rng.integers(1, 97, size=5000)
    lengths[rng.integers(0, 5000, size=40)] = 0  # empty sequences inside workgroups
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, 64, size=int(off[-1])).astype(np.int32)
    np.savez(tmp_path / "in.npz", pi=pi, a=a, b=b, off=off, obs=obs)
    got = cv.decode_batch(cv.HMM(pi, a, b), off, obs, dtype="f64", rescore_f64=False)
    code = (
        "import sys, numpy as np; sys.path.insert(0, sys.argv[1]); import cviterbi as cv; "
        "d = np.load(sys.argv[2]); h = cv.HMM(d['pi'], d['a'], d['b']); "
        "p, s, st = cv.decode_batch(h, d['off'], d['obs'], dtype='f64', rescore_f64=False); "
        f"assert cv.last_timing(h)['seqs_per_wave'] == {s}; "
        "np.savez(sys.argv[3], p=p, s=s, st=st)")
    for wg in ("1", "0"):  # ragged and < 4 rounds: the default takes one-wave units, so force
        env = dict(os.environ, CV_T64_S=str(s), CV_T64_WG=wg, CV_T64_WG_FORCE="1")
        out = tmp_path / f"out{wg}.npz"
        subprocess.run([sys.executable, "-c", code, PKG, str(tmp_path / "in.npz"), str(out)],
                       env=env, check=True, timeout=120)
        ref = np.load(out)
        _assert_same(got, (ref["p"], ref["s"], ref["st"]), f"CV_T64_WG={wg} S={s} N={n}")


@pytest.mark.parametrize("n", [64, 200, 256])
@pytest.mark.parametrize("kind", ["near_ties", "positive", "huge"])
def test_t64_backtrack_interval_paths(gpu, n, kind):
    """The backtrack's two interval tests (trellis64.hip bt_chain_f64).  near_ties: a log-prob
    model whose transitions differ below f32 resolution (1e-12 perturbations of a quantised
    matrix), so the NONPOS f32 test finds several survivors at most steps and the exact f64
    fallback decides; positive / huge: a model with an entry > 0, or one below -2^80 -- the
    NONPOS test does not apply and the general f64 interval test runs."""
    rng = np.random.default_rng(900 + n)
    v = 17
    pi = np.round(rng.uniform(-2, 0, n) * 4) / 4
    a = np.round(rng.uniform(-2, 0, (n, n)) * 4) / 4
    b = np.round(rng.uniform(-2, 0, (n, v)) * 4) / 4
    if kind == "near_ties":
        a = a - rng.uniform(0, 1e-12, (n, n))
        b = b - rng.uniform(0, 1e-12, (n, v))
    elif kind == "positive":
        a = a + 0.75  # some transitions > 0: scores, not log-probabilities
    else:
        a[rng.random((n, n)) < 0.02] = -1e30
    lengths = np.array([1, 2, 17, 40, 5, 33, 60, 12, 64, 65, 128, 3])
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    for assoc in ("viterbi", "decode", "dp"):
        got = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False)
        assert cv.last_timing(h)["kernel"] == "trellis_f64"
        _assert_same(got, O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], np.float64), f"{kind} {assoc} N={n}")


@pytest.mark.parametrize("kernel", ["auto", "generic"])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_decode_infeasible_backtrack(gpu, kernel, dtype):
    """viterbi::decode (CV_ASSOC_DECODE) on infeasible sequences follows bt from argmax 0
    (viterbi.rs:19-30), on the f64 trellis (backtrack_f64) and the generic kernel, f32 and f64:
    the hand-worked case of test_oracle.py plus random ones, all equal to the oracle."""
    if dtype == "f32" and kernel == "auto":
        pytest.skip("f32 DECODE always runs the generic kernel")
    pi = np.array([-0.3, -0.3])
    a = np.array([[-1.0, -0.5], [-0.25, -2.0]])
    b = np.array([[-0.5, -1.0, -np.inf], [-1.0, -0.5, -np.inf]])
    h = cv.HMM(pi, a, b)
    p, s, st = cv.decode_batch(h, [0, 3], np.array([0, 0, 2], np.int32), dtype=dtype, assoc="decode",
                               kernel=kernel, rescore_f64=False)
    assert st[0] == 1 and s[0] == -np.inf and p.tolist() == [1, 0, 0]
    rng = np.random.default_rng(5)
    for n in (3, 64, 130, 256):
        pi, a, b = synth.random_hmm(n, 6, seed=n, zero_frac=0.3)
        b[:, 5] = -np.inf  # observation 5: infeasible wherever it occurs
        lengths = rng.integers(1, 40, size=30)
        off = synth.offsets_from_lengths(lengths)
        obs = rng.integers(0, 6, size=int(off[-1])).astype(np.int32)
        h = cv.HMM(pi, a, b)
        got = cv.decode_batch(h, off, obs, dtype=dtype, assoc="decode", kernel=kernel, rescore_f64=False)
        ref = O.decode_batch(pi, a, b, off, obs, O.DECODE, np.float64 if dtype == "f64" else np.float32)
        assert (ref[2] == 1).sum() > 5
        _assert_same(got, ref, f"decode infeasible N={n} {kernel} {dtype}")


@pytest.mark.parametrize("n", [45, 256])
@pytest.mark.parametrize("serial", [False, True])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp"])
def test_t64_matches_generic_f64_large(gpu, n, serial, assoc):
    """Batches large enough for 8 sequences per wave and several chunks (workspace cap),
    ragged lengths (longest-first schedule): identical to the generic f64 kernel, whose
    inline first-argmax is itself bit-exact against the oracle (test_gpu_parity.py)."""
    pi, a, b = synth.random_hmm(n, 200, seed=n + 9)
    rng = np.random.default_rng(n + 9)
    nseq = 20000
    lengths = rng.integers(1, 24, size=nseq)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, 200, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    per_elem = 2 * n if assoc == "cp" else 8 * 64 * ((n + 63) // 64)  # u16 psi row / f64 delta row
    ws = int(off[-1]) * per_elem // 3  # >= 3 chunks
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False, workspace_bytes=ws,
                          serial=serial)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["launches"] >= 3, t
    gen = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, kernel="generic", rescore_f64=False)
    _assert_same(got, gen, f"t64 vs generic {assoc} N={n}")
    # spot-check against the oracle
    idx = rng.choice(nseq, 24, replace=False)
    for k in idx:
        lo, hi = off[k], off[k + 1]
        rp, rs, rst = O.decode_batch(pi, a, b, np.array([0, hi - lo]), obs[lo:hi], ASSOC[assoc], np.float64)
        assert rst[0] == got[2][k] and rs[0] == got[1][k] and np.array_equal(rp, got[0][lo:hi])


def test_t64_config4_shape_sample(gpu):
    """Config-4 shape (N=256, V=1,024, T=512) on 512 sequences (S=2 per wave): bit-exact vs
    the f64 oracle on a sample, and the f32 trellis differs from the f64 reference on some
    paths (why the exact kernel exists) while agreeing where both are exact."""
    pi, a, b = synth.random_hmm(256, 1024, seed=20261015)
    nseq, T = 512, 512
    off = np.arange(nseq + 1, dtype=np.int64) * T
    obs = synth.iid_obs(1024, nseq * T, 20261015)
    h = cv.HMM(pi, a, b)
    p64, s64, st64 = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    sample = np.arange(0, nseq, 64)
    for k in sample:
        lo, hi = off[k], off[k + 1]
        rp, rs, rst = O.decode_batch(pi, a, b, np.array([0, T]), obs[lo:hi], O.VITERBI, np.float64)
        assert rst[0] == st64[k] and rs[0] == s64[k] and np.array_equal(rp, p64[lo:hi]), f"seq {k}"
    p32, s32, _ = cv.decode_batch(h, off, obs, dtype="f32", rescore_f64=True)
    same = np.array([np.array_equal(p32[off[k]:off[k + 1]], p64[off[k]:off[k + 1]]) for k in range(nseq)])
    # where the f32 path equals the f64 one, the f64 re-score equals the f64 decode's score exactly
    assert np.array_equal(s32[same], s64[same])
    # the f32 trellis is bit-exact against the f32 oracle (test_gpu_parity.py), so this count is a
    # property of the inputs, not of the kernels: measured on MI355X and pinned here
    ndiff = int((~same).sum())
    print(f"f32/f64 path disagreement: {ndiff}/{nseq} sequences")
    assert ndiff == F32_F64_DIFF_C4_512, ndiff
    # where they differ, the f64 path scores at least as high in f64 (it is the f64 optimum)
    assert np.all(s64[~same] >= s32[~same])


F32_F64_DIFF_C4_512 = 19  # measured on MI355X (profiles/r02_pytest_f64.log): 3.7% of these paths


def test_t64_config4_full_batch_vs_generic(gpu):
    """The bench's headline mode on the FULL config-4 batch (65,536 sequences, N=256, T=512):
    every path, score and status of the default f64 decode (trellis_fwd_f64 + backtrack_f64) is
    identical to the generic f64 kernel (inline first-argmax, an independent implementation
    that is itself bit-exact against the oracle), and a 16-sequence sample matches the f64
    oracle (the reference recurrence, viterbi.rs:13-18 in f64)."""
    c = synth.config("c4")
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b.reshape(256, 32, 32))
    p64, s64, st64 = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    assert np.all(st64 == 0)
    pg, sg, stg = cv.decode_batch(h, off, obs, dtype="f64", kernel="generic", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "generic"
    _assert_same((p64, s64, st64), (pg, sg, stg), "config 4 full batch: t64 vs generic f64")
    T = 512
    for k in np.linspace(0, len(off) - 2, 16).astype(int):
        lo, hi = off[k], off[k + 1]
        rp, rs, rst = O.decode_batch(pi, a, b, np.array([0, T]), obs[lo:hi], O.VITERBI, np.float64)
        assert rst[0] == st64[k] and rs[0] == s64[k] and np.array_equal(rp, p64[lo:hi]), f"seq {k}"


def test_t64_concurrent_handles_two_streams(gpu):
    """Two handles decode different N = 256 batches on two streams at once (their forward
    kernels co-run and share the process-global SIMD-balancing table, trellis64.hip
    g_t64_simd): each result is bit-identical to the same decode run alone."""
    import torch

    dev = torch.device("cuda:0")
    runs = []
    for seed, nseq, T in ((81, 8192, 48), (82, 6144, 64)):
        pi, a, b = synth.random_hmm(256, 64, seed=seed)
        off = np.arange(nseq + 1, dtype=np.int64) * T
        obs = np.random.default_rng(seed).integers(0, 64, size=nseq * T).astype(np.int32)
        h = cv.HMM(pi, a, b)
        bufs = (torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev),
                torch.empty(nseq * T, dtype=torch.int32, device=dev), torch.empty(nseq, dtype=torch.float64, device=dev),
                torch.empty(nseq, dtype=torch.uint8, device=dev))
        runs.append((h, off, bufs, torch.cuda.Stream(dev)))

    def launch(r):
        h, off, (o_d, ob_d, p_d, s_d, st_d), s = r
        cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=s.cuda_stream, dtype="f64",
                               rescore_f64=False)

    def result(r):
        return tuple(x.cpu().numpy().copy() for x in r[2][2:])

    solo = []
    for r in runs:
        launch(r)
        torch.cuda.synchronize()
        assert cv.last_timing(r[0])["kernel"] == "trellis_f64"
        solo.append(result(r))
    for _ in range(3):
        for r in runs:
            r[2][2].fill_(-1)
        for r in runs:  # both enqueued before either finishes
            launch(r)
        torch.cuda.synchronize()
        for r, ref in zip(runs, solo):
            _assert_same(result(r), ref, "concurrent decode")


def test_timing_sums_every_call(gpu):
    """cv_timing_begin / cv_timing_end: the device times of every decode call in between,
    with no synchronisation per call (what bench.py's timed loop reads)."""
    pi, a, b, off, obs = _case(64, 30, seed=5, nseq=200, tmax=60)
    h = cv.HMM(pi, a, b)
    cv.decode_batch(h, off, obs, rescore_f64=False)
    one = cv.last_timing(h)
    cv.timing_begin(h)
    for _ in range(3):
        cv.decode_batch(h, off, obs, rescore_f64=False)
    t = cv.timing_end(h)
    assert t["launches"] == 3 * one["launches"] and t["fwd_ms"] > 0 and t["bt_ms"] > 0
    assert t["total_ms"] >= t["fwd_ms"] / 3
    # last_timing still describes the last call alone
    assert cv.last_timing(h)["launches"] == one["launches"]
    with pytest.raises(cv.CVError):
        cv.timing_end(h)  # no timing_begin pending


@pytest.mark.parametrize("s", ["1", "2", "4"])
@pytest.mark.parametrize("n", [7, 100, 256])
def test_t64_cp_seqs_per_wave(gpu, monkeypatch, s, n):
    """trellis_cp_f64 at S = 1 (one sequence per wave: the default up to 1,024 sequences, the
    parallel chain's speculative batches), 2 and 4 (CV_T64_CP_S): CPSolver's association against
    the oracle on quantised ties (first index), -inf entries and ragged / empty sequences; the
    reported seqs_per_wave is the S launched."""
    monkeypatch.setenv("CV_T64_CP_S", s)
    rng = np.random.default_rng(n + 5)
    v = 9
    pi = np.round(rng.uniform(-2, 0, n) * 2) / 2
    a = np.round(rng.uniform(-2, 0, (n, n)) * 2) / 2
    b = np.round(rng.uniform(-2, 0, (n, v)) * 2) / 2
    a[rng.random((n, n)) < 0.2] = -np.inf
    b[:, 3] = -np.inf
    lengths = rng.integers(0, 70, size=37)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc="cp", rescore_f64=False)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["seqs_per_wave"] == int(s), t
    _assert_same(got, O.decode_batch(pi, a, b, off, obs, O.CP, np.float64), f"cp S={s} N={n}")
    pi2, a2, b2, off2, obs2 = _case(n, 41, seed=900 + n)
    h2 = cv.HMM(pi2, a2, b2)
    _assert_same(cv.decode_batch(h2, off2, obs2, dtype="f64", assoc="cp", rescore_f64=False),
                 O.decode_batch(pi2, a2, b2, off2, obs2, O.CP, np.float64), f"cp random S={s} N={n}")


@pytest.mark.parametrize("assoc", ["viterbi", "decode"])
@pytest.mark.parametrize("n", [5, 17, 33, 45, 48, 49])
def test_t64_wave48_vs_wave64_and_oracle(gpu, n, assoc):
    """N <= 48: trellis_wave48_f64 (48 states, 3 columns x 12 rows per lane, the four row groups'
    maxima through LDS, four waves per SIMD) == trellis_wave_f64 on 64 padded states (tuning key
    t64_wave = 2) == the oracle, bit for bit: ragged, empty and infeasible sequences, -inf
    transitions, viterbi::decode's row 0 = 0 (ZI).  N = 49 keeps the 64-state kernel."""
    pi, a, b = synth.random_hmm(n, 40, seed=480 + n, zero_frac=0.1)
    b = b.copy()
    b[:, 39] = -np.inf  # observation 39: no state emits it
    rng = np.random.default_rng(480 + n)
    lengths = rng.integers(0, 140, size=3000)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, 39, size=int(off[-1])).astype(np.int32)
    obs[rng.integers(0, len(obs), size=4)] = 39
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    with h.tuned(t64_wave=2):
        ref64 = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False)
    _assert_same(got, ref64, f"wave48 vs wave64 N={n} {assoc}")
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI if assoc == "viterbi" else O.DECODE, np.float64)
    _assert_same(got, ref, f"wave48 vs oracle N={n} {assoc}")
    assert np.any(got[2] == 1) and np.any(got[2] == 2)  # infeasible, empty


def test_release_workspaces(gpu):
    """cv_hmm_release_workspaces frees the grow-only decode workspaces (the parallel
    chain's ~0.4 GB of per-call buffers stayed for the handle's life); the next decode
    allocates again and returns the same bits."""
    c = synth.config("c4", 2048)
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    p0, o0 = cv.decode_superseq_cp(h, off, obs)
    ref = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    held = cv.device_memory()["current"]
    h.release_workspaces()
    after = cv.device_memory()["current"]
    assert after < held - 2048 * 512 * 256 * 8, (held, after)  # at least the delta rows went
    p1, o1 = cv.decode_superseq_cp(h, off, obs)
    assert o1 == o0 and np.array_equal(p1, p0)
    _assert_same(cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False), ref, "after release")
