"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): paths bit-exact and scores bit-exact in
the SAME precision and association; f64 re-scored log-likelihoods equal the oracle's f64
re-score of the same path exactly (tolerance 0; the north-star allows 1e-6 relative).
"""
import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth
from conftest import load_golden

pytestmark = pytest.mark.gpu

ASSOC = {"viterbi": O.VITERBI, "cp": O.CP, "dp": O.DP, "decode": O.DECODE}


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


@pytest.mark.parametrize("n", [1, 2, 5, 16, 31, 32, 33, 45, 64, 65, 96, 100, 128, 129, 160, 192, 200, 224, 255, 256])
def test_trellis_f32_bit_exact(gpu, n):
    pi, a, b, off, obs = _case(n, 37, seed=n, zero_frac=0.05 if n % 2 else 0.0)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f32", kernel="trellis", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "trellis"
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32)
    _assert_same(got, ref, f"trellis N={n}")
    # f64 re-score along the decoded path == oracle's f64 re-score, exactly
    path, score, status = cv.decode_batch(h, off, obs, dtype="f32", kernel="trellis", rescore_f64=True)
    for s in range(len(off) - 1):
        if status[s] == 0:
            lo, hi = off[s], off[s + 1]
            assert score[s] == O.rescore_f64(pi, a, b, obs[lo:hi], path[lo:hi])


@pytest.mark.parametrize("n", [40, 64, 100, 128, 160, 200, 224, 256])
@pytest.mark.parametrize("variant", ["valu", "valu1"])
@pytest.mark.parametrize("serial", [False, True])
def test_trellis_variants_bit_exact(gpu, n, variant, serial):
    """Both f32 trellis variants (2 or 1 sequences per workgroup) and both schedules
    (pipelined chunks / serial) give the oracle's f32 result bit for bit."""
    pi, a, b, off, obs = _case(n, 29, seed=300 + n, nseq=30, tmax=50, zero_frac=0.03)
    h = cv.HMM(pi, a, b)
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32)
    got = cv.decode_batch(h, off, obs, rescore_f64=False, variant=variant, serial=serial,
                          workspace_bytes=0 if serial else 256 * 4 * 300, dtype="f32")
    assert cv.last_timing(h)["kernel"] == "trellis"
    _assert_same(got, ref, f"{variant} N={n} serial={serial}")


@pytest.mark.parametrize("n", [45, 64, 128, 192, 256])
@pytest.mark.parametrize("serial", [False, True])
def test_pair_kernel_equal_and_ragged(gpu, n, serial):
    """Two sequences per workgroup (trellis_fwd2_f32): lengths from a small set so most
    sequences pair with an equal-length neighbour, an odd leftover per length, T = 1 and 2
    (no or one step), zeros in A -- bit-identical to the oracle and to one per workgroup."""
    pi, a, b = synth.random_hmm(n, 23, seed=n, zero_frac=0.02)
    rng = np.random.default_rng(n)
    off = synth.offsets_from_lengths(rng.choice([1, 2, 3, 17, 64], size=37))
    obs = rng.integers(0, 23, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32)
    ws = 0 if serial else n * 4 * 400
    for variant in ("valu", "valu1"):
        got = cv.decode_batch(h, off, obs, rescore_f64=False, variant=variant, serial=serial, workspace_bytes=ws, dtype="f32")
        _assert_same(got, ref, f"{variant} N={n} serial={serial}")
    # equal lengths, odd count: pairs (2k, 2k+1) straight from the CSR order, one single
    off2 = synth.offsets_from_lengths(np.full(9, 33))
    obs2 = rng.integers(0, 23, size=int(off2[-1])).astype(np.int32)
    ref2 = O.decode_batch(pi, a, b, off2, obs2, O.VITERBI, np.float32)
    _assert_same(cv.decode_batch(h, off2, obs2, rescore_f64=False, serial=serial, dtype="f32"), ref2, f"equal N={n}")


@pytest.mark.parametrize("n", [1, 5, 16, 17, 31, 32, 33, 45, 48, 49, 64])
@pytest.mark.parametrize("serial", [False, True])
def test_wave_kernel_small_n(gpu, n, serial):
    """N <= 64: one wave per sequence with the backtrack fused (trellis_wave_f32, tables
    padded to 16/32/48/64 states): ragged lengths incl. T = 0 and 1, -inf entries, a chunked
    workspace -- bit-identical to the oracle and to the workgroup kernels."""
    pi, a, b = synth.random_hmm(n, 17, seed=2000 + n, zero_frac=0.03)
    rng = np.random.default_rng(n + 11)
    off = synth.offsets_from_lengths(rng.choice([0, 1, 2, 7, 40, 129, 300], size=53))
    obs = rng.integers(0, 17, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32)
    ws = 0 if serial else 64 * 4 * 700
    got = cv.decode_batch(h, off, obs, rescore_f64=False, serial=serial, workspace_bytes=ws, dtype="f32")
    assert cv.last_timing(h)["padded_states"] == (n + 15) // 16 * 16
    _assert_same(got, ref, f"wave N={n}")
    other = cv.decode_batch(h, off, obs, rescore_f64=False, variant="nowave", serial=serial, workspace_bytes=ws, dtype="f32")
    _assert_same(got, other, f"wave vs workgroup N={n}")
    # f64 re-score along the path
    path, score, status = cv.decode_batch(h, off, obs, rescore_f64=True, serial=serial, workspace_bytes=ws, dtype="f32")
    for s in range(len(off) - 1):
        if status[s] == 0:
            lo, hi = off[s], off[s + 1]
            assert score[s] == O.rescore_f64(pi, a, b, obs[lo:hi], path[lo:hi])


def test_retired_mfma_flags_rejected(gpu):
    """The MFMA-assisted f32 trellis was retired (slower than the all-VALU one, DESIGN.md
    §3): its flag bits are reserved and rejected."""
    import ctypes
    from cviterbi import _lib as L
    from cviterbi.decode import make_opts
    pi, a, b, off, obs = _case(64, 9, seed=1, nseq=2, tmax=5)
    h = cv.HMM(pi, a, b)
    for flags in (0x1, 7 << 8):
        o = make_opts("f32")
        o.flags = flags
        path, score, status = np.zeros(int(off[-1]), np.int32), np.zeros(2), np.zeros(2, np.uint8)
        st = L.lib().cv_decode_batch(h.handle, 2, off.ctypes.data_as(ctypes.c_void_p),
                                     np.ascontiguousarray(obs, np.int32).ctypes.data_as(ctypes.c_void_p),
                                     ctypes.byref(o), path.ctypes.data_as(ctypes.c_void_p),
                                     score.ctypes.data_as(ctypes.c_void_p), status.ctypes.data_as(ctypes.c_void_p))
        assert st == L.CV_EUNSUPPORTED


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp", "decode"])
@pytest.mark.parametrize("n", [3, 45, 64, 300])
def test_generic_all_modes(gpu, dtype, assoc, n):
    pi, a, b, off, obs = _case(n, 23, seed=1000 + n, nseq=8, tmax=40, zero_frac=0.15)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype=dtype, assoc=assoc, kernel="generic", rescore_f64=False)
    ref = O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], np.float32 if dtype == "f32" else np.float64)
    _assert_same(got, ref, f"generic {dtype} {assoc} N={n}")


@pytest.mark.parametrize("name", ["golden_small.npz", "golden_ties.npz", "golden_inf.npz", "golden_ar_house_a.npz"])
def test_golden_fixtures(gpu, name):
    g = load_golden(name)
    h = cv.HMM(g["pi"], g["a"], g["b"])
    for dt, key in (("f32", "f32"), ("f64", "f64")):
        for assoc in ("viterbi", "cp", "dp", "decode"):
            k = f"{key}_{assoc}"
            if k + "_path" not in g:
                continue
            got = cv.decode_batch(h, g["offsets"], g["obs"], dtype=dt, assoc=assoc, rescore_f64=False)
            ref = (g[k + "_path"], g[k + "_score"], g[k + "_status"])
            _assert_same(got, ref, f"{name} {k}")


def test_edge_cases(gpu):
    n, v = 8, 6
    pi, a, b = synth.random_hmm(n, v, seed=3)
    b[:, 5] = -np.inf  # observation 5 cannot be emitted -> infeasible sequences
    lengths = np.array([0, 1, 1, 2, 0, 9, 3, 64, 65, 129])
    off = synth.offsets_from_lengths(lengths)
    rng = np.random.default_rng(0)
    obs = rng.integers(0, 5, size=int(off[-1])).astype(np.int32)
    obs[off[6] + 1] = 5  # sequence 6 infeasible
    h = cv.HMM(pi, a, b)
    for kernel, dt in (("trellis", "f32"), ("generic", "f32"), ("generic", "f64")):
        got = cv.decode_batch(h, off, obs, dtype=dt, kernel=kernel, rescore_f64=False)
        ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32 if dt == "f32" else np.float64)
        _assert_same(got, ref, f"edge {kernel} {dt}")
        assert got[2][0] == cv._lib.SEQ_EMPTY and got[2][6] == cv._lib.SEQ_INFEASIBLE


def test_ties_first_index(gpu):
    """Dyadic (exactly representable) log-probs: every add is exact, ties everywhere."""
    g = load_golden("golden_ties.npz")
    h = cv.HMM(g["pi"], g["a"], g["b"])
    got = cv.decode_batch(h, g["offsets"], g["obs"], dtype="f32", kernel="trellis", rescore_f64=False)
    _assert_same(got, (g["f32_viterbi_path"], g["f32_viterbi_score"], g["f32_viterbi_status"]), "ties")


def test_chunked_workspace(gpu):
    pi, a, b, off, obs = _case(64, 40, seed=5, nseq=40, tmax=90)
    h = cv.HMM(pi, a, b)
    full = cv.decode_batch(h, off, obs, rescore_f64=False, dtype="f32")
    small = cv.decode_batch(h, off, obs, rescore_f64=False, workspace_bytes=64 * 4 * 200, dtype="f32")
    assert cv.last_timing(h)["launches"] > 1
    for x, y in zip(full, small):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("n", [32, 64, 256])
def test_device_api_badobs(gpu, n):
    import torch

    pi, a, b, off, obs = _case(n, 10, seed=9, nseq=6, tmax=30, tmin=5)
    obs = obs.copy()
    obs[off[2] + 3] = 10  # out of range on the device path
    h = cv.HMM(pi, a, b)
    dev = torch.device("cuda:0")
    o_d = torch.from_numpy(off).to(dev)
    ob_d = torch.from_numpy(obs).to(dev)
    p_d = torch.zeros(int(off[-1]), dtype=torch.int32, device=dev)
    s_d = torch.zeros(len(off) - 1, dtype=torch.float64, device=dev)
    st_d = torch.zeros(len(off) - 1, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream, dtype="f32")
    torch.cuda.synchronize()
    st = st_d.cpu().numpy()
    assert st[2] == cv._lib.SEQ_BADOBS
    assert (np.delete(st, 2) == 0).all()
    # host API rejects it up front
    with pytest.raises(cv.CVError):
        cv.decode_batch(h, off, obs, dtype="f32")


@pytest.mark.parametrize("cfg,nseq", [("c2", 256), ("c3", 24), ("c4", 48)])
def test_config_subsets_bit_exact(gpu, cfg, nseq):
    c = synth.config(cfg, nseq=nseq)
    h = cv.HMM(c["pi"], c["a"], c["b"])
    got = cv.decode_batch(h, c["offsets"], c["obs"], rescore_f64=False, dtype="f32")
    ref = O.decode_batch(c["pi"], c["a"], c["b"], c["offsets"], c["obs"], O.VITERBI, np.float32, nthreads=8)
    _assert_same(got, ref, cfg)


def test_config4_full_properties(gpu):
    """Full config 4 (N=256, T=512, B=65,536): size-independent properties + a sampled
    bit-exact check.  (1) every path is in range and feasible; (2) the kernel's f32 score
    equals the f32 row-A0 score of the returned path (sequential f32 adds, exact); (3) the
    f64 re-score equals numpy's f64 re-score of the same path; (4) 16 sampled sequences
    match the oracle bit-exactly."""
    c = synth.config("c4")
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    path, s32, st = cv.decode_batch(h, off, obs, rescore_f64=False, dtype="f32")
    assert (st == 0).all()
    assert path.min() >= 0 and path.max() < 256
    B, T = len(off) - 1, 512
    P = path.reshape(B, T)
    Ob = obs.reshape(B, T)
    for dt, ref_score in ((np.float32, s32), (np.float64, None)):
        A_, B_, pi_ = a.astype(dt), b.astype(dt), pi.astype(dt)
        d = pi_[P[:, 0]] + B_[P[:, 0], Ob[:, 0]]
        for t in range(1, T):
            d = d + A_[P[:, t - 1], P[:, t]]
            d = d + B_[P[:, t], Ob[:, t]]
        if dt == np.float32:
            assert np.array_equal(d.astype(np.float64), ref_score)
        else:
            _, s64, _ = cv.decode_batch(h, off, obs, rescore_f64=True, dtype="f32")
            assert np.array_equal(d, s64)
    rng = np.random.default_rng(1)
    pick = np.sort(rng.choice(B, size=16, replace=False))
    sub_off = np.arange(17, dtype=np.int64) * T
    sub_obs = Ob[pick].reshape(-1)
    rp, rs, rst = O.decode_batch(pi, a, b, sub_off, sub_obs, O.VITERBI, np.float32, nthreads=8)
    assert np.array_equal(P[pick].reshape(-1), rp)
    assert np.array_equal(s32[pick], rs)


def test_solver_api(gpu):
    pi, a, b = synth.random_hmm(12, 20, seed=4)
    rng = np.random.default_rng(4)
    seqs = [[int(x) for x in rng.integers(0, 20, size=int(t))] for t in rng.integers(1, 30, size=9)]
    h = cv.HMM(pi, a, b)
    ss = cv.SuperSequence(seqs, None, h)
    ss.recompute_constraints(0.0)  # main.rs:107 -> reorder (utils.rs:138-165)
    for kind, assoc, dt in (("gpu", O.VITERBI, np.float32), ("gpu-f64", O.VITERBI, np.float64),
                            ("gpu-cp-seq", O.CP, np.float64), ("gpu-dp", O.DP, np.float64), ("gpu-cp", None, None)):
        s = cv.GpuSolver(h, ss, kind)
        s.solve()
        sol = s.get_solution()
        assert s.get_name() == kind and s.get_explored_nodes() == 0
        offsets, obs, _ = ss.sequence_blocks()
        if kind == "gpu-cp":  # CPSolver exactly: the chained super-sequence, path and objective bits
            rp, robj = O.cp_superseq_f64(pi, a, b, offsets, obs)
            assert np.array_equal(sol, rp) and s.get_objective() == robj
            continue
        rp, rs, _ = O.decode_batch(pi, a, b, offsets, obs, assoc, dt)
        assert np.array_equal(sol, rp)
        if kind == "gpu":
            exp = sum(O.rescore_f64(pi, a, b, obs[offsets[k]:offsets[k + 1]], rp[offsets[k]:offsets[k + 1]])
                      for k in range(len(offsets) - 1))
        else:
            exp = float(np.sum(rs))
        assert s.get_objective() == pytest.approx(exp, rel=1e-12)
        per_seq = ss.parse_solution(sol)
        assert [len(x) for x in per_seq] == [len(x) for x in seqs]


def test_long_sequence_large_alphabet(gpu):
    """Maximum-size corner: N = 256, a 40,000-step sequence next to short ones, V = 200,000
    observations (800 MB emission image) -- bit-exact vs the oracle, also with a workspace
    cap below the long sequence's delta rows (a chunk never splits a sequence: it gets a
    chunk of its own, the short ones others)."""
    n, v = 256, 200_000
    pi, a, b = synth.random_hmm(n, 64, seed=31)
    rng = np.random.default_rng(31)
    b = np.repeat(b, v // 64, axis=1)[:, :v] + rng.normal(0, 0.01, size=(n, v))  # log10, distinct values
    off = synth.offsets_from_lengths(np.array([3, 40_000, 1, 17]))
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32, nthreads=4)
    _assert_same(cv.decode_batch(h, off, obs, rescore_f64=False, dtype="f32"), ref, "long")
    _assert_same(cv.decode_batch(h, off, obs, rescore_f64=False, workspace_bytes=256 * 4 * 9000, dtype="f32"), ref, "long, capped")
