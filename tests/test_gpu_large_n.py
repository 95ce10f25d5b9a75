"""GPU: models beyond the padded kernels' N <= 256: the generic decode with its rows in LDS
(two rows of N in <= 160 KiB: N <= 10,240 in f64, 20,480 in f32) and wide above that (each step
over many workgroups, the rows in global memory, up to the u16 back-pointers' N <= 65,535), the
same for the serial super-sequence chain.  The reference has no state limit (hmm.rs:10-18 stores
any N; viterbi.rs:5-32, cp.rs:63-93 loop over it); every case is checked against the C oracle
bit for bit.
"""
import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu


def _case(n, v, seed, lengths):
    rng = np.random.default_rng(seed)
    pi = np.log10(rng.dirichlet(np.ones(n)))
    a = rng.uniform(-4.0, 0.0, (n, n))
    b = rng.uniform(-3.0, 0.0, (n, v))
    a[rng.random((n, n)) < 0.05] = -np.inf
    off = synth.offsets_from_lengths(np.asarray(lengths))
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    return pi, a, b, off, obs


@pytest.mark.parametrize("dtype,n", [("f64", 4200), ("f64", 10240), ("f32", 8300)])
def test_generic_decode_beyond_64k_lds(gpu, monkeypatch, dtype, n):
    """The generic kernel's two rows above 64 KiB of LDS (the launch raises the limit; the wide
    decode, the default at these N, off: CV_GENERIC_WIDE=0)."""
    monkeypatch.setenv("CV_GENERIC_WIDE", "0")
    pi, a, b, off, obs = _case(n, 5, seed=n, lengths=[3, 0, 4] if n > 5000 else [5, 1, 6])
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype=dtype, assoc="viterbi", rescore_f64=False)
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32 if dtype == "f32" else np.float64)
    assert np.array_equal(got[2], ref[2])
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0], ref[0])


@pytest.mark.parametrize("dtype,n,assocs", [("f64", 10241, ("viterbi", "cp", "dp", "decode", "forced")),
                                            ("f32", 20481, ("viterbi", "cp"))])
def test_generic_decode_beyond_lds(gpu, dtype, n, assocs):
    """One state past the LDS-resident rows (2 N REAL > 160 KiB): the wide generic decode (each
    step one launch, the states over workgroups, the rows in global memory) against the oracle,
    incl. an empty sequence, a one-element sequence and forced states."""
    pi, a, b, off, obs = _case(n, 4, seed=n, lengths=[3, 0, 2, 1])
    h = cv.HMM(pi, a, b)
    dt = np.float32 if dtype == "f32" else np.float64
    ASSOC = {"viterbi": O.VITERBI, "cp": O.CP, "dp": O.DP, "decode": O.DECODE, "forced": O.VITERBI}
    for assoc in assocs:
        fr = np.array([-1, n - 1, -1, 5, -1, -1], np.int32) if assoc == "forced" else None
        got = cv.decode_batch(h, off, obs, dtype=dtype, assoc="viterbi" if fr is not None else assoc,
                              rescore_f64=False, forced=fr)
        t = cv.last_timing(h)
        assert t["kernel"] == "generic" and t["seqs_per_wave"] == 0, t
        ref = O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], dt, forced=fr)
        assert np.array_equal(got[2], ref[2]), assoc
        ok = got[2] == 0
        assert np.array_equal(got[1][ok], ref[1][ok]), assoc
        assert np.array_equal(got[0], ref[0]), assoc


@pytest.mark.parametrize("S", ["1", "2", "4"])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp", "decode", "forced"])
@pytest.mark.parametrize("dtype,n", [("f64", 300), ("f32", 300), ("f64", 1100)])
def test_generic_wide_vs_oracle(gpu, monkeypatch, S, assoc, dtype, n):
    """The wide generic decode at small N (CV_GENERIC_WIDE_MIN=1), S slots per workgroup
    (CV_WIDE_S; ragged groups with finished and empty slots): ragged and empty sequences, -inf
    transitions and emissions, forced states, every association -- the oracle bit for bit."""
    monkeypatch.setenv("CV_GENERIC_WIDE_MIN", "1")
    monkeypatch.setenv("CV_WIDE_S", S)
    pi, a, b = synth.random_hmm(n, 11, seed=n + 55, zero_frac=0.1)
    rng = np.random.default_rng(n + 55)
    lens = rng.integers(1, 20, size=19)
    lens[[4, 9]] = 0
    lens[6] = 1
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 11, size=int(off[-1])).astype(np.int32)
    fr = None
    if assoc == "forced":
        fr = np.where(rng.random(len(obs)) < 0.08, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    ak = "viterbi" if assoc == "forced" else assoc
    dt = np.float32 if dtype == "f32" else np.float64
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype=dtype, assoc=ak, kernel="generic", rescore_f64=False, forced=fr)
    t = cv.last_timing(h)
    assert t["kernel"] == "generic" and t["seqs_per_wave"] == 0, t
    ref = O.decode_batch(pi, a, b, off, obs, {"viterbi": O.VITERBI, "cp": O.CP, "dp": O.DP, "decode": O.DECODE}[ak],
                         dt, forced=fr)
    assert np.array_equal(got[2], ref[2])
    ok = got[2] == 0
    assert np.array_equal(got[1][ok], ref[1][ok])
    assert np.array_equal(got[0], ref[0])


def test_superseq_chain_wide_beyond_lds(gpu):
    """The serial super-sequence chain one state past its LDS-resident rows (N = 10,241: the
    wide chain, then the segmented backtrack) against the chained restatement."""
    n, v = 10241, 3
    rng = np.random.default_rng(10241)
    pi = np.round(rng.uniform(-2, 0, n) * 4) / 4
    a = np.round(rng.uniform(-2, 0, (n, n)) * 4) / 4
    b = np.round(rng.uniform(-2, 0, (n, v)) * 4) / 4
    off = synth.offsets_from_lengths(np.asarray([2, 0, 1, 2]))
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    path, obj = cv.decode_superseq_cp(h, off, obs)
    assert not cv.last_superseq_stats(h)["parallel"]
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj
    assert np.array_equal(path, rp)


@pytest.mark.parametrize("wide", ["0", "1"])
@pytest.mark.parametrize("n", [300, 1100, 2500])
def test_superseq_chain_strided_states(gpu, monkeypatch, n, wide):
    """cp_superseq_chain with N > 256 (and > 1,024: states strided over the workgroup's 1,024
    threads), every element and the objective against the chained restatement; wide = "1": the
    serial chain as the wide kernels (CV_CHAIN_WIDE_MIN=1, CV_CHAIN_PAR=0)."""
    if wide == "1":
        monkeypatch.setenv("CV_CHAIN_WIDE_MIN", "1")
        monkeypatch.setenv("CV_CHAIN_PAR", "0")
    else:  # the one-workgroup chain (states strided above 1,024 threads; wide is the default there)
        monkeypatch.setenv("CV_CHAIN_WIDE", "0")
    rng = np.random.default_rng(70 + n)
    v = 7
    # quantised tables: exact ties, the first index must win in every strided slice
    pi = np.round(rng.uniform(-2, 0, n) * 4) / 4
    a = np.round(rng.uniform(-2, 0, (n, n)) * 4) / 4
    b = np.round(rng.uniform(-2, 0, (n, v)) * 4) / 4
    a[rng.random((n, n)) < 0.1] = -np.inf
    lengths = [3, 0, 1, 5, 2] if n > 1024 else [6, 0, 1, 9, 4, 3]
    off = synth.offsets_from_lengths(np.asarray(lengths))
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    path, obj = cv.decode_superseq_cp(h, off, obs)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj
    assert np.array_equal(path, rp)


def _constrained_case(n, seed, nseq=10, tmax=14, multi=True):
    """One- and several-position constrained sequences over N states: components 0..3 when
    every sequence has one position; 0..1 with several (the oracle's exhaustive search runs
    over N^(components coupled by pairs))."""
    pi, a, b = synth.random_hmm(n, 9, seed=seed, zero_frac=0.05)
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, tmax, size=nseq)
    lens[:3] = [1, 2, tmax]
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 9, size=int(off[-1])).astype(np.int32)
    comp = np.full(len(obs), -1, np.int32)
    for s in range(nseq):
        if rng.random() < 0.8:
            k = int(rng.integers(1, 4)) if multi else 1
            pos = rng.choice(lens[s], size=min(k, lens[s]), replace=False)
            comp[off[s] + pos] = rng.integers(0, 2 if multi else 4, size=len(pos))
    comp[off[2]:off[3]] = -1
    comp[off[0]] = 0                 # t_1 = first element (length-1 sequence)
    comp[off[2] + lens[2] - 1] = 1   # t_1 = last element
    return pi, a, b, off, obs, comp


@pytest.mark.parametrize("S", ["1", "4"])
@pytest.mark.parametrize("n,multi", [(257, True), (300, False), (400, True), (520, False)])
def test_constrained_f64_beyond_256(gpu, monkeypatch, S, n, multi):
    """The constrained decode at N > 256 (generic_ext terms passes + segment tables with S
    slots per workgroup, CV_GENERIC_S; host exact sums; the forced decode) against the oracle
    spec (np_oracle.constrained_decode): the component states, paths and f64 scores bit for
    bit, every active element on its state."""
    monkeypatch.setenv("CV_GENERIC_S", S)
    pi, a, b, off, obs, comp = _constrained_case(n, seed=n, multi=multi)
    h = cv.HMM(pi, a, b)
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, dtype="f64")
    ref_states, forced = O.constrained_forced(pi, a, b, off, obs, comp, np.float64)
    for c, s in ref_states.items():
        assert states[c] == s, (c, states[c], s)
    rp, rs, rst = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, forced=forced)
    assert np.array_equal(status, rst)
    assert np.array_equal(path, rp)
    assert np.array_equal(score[status == 0], rs[status == 0])
    for e in np.nonzero(comp >= 0)[0]:
        assert path[e] == states[comp[e]]
    assert obj == pytest.approx(float(np.sum(score)), rel=1e-12)


@pytest.mark.parametrize("n,multi", [(257, True), (400, True), (520, False)])
def test_constrained_f64_wide(gpu, monkeypatch, n, multi):
    """The constrained decode with the wide kernels (what runs above N = 10,240): the terms
    passes and segment tables through generic_ext's wide step (CV_EXT_WIDE_MIN=1), the final
    forced decode through the wide generic decode (CV_GENERIC_WIDE_MIN=1) -- the oracle spec."""
    monkeypatch.setenv("CV_EXT_WIDE_MIN", "1")
    monkeypatch.setenv("CV_GENERIC_WIDE_MIN", "1")
    pi, a, b, off, obs, comp = _constrained_case(n, seed=n + 7, multi=multi)
    h = cv.HMM(pi, a, b)
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, dtype="f64")
    ref_states, forced = O.constrained_forced(pi, a, b, off, obs, comp, np.float64)
    for c, s in ref_states.items():
        assert states[c] == s, (c, states[c], s)
    rp, rs, rst = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, forced=forced)
    assert np.array_equal(status, rst)
    assert np.array_equal(path, rp)
    assert np.array_equal(score[status == 0], rs[status == 0])


def test_constrained_f64_beyond_lds(gpu):
    """One state past the LDS-resident rows (N = 10,241): the constrained decode's terms passes
    wide, one-position sequences (the oracle's C max-marginal), the oracle spec bit for bit."""
    n = 10241
    rng = np.random.default_rng(n)
    pi = np.log10(rng.dirichlet(np.ones(n)))
    a = rng.uniform(-4.0, 0.0, (n, n))
    b = rng.uniform(-3.0, 0.0, (n, 5))
    a[rng.random((n, n)) < 0.05] = -np.inf
    lens = np.array([3, 1, 4, 2])
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 5, size=int(off[-1])).astype(np.int32)
    comp = np.full(len(obs), -1, np.int32)
    comp[[0, 3, 6, 8]] = [0, 1, 0, 1]  # one position each: t = 0, the one-element sequence, t = 2, t = 0
    h = cv.HMM(pi, a, b)
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, dtype="f64")
    ref_states, forced = O.constrained_forced(pi, a, b, off, obs, comp, np.float64)
    for c, s in ref_states.items():
        assert states[c] == s, (c, states[c], s)
    rp, rs, rst = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, forced=forced)
    assert np.array_equal(status, rst)
    assert np.array_equal(path, rp)
    assert np.array_equal(score[status == 0], rs[status == 0])


def test_constrained_device_and_sharded_beyond_256(gpu):
    """The device API and the sharded partials (integer SUM over shards) at N = 300 equal the
    host API's result."""
    import torch
    pi, a, b, off, obs, comp = _constrained_case(300, seed=31)
    h = cv.HMM(pi, a, b)
    ref = cv.decode_constrained(h, off, obs, comp, ncomp=4, dtype="f64")
    dev = torch.device("cuda", 0)
    path_d = torch.empty(int(off[-1]), dtype=torch.int32, device=dev)
    score_d = torch.empty(len(off) - 1, dtype=torch.float64, device=dev)
    status_d = torch.empty(len(off) - 1, dtype=torch.uint8, device=dev)
    states, obj = cv.decode_constrained_device(h, off, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev),
                                               comp, path_d, score_d, status_d, ncomp=4, dtype="f64")
    assert np.array_equal(states, ref[3])
    assert np.array_equal(path_d.cpu().numpy(), ref[0])
    assert np.array_equal(score_d.cpu().numpy(), ref[1])
    assert np.array_equal(status_d.cpu().numpy(), ref[2])
    assert obj == ref[4]
    from cviterbi import dist as cvdist
    pairs = cv.constrained_pairs(off, comp, 4)
    part = 0
    for s0, s1 in ((0, 4), (4, len(off) - 1)):
        lo, hi = off[s0], off[s1]
        part = part + cv.constrained_partials(h, cvdist.shard_offsets(off, s0, s1), obs[lo:hi], comp[lo:hi], 4, pairs,
                                              dtype="f64")
    got_states, _ = cv.constrained_select(300, 4, part, pairs)
    assert np.array_equal(got_states, ref[3])


@pytest.mark.parametrize("rows", ["1", "0"])
@pytest.mark.parametrize("S", ["1", "2", "4"])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp", "decode"])
@pytest.mark.parametrize("dtype,n", [("f64", 300), ("f32", 300), ("f64", 700), ("f64", 1100)])
def test_generic_multi_sequence_workgroups(gpu, monkeypatch, rows, S, assoc, dtype, n):
    """generic_fwd_ms (S sequences per workgroup, CV_GENERIC_S) in rows mode (the maximum
    only, argmax recomputed by generic_bt_rows; CV_GENERIC_ROWS=1, CP always psi) and psi
    mode against the oracle in every association: ragged and empty sequences in one
    workgroup, forced states, -inf transitions and emissions, N above 1,024 threads."""
    monkeypatch.setenv("CV_GENERIC_S", S)
    monkeypatch.setenv("CV_GENERIC_ROWS", rows)
    monkeypatch.setenv("CV_GENERIC_WIDE", "0")  # N = 1,100: the one-workgroup kernels, not wide
    pi, a, b = synth.random_hmm(n, 11, seed=n + 5, zero_frac=0.1)
    rng = np.random.default_rng(n + int(S))
    lens = rng.integers(1, 24, size=23)
    lens[[4, 9]] = 0
    lens[6] = 1
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 11, size=int(off[-1])).astype(np.int32)
    forced = np.where(rng.random(len(obs)) < 0.05, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    dt = np.float32 if dtype == "f32" else np.float64
    ASSOC = {"viterbi": O.VITERBI, "cp": O.CP, "dp": O.DP, "decode": O.DECODE}
    h = cv.HMM(pi, a, b)
    fr = forced if assoc == "viterbi" else None
    got = cv.decode_batch(h, off, obs, dtype=dtype, assoc=assoc, kernel="generic", rescore_f64=False, forced=fr)
    ref = O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], dt, forced=fr)
    assert np.array_equal(got[2], ref[2])
    ok = got[2] == 0
    assert np.array_equal(got[1][ok], ref[1][ok])
    assert np.array_equal(got[0], ref[0])


@pytest.mark.parametrize("rows", ["1", "0"])
@pytest.mark.parametrize("name", ["golden_ties.npz", "golden_inf.npz", "golden_small.npz"])
def test_generic_rows_golden(gpu, monkeypatch, rows, name):
    """The golden fixtures (exact ties everywhere, -inf entries and infeasible sequences incl.
    viterbi::decode's infeasible walk) through the generic kernels in both modes."""
    from conftest import load_golden
    monkeypatch.setenv("CV_GENERIC_ROWS", rows)
    g = load_golden(name)
    h = cv.HMM(g["pi"], g["a"], g["b"])
    seen = 0
    for dt in ("f32", "f64"):
        for assoc in ("viterbi", "cp", "dp", "decode"):
            k = f"{dt}_{assoc}"
            if k + "_path" not in g:
                continue
            got = cv.decode_batch(h, g["offsets"], g["obs"], dtype=dt, assoc=assoc, kernel="generic",
                                  rescore_f64=False)
            for x, y, what in zip(got, (g[k + "_path"], g[k + "_score"], g[k + "_status"]), ("path", "score", "status")):
                assert np.array_equal(x, y), (k, what)
            seen += 1
    assert seen > 0


@pytest.mark.parametrize("S", ["2", "4", "8"])
@pytest.mark.parametrize("assoc", ["viterbi", "decode", "dp"])
@pytest.mark.parametrize("n", [300, 512])
def test_t64_512_vs_oracle(gpu, monkeypatch, S, assoc, n):
    """256 < N <= 512 on the f64 trellis (NP = 512: column-split pairs of C = 4 waves,
    backtrack_f64 at KP = 8), S sequences per pair (CV_T64_S), one pair per workgroup (ragged
    batch): paths, scores and statuses bit for bit against the oracle, incl. empty sequences
    and infeasible ones (viterbi::decode's infeasible walk for `decode`)."""
    monkeypatch.setenv("CV_T64_S", S)
    monkeypatch.setenv("CV_T64_512", "1")
    pi, a, b = synth.random_hmm(n, 13, seed=n + 17, zero_frac=0.05)
    b = b.copy()
    b[:, 12] = -np.inf  # observation 12: no state emits it
    rng = np.random.default_rng(n + int(S))
    lens = rng.integers(1, 30, size=40)
    lens[[3, 17]] = 0
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 12, size=int(off[-1])).astype(np.int32)
    obs[int(off[5]) + lens[5] // 2] = 12  # sequence 5 infeasible
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, rescore_f64=False)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["padded_states"] == 512
    ref = O.decode_batch(pi, a, b, off, obs, {"viterbi": O.VITERBI, "decode": O.DECODE, "dp": O.DP}[assoc], np.float64)
    assert np.array_equal(got[2], ref[2])
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0], ref[0])


def test_t64_512_eight_wave_batch_vs_generic(gpu, monkeypatch):
    """The four-pairs-per-workgroup layout (equal lengths, S = 8 at 16,384 sequences) against
    the generic kernel (itself oracle-checked above) over the whole batch."""
    monkeypatch.setenv("CV_T64_512", "1")
    n = 449
    pi, a, b = synth.random_hmm(n, 64, seed=449)
    off = synth.offsets_from_lengths(np.full(16384, 24))
    obs = synth.iid_obs(64, int(off[-1]), 449)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["padded_states"] == 512 and t["seqs_per_wave"] == 8
    ref = cv.decode_batch(h, off, obs, dtype="f64", kernel="generic", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "generic"
    for x, y, what in zip(got, ref, ("path", "score", "status")):
        assert np.array_equal(x, y), what


@pytest.mark.parametrize("S", ["2", "4", "8"])
@pytest.mark.parametrize("n", [300, 449])
def test_t64_512_forced_vs_oracle(gpu, monkeypatch, S, n):
    """Forced states on the NP = 512 f64 trellis (EXT pairs; S = 8 runs at 4): paths, scores and
    statuses bit for bit against the oracle, incl. infeasible forced states."""
    monkeypatch.setenv("CV_T64_S", S)
    monkeypatch.setenv("CV_T64_512", "1")
    pi, a, b = synth.random_hmm(n, 19, seed=n + 300, zero_frac=0.1)
    rng = np.random.default_rng(n + 300)
    off = synth.offsets_from_lengths(rng.integers(1, 40, size=40))
    obs = rng.integers(0, 19, size=int(off[-1])).astype(np.int32)
    forced = np.where(rng.random(len(obs)) < 0.05, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, rescore_f64=False, forced=forced, dtype="f64")
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["padded_states"] == 512
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, forced=forced)
    for x, y, what in zip(got, ref, ("path", "score", "status")):
        assert np.array_equal(x, y), what


def test_generic_rows_f32_rescore(gpu):
    """f32 generic decode at N > 256 (rows mode) with the default f64 re-score: each score is
    the oracle's f64 fold along the decoded path, the paths are the f32 oracle's."""
    n = 333
    pi, a, b = synth.random_hmm(n, 9, seed=333)
    rng = np.random.default_rng(333)
    off = synth.offsets_from_lengths(rng.integers(0, 30, size=24))
    obs = rng.integers(0, 9, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    path, score, status = cv.decode_batch(h, off, obs, dtype="f32")
    rp, _, rst = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32)
    assert np.array_equal(path, rp) and np.array_equal(status, rst)
    for k in range(len(off) - 1):
        if status[k] == 0:
            assert score[k] == O.rescore_f64(pi, a, b, obs[off[k]:off[k + 1]], path[off[k]:off[k + 1]])


@pytest.mark.parametrize("S", ["2", "4"])
@pytest.mark.parametrize("assoc", ["viterbi", "decode", "dp", "forced"])
@pytest.mark.parametrize("n", [600, 1024])
def test_t64_1024_vs_oracle(gpu, monkeypatch, S, assoc, n):
    """512 < N <= 1,024 on the f64 trellis (NP = 1,024: quads of C = 4 waves, backtrack_f64 at
    KP = 16; CV_T64_1024=1): paths, scores and statuses bit for bit against the oracle, incl.
    empty and infeasible sequences and forced states."""
    monkeypatch.setenv("CV_T64_S", S)
    monkeypatch.setenv("CV_T64_1024", "1")
    pi, a, b = synth.random_hmm(n, 13, seed=n + 71, zero_frac=0.05)
    b = b.copy()
    b[:, 12] = -np.inf
    rng = np.random.default_rng(n + int(S))
    lens = rng.integers(1, 16, size=24)
    lens[[3, 17]] = 0
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 12, size=int(off[-1])).astype(np.int32)
    obs[int(off[5]) + lens[5] // 2] = 12
    forced = None
    if assoc == "forced":
        forced = np.where(rng.random(len(obs)) < 0.08, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    ak = "viterbi" if assoc == "forced" else assoc
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc=ak, rescore_f64=False, forced=forced)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["padded_states"] == 1024
    ref = O.decode_batch(pi, a, b, off, obs, {"viterbi": O.VITERBI, "decode": O.DECODE, "dp": O.DP}[ak], np.float64,
                         forced=forced)
    assert np.array_equal(got[2], ref[2])
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0], ref[0])


@pytest.mark.parametrize("n", [300, 600])
def test_t64_explicit_request_below_auto_pick(gpu, n):
    """An explicit kernel='trellis_f64' gets the f64 trellis wherever it exists (N <= 1,024),
    not only where AUTO picks it: N = 300 with 100 sequences (AUTO: generic) and N = 600 (AUTO:
    generic, NP = 1,024 on request) -- bit for bit the generic kernel's results."""
    pi, a, b = synth.random_hmm(n, 21, seed=n + 900, zero_frac=0.05)
    rng = np.random.default_rng(n + 900)
    off = synth.offsets_from_lengths(rng.integers(0, 20, size=100))
    obs = rng.integers(0, 21, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", kernel="trellis_f64", rescore_f64=False)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["padded_states"] == (512 if n <= 512 else 1024)
    auto = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    assert cv.last_timing(h)["kernel"] == "generic"
    for x, y, what in zip(got, auto, ("path", "score", "status")):
        assert np.array_equal(x, y), what


def test_t64_1024_equal_batch_chunks_vs_generic(gpu, monkeypatch):
    """NP = 1,024 quads on a large equal-length batch (S = 8 clamped to 4, many workgroups) with a
    small workspace forcing several chunks (8 KiB of rows per element): the generic kernel's
    results bit for bit, and last_timing reports the S actually launched."""
    n = 900
    pi, a, b = synth.random_hmm(n, 32, seed=901)
    off = synth.offsets_from_lengths(np.full(32768, 12))
    obs = synth.iid_obs(32, int(off[-1]), 901)
    h = cv.HMM(pi, a, b)
    # two chunks of 16,384 sequences (8 KiB of split-plane rows per element): S = 8 picked, 4 run
    got = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False, workspace_bytes=16384 * 12 * 8192)
    t = cv.last_timing(h)
    assert t["kernel"] == "trellis_f64" and t["padded_states"] == 1024 and t["seqs_per_wave"] == 4
    assert t["launches"] >= 2, t
    ref = cv.decode_batch(h, off, obs, dtype="f64", kernel="generic", rescore_f64=False)
    for x, y, what in zip(got, ref, ("path", "score", "status")):
        assert np.array_equal(x, y), what


@pytest.mark.parametrize("split", ["1:", "1:8", "0:"])
@pytest.mark.parametrize("assoc", ["viterbi", "cp", "dp", "decode"])
@pytest.mark.parametrize("dtype,n", [("f64", 5), ("f64", 64), ("f64", 100), ("f32", 200), ("f64", 256), ("f64", 300),
                                     ("f64", 512)])
def test_generic_split_candidates(gpu, monkeypatch, split, assoc, dtype, n):
    """generic_fwd_split (one sequence per workgroup, K = 2..8 threads per state walking
    ranges of the candidates, merged in range order; CV_GENERIC_SPLIT, K from the state count
    or CV_GENERIC_SPLIT_K) and the one-thread-per-state kernel against the oracle in every
    association: ragged and empty sequences, forced states, -inf transitions and emissions, an
    observation no state emits."""
    split, k = split.split(":")
    monkeypatch.setenv("CV_GENERIC_SPLIT", split)
    monkeypatch.setenv("CV_GENERIC_SPLIT_K", k)
    monkeypatch.setenv("CV_GENERIC_S", "1")
    monkeypatch.setenv("CV_GENERIC_ROWS", "0")
    pi, a, b = synth.random_hmm(n, 11, seed=n + 31, zero_frac=0.1)
    b = b.copy()
    b[:, 10] = -np.inf
    rng = np.random.default_rng(n + 77)
    lens = rng.integers(1, 30, size=19)
    lens[[3, 11]] = 0
    lens[5] = 1
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 11, size=int(off[-1])).astype(np.int32)
    forced = np.where(rng.random(len(obs)) < 0.05, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    dt = np.float32 if dtype == "f32" else np.float64
    ASSOC = {"viterbi": O.VITERBI, "cp": O.CP, "dp": O.DP, "decode": O.DECODE}
    h = cv.HMM(pi, a, b)
    fr = forced if assoc == "viterbi" else None
    got = cv.decode_batch(h, off, obs, dtype=dtype, assoc=assoc, kernel="generic", rescore_f64=False, forced=fr)
    ref = O.decode_batch(pi, a, b, off, obs, ASSOC[assoc], dt, forced=fr)
    assert np.array_equal(got[2], ref[2])
    ok = got[2] == 0
    assert np.array_equal(got[1][ok], ref[1][ok])
    assert np.array_equal(got[0], ref[0])


@pytest.mark.parametrize("split", ["1", "0"])
@pytest.mark.parametrize("name", ["golden_ties.npz", "golden_inf.npz", "golden_small.npz"])
def test_generic_split_golden(gpu, monkeypatch, split, name):
    """The golden fixtures (exact ties everywhere: the range merge must keep the first index)
    through the one-sequence psi-mode kernels with and without the candidate split."""
    from conftest import load_golden
    monkeypatch.setenv("CV_GENERIC_SPLIT", split)
    monkeypatch.setenv("CV_GENERIC_S", "1")
    monkeypatch.setenv("CV_GENERIC_ROWS", "0")
    g = load_golden(name)
    h = cv.HMM(g["pi"], g["a"], g["b"])
    seen = 0
    for dt in ("f32", "f64"):
        for assoc in ("viterbi", "cp", "dp", "decode"):
            k = f"{dt}_{assoc}"
            if k + "_path" not in g:
                continue
            got = cv.decode_batch(h, g["offsets"], g["obs"], dtype=dt, assoc=assoc, kernel="generic",
                                  rescore_f64=False)
            for x, y, what in zip(got, (g[k + "_path"], g[k + "_score"], g[k + "_status"]), ("path", "score", "status")):
                assert np.array_equal(x, y), (k, what)
            seen += 1
    assert seen > 0


@pytest.mark.parametrize("assoc", ["cp", "viterbi"])
@pytest.mark.parametrize("n", [100, 300])
def test_generic_psi_two_per_workgroup_default(gpu, monkeypatch, assoc, n):
    """CP psi mode from 256 sequences on runs two sequences per workgroup by default (the walk
    unrolled; the other associations' psi mode keeps one -- ADVICE r5: only the CP batch was
    measured): 300 ragged sequences against the oracle and against one per workgroup (tuning
    key generic_s = 1), bit for bit."""
    monkeypatch.setenv("CV_GENERIC_ROWS", "0")
    monkeypatch.delenv("CV_GENERIC_S", raising=False)
    pi, a, b = synth.random_hmm(n, 13, seed=n + 404, zero_frac=0.05)
    rng = np.random.default_rng(n + 405)
    lens = rng.integers(0, 20, size=300)
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 13, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, kernel="generic", rescore_f64=False)
    ref = O.decode_batch(pi, a, b, off, obs, O.CP if assoc == "cp" else O.VITERBI, np.float64)
    assert np.array_equal(got[2], ref[2])
    ok = got[2] == 0
    assert np.array_equal(got[1][ok], ref[1][ok])
    assert np.array_equal(got[0], ref[0])
    h.set_tuning(generic_s=1)
    one = cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, kernel="generic", rescore_f64=False)
    for x, y in zip(got, one):
        assert np.array_equal(x, y)
