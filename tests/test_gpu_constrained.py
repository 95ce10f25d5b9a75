"""GPU: forced-state decoding and the consistency-constrained decode (config 5) against
the oracle spec (oracle/np_oracle.py constrained_decode, C-accelerated in c_oracle), in both
precisions: f64 (the reference's, cp.rs:95-126 / dp.rs:147-166; the default) and f32.
Component states identical, paths bit-exact in the same precision, scores = the f64 decode's
own score (f64) or the f64 re-score of the path (f32)."""
import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [5, 45, 64, 200, 256])
@pytest.mark.parametrize("variant", ["valu", "nowave", "valu1"])
def test_forced_decode_bit_exact(gpu, n, variant):
    pi, a, b = synth.random_hmm(n, 19, seed=n)
    rng = np.random.default_rng(n)
    off = synth.offsets_from_lengths(rng.integers(1, 60, size=20))
    obs = rng.integers(0, 19, size=int(off[-1])).astype(np.int32)
    forced = np.where(rng.random(len(obs)) < 0.05, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, rescore_f64=False, forced=forced, variant=variant, dtype="f32")
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float32, forced=forced)
    for x, y, what in zip(got, ref, ("path", "score", "status")):
        assert np.array_equal(x, y), what


@pytest.mark.parametrize("n", [1, 5, 45, 64, 65, 200, 256])
def test_forced_decode_f64_bit_exact(gpu, n):
    """Forced states on the exact-f64 trellis (trellis_fwd_f64 EXT + backtrack_f64) against
    the f64 oracle; incl. infeasible sequences (a forced state whose emission is -inf)."""
    pi, a, b = synth.random_hmm(n, 19, seed=n + 300, zero_frac=0.1 if n > 1 else 0.0)
    rng = np.random.default_rng(n + 300)
    off = synth.offsets_from_lengths(rng.integers(1, 60, size=40))
    obs = rng.integers(0, 19, size=int(off[-1])).astype(np.int32)
    forced = np.where(rng.random(len(obs)) < 0.05, rng.integers(0, n, size=len(obs)), -1).astype(np.int32)
    h = cv.HMM(pi, a, b)
    got = cv.decode_batch(h, off, obs, rescore_f64=False, forced=forced, dtype="f64")
    assert cv.last_timing(h)["kernel"] == "trellis_f64"
    ref = O.decode_batch(pi, a, b, off, obs, O.VITERBI, np.float64, forced=forced)
    for x, y, what in zip(got, ref, ("path", "score", "status")):
        assert np.array_equal(x, y), what


DTYPES = [("f64", np.float64), ("f32", np.float32)]


def _check(h, pi, a, b, off, obs, comp, dtype="f64"):
    dt = dict(DTYPES)[dtype]
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, dtype=dtype)
    ref_states, forced = O.constrained_forced(pi, a, b, off, obs, comp, dt)
    for c, s in ref_states.items():
        assert states[c] == s, (c, states[c], s)
    rp, rs, rst = O.decode_batch(pi, a, b, off, obs, O.VITERBI, dt, forced=forced)
    assert np.array_equal(status, rst)
    assert np.array_equal(path, rp)
    if dtype == "f64":  # the f64 decode's own score: the reference's value, bit for bit
        assert np.array_equal(score[status == 0], rs[status == 0])
    for k in range(len(off) - 1):
        if status[k] == 0:
            assert score[k] == O.rescore_f64(pi, a, b, obs[off[k]:off[k + 1]], path[off[k]:off[k + 1]])
    assert obj == pytest.approx(float(np.sum(score)), rel=1e-12)
    for e in np.nonzero(comp >= 0)[0]:
        assert path[e] == states[comp[e]]


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("n", [4, 33, 64, 256])
def test_constrained_small(gpu, n, dtype):
    pi, a, b = synth.random_hmm(n, 11, seed=50 + n)
    rng = np.random.default_rng(n)
    off = synth.offsets_from_lengths(rng.integers(1, 40, size=24))
    obs = rng.integers(0, 11, size=int(off[-1])).astype(np.int32)
    comp = synth.constraint_components(off, seed=n, ncomp=3, prob=0.6)
    _check(cv.HMM(pi, a, b), pi, a, b, off, obs, comp, dtype)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_constrained_config5_subset(gpu, dtype):
    c = synth.config("c5", nseq=48)
    _check(cv.HMM(c["pi"], c["a"], c["b"]), c["pi"], c["a"], c["b"], c["offsets"], c["obs"], c["component"], dtype)


@pytest.mark.parametrize("kind,dtype", [("gpu", "f32"), ("gpu-f64", "f64"), ("gpu-cp", "f64"), ("gpu-dp", "f64")])
def test_constrained_solver_api(gpu, kind, dtype):
    """trait Solver with active constraints: every kind runs the constrained decode (row A0)
    at its precision -- f64 for the reference-numerics kinds (what main.rs:120 runs)."""
    pi, a, b = synth.random_hmm(10, 8, seed=9)
    rng = np.random.default_rng(9)
    seqs = [[int(x) for x in rng.integers(0, 8, size=int(t))] for t in rng.integers(2, 20, size=12)]
    tags = [[(int(rng.integers(0, 3)) if (t == 0 and rng.random() < 0.6) else None) for t in range(len(s))]
            for s in seqs]
    h = cv.HMM(pi, a, b)
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags(tags), h)
    ss.recompute_constraints(1.0)
    s = cv.GpuSolver(h, ss, kind)
    s.solve()
    sol = s.get_solution()
    assert s.get_explored_nodes() == 10 * ss.number_constraints()
    # every active element of a component decodes to one state
    for c in set(ss.component[ss.active == 1].tolist()):
        assert len(set(sol[(ss.component == c) & (ss.active == 1)].tolist())) == 1
    offsets, obs, _ = ss.sequence_blocks()
    comp = np.where(ss.active == 1, ss.component, -1).astype(np.int32)
    _, _, _, _, obj = cv.decode_constrained(h, offsets, obs, comp, dtype=dtype)
    assert s.get_objective() == obj


def test_cli_end_to_end(gpu, tmp_path):
    """main.rs workflow: input dir (sequences, tags, test_tags, hmm.json) -> output {prop}_0."""
    from cviterbi import cli

    pi, a, b = synth.random_hmm(6, 12, seed=2)
    h = cv.HMM(pi, a, b.reshape(6, 4, 3))
    h.write(tmp_path / "hmm.json")
    rng = np.random.default_rng(2)
    seqs, tags, test_tags = [], [], []
    for sid in range(8):
        T = int(rng.integers(2, 9))
        seqs += [f"{sid} {rng.integers(0, 4)} {rng.integers(0, 3)}" for _ in range(T)]
        tags += [f"{sid} {rng.integers(0, 6)}" for _ in range(T)]
        test_tags += [f"{sid} {rng.integers(0, 2) if t == 0 and sid % 2 == 0 else -1}" for t in range(T)]
    (tmp_path / "sequences").write_text("\n".join(seqs) + "\n")
    (tmp_path / "tags").write_text("\n".join(tags) + "\n")
    (tmp_path / "test_tags").write_text("\n".join(test_tags) + "\n")
    assert cli.main(["-i", str(tmp_path), "-o", str(tmp_path / "out"), "-n", "6", "-b", "4", "3", "-p", "1"]) == 0
    lines = (tmp_path / "out" / "1_0").read_text().splitlines()
    obj, nodes = lines[0].split()
    assert float(obj) < 0 and int(nodes) > 0 and int(lines[1]) >= 0
    assert len(lines) == 2 + len(seqs)


def _read_out(path):
    lines = path.read_text().splitlines()
    obj, nodes = lines[0].split()
    return float(obj), int(nodes), [tuple(int(x) for x in ln.split()) for ln in lines[2:]]


@pytest.mark.parametrize("seed", [2, 3])
def test_cli_prop0_matches_cpsolver_superseq(gpu, tmp_path, seed):
    """main.rs with prop = 0 on the default solver kind (gpu-cp = CPSolver, main.rs:120):
    every "{seq} {state}" line of OUTPUT/0_0 equals the CP super-sequence restatement
    (oracle cvo_cp_superseq_f64: cp.rs:63-93 over utils.rs:62-103, chained in f64) and the
    objective is the same double."""
    from cviterbi import cli

    pi, a, b = synth.random_hmm(6, 12, seed=seed)
    h = cv.HMM(pi, a, b.reshape(6, 4, 3))
    h.write(tmp_path / "hmm.json")
    _cli_input(tmp_path, seed=seed)
    assert cli.main(["-i", str(tmp_path), "-o", str(tmp_path / "out"), "-n", "6", "-b", "4", "3", "-p", "0"]) == 0
    obj, nodes, got = _read_out(tmp_path / "out" / "0_0")
    seqs = cv.load_sequences(tmp_path / "sequences", D=2)
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags(cv.load_tags(tmp_path / "test_tags")), h)
    ss.recompute_constraints(0.0)
    offsets, obs, _ = ss.sequence_blocks()
    rp, robj = O.cp_superseq_f64(pi, a, b, offsets, obs)
    assert got == [(int(ss.seq[k]), int(rp[k])) for k in range(len(rp))]
    assert obj == robj and nodes == 0


def test_cli_prop1_matches_constrained_spec_f64(gpu, tmp_path):
    """main.rs with prop = 1 (every test tag active) on the default kind: the f64
    consistency-constrained decode; every line equals the spec's forced decode in f64 given
    the spec's component states (oracle/np_oracle.py constrained_decode, dtype f64)."""
    from cviterbi import cli

    pi, a, b = synth.random_hmm(6, 12, seed=4)
    h = cv.HMM(pi, a, b.reshape(6, 4, 3))
    h.write(tmp_path / "hmm.json")
    _cli_input(tmp_path, seed=4)
    assert cli.main(["-i", str(tmp_path), "-o", str(tmp_path / "out"), "-n", "6", "-b", "4", "3", "-p", "1"]) == 0
    obj, nodes, got = _read_out(tmp_path / "out" / "1_0")
    seqs = cv.load_sequences(tmp_path / "sequences", D=2)
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags(cv.load_tags(tmp_path / "test_tags")), h)
    ss.recompute_constraints(1.0)
    offsets, obs, _ = ss.sequence_blocks()
    comp = np.where(ss.active == 1, ss.component, -1).astype(np.int32)
    _, forced = O.constrained_forced(pi, a, b, offsets, obs, comp, np.float64)
    rp, rs, rst = O.decode_batch(pi, a, b, offsets, obs, O.VITERBI, np.float64, forced=forced)
    assert np.all(rst == 0)
    assert got == [(int(ss.seq[k]), int(rp[k])) for k in range(len(rp))]
    assert obj == pytest.approx(float(np.sum(rs)), rel=1e-12) and nodes == 6 * ss.number_constraints()


def test_superseq_cp_chain_rounding(gpu):
    """The chained super-sequence rounds like the reference: a running total of -2^40 makes
    two predecessors 2^-20 apart tie (ulp(2^40) = 2^-12), so the first index wins in the chain
    while the per-sequence CP decode takes the strictly larger one."""
    big = 2.0 ** 40
    pi = np.array([-1.0, -1.0, -3.0])
    a = np.array([[-1.0] * 3, [-1.0 + 2.0 ** -20] * 3, [-5.0] * 3])
    b = np.array([[-0.5, -big], [-0.5, -big], [-0.5, -big]])
    off = np.array([0, 1, 3], np.int64)
    obs = np.array([1, 0, 0], np.int32)
    h = cv.HMM(pi, a, b)
    path, obj = cv.decode_superseq_cp(h, off, obs)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert np.array_equal(path, rp) and obj == robj
    assert path[1] == 0  # the chain's tie -> first index
    seq_path, _, _ = cv.decode_batch(h, off, obs, dtype="f64", assoc="cp", rescore_f64=False)
    assert seq_path[1] == 1  # per sequence: the strictly larger predecessor


@pytest.mark.parametrize("n", [1, 7, 64, 126, 127, 200, 256])
def test_superseq_cp_chain_sizes(gpu, n):
    """cp_superseq_chain with A staged in LDS (N <= 126) and read from L2 (N >= 127), every
    element against the chained restatement; quantised tables give exact ties (first index)."""
    rng = np.random.default_rng(50 + n)
    v = 13
    pi = np.round(rng.uniform(-2, 0, n) * 4) / 4
    a = np.round(rng.uniform(-2, 0, (n, n)) * 4) / 4
    b = np.round(rng.uniform(-2, 0, (n, v)) * 4) / 4
    if n > 1:  # keep one state feasible at N = 1
        a[rng.random((n, n)) < 0.1] = -np.inf
    lengths = rng.integers(1, 40, size=9)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    path, obj = cv.decode_superseq_cp(h, off, obs)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert np.array_equal(path, rp) and obj == robj


@pytest.mark.parametrize("n,quant", [(3, True), (64, False), (65, True), (128, False), (192, True), (256, False),
                                     (256, True)])
def test_superseq_cp_chain_segmented_backtrack(gpu, n, quant):
    """The N <= 256 chain (one workgroup, candidates split over its waves, kernels/chain.hip)
    over super-sequences long enough for a multi-segment parallel backtrack (256-element
    segments), incl. empty and one-element sequences: every element and the objective equal the
    chained restatement (cp.rs:63-93 over utils.rs:24-38)."""
    rng = np.random.default_rng(900 + n)
    v = 17
    if quant:  # exact ties everywhere: the first index must win in every group and across groups
        pi = np.round(rng.uniform(-2, 0, n) * 2) / 2
        a = np.round(rng.uniform(-2, 0, (n, n)) * 2) / 2
        b = np.round(rng.uniform(-2, 0, (n, v)) * 2) / 2
        a[rng.random((n, n)) < 0.1] = -np.inf
    else:
        pi, a, b = synth.random_hmm(n, v, seed=n)
    lengths = rng.integers(1, 200, size=24)
    lengths[[3, 11]] = 0
    lengths[5] = 1
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    assert off[-1] > 4 * 256
    h = cv.HMM(pi, a, b)
    path, obj = cv.decode_superseq_cp(h, off, obs)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj
    bad = np.nonzero(path != rp)[0]
    assert bad.size == 0, f"elements {bad[:10]} of {len(rp)}"
    # one element
    p1, o1 = cv.decode_superseq_cp(h, off[:2] * 0 + np.array([0, 1]), obs[:1])
    r1, ro1 = O.cp_superseq_f64(pi, a, b, np.array([0, 1]), obs[:1])
    assert np.array_equal(p1, r1) and o1 == ro1


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("nshards", [2, 5])
def test_constrained_sharded_equals_single(gpu, nshards, dtype):
    """The multi-GPU split (cv_constrained_partials per shard, integer SUM, select, per-shard
    cv_decode_forced_components) reproduces cv_decode_constrained bit for bit, whatever the
    shard boundaries (the exchange step of cviterbi.dist.constrained_decode_sharded)."""
    from cviterbi import dist as cvdist

    c = synth.config("c5", nseq=60)
    h = cv.HMM(c["pi"], c["a"], c["b"])
    off, obs, comp = c["offsets"], c["obs"], c["component"]
    ncomp = int(comp.max()) + 1
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, ncomp, dtype=dtype)
    B = len(off) - 1
    pairs = cv.constrained_pairs(off, comp, ncomp)
    part = 0
    shards = [cvdist.shard_range(B, nshards, r)[:2] for r in range(nshards)]
    for s0, s1 in shards:
        lo, hi = off[s0], off[s1]
        part = part + cv.constrained_partials(h, cvdist.shard_offsets(off, s0, s1), obs[lo:hi], comp[lo:hi], ncomp,
                                              pairs, dtype=dtype)
    got_states, explored = cv.constrained_select(h.nstates(), ncomp, part, pairs)
    assert np.array_equal(got_states, states)
    assert explored == h.nstates() * len(set(comp[comp >= 0].tolist()))
    for s0, s1 in shards:
        lo, hi = off[s0], off[s1]
        p, s, st, _ = cv.decode_forced_components(h, cvdist.shard_offsets(off, s0, s1), obs[lo:hi], comp[lo:hi],
                                                  got_states, dtype=dtype)
        assert np.array_equal(p, path[lo:hi]) and np.array_equal(s, score[s0:s1]) and np.array_equal(st, status[s0:s1])


def _multi_case(n, seed, nseq=16, tmax=24, ncomp=3, maxpos=3, v=7):
    pi, a, b = synth.random_hmm(n, v, seed=seed)
    rng = np.random.default_rng(seed)
    lengths = rng.integers(1, tmax, size=nseq)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    comp = np.full(len(obs), -1, np.int32)
    for k in range(nseq):
        m = int(rng.integers(0, maxpos + 1))
        for t in rng.choice(lengths[k], size=min(m, lengths[k]), replace=False):
            comp[off[k] + t] = rng.integers(0, ncomp)
    return pi, a, b, off, obs, comp


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("n,seed", [(3, 1), (5, 2), (8, 3), (13, 4), (16, 5), (32, 6)])
def test_constrained_multi_position(gpu, n, seed, dtype):
    """Several constrained positions per sequence: alpha / segment tables (the trellis
    kernel's `start` mode) / beta terms, pairwise component terms and the exact search;
    component states equal the spec's, paths bit-exact, scores the f64 re-score."""
    pi, a, b, off, obs, comp = _multi_case(n, seed, ncomp=3 if n <= 16 else 2)
    _check(cv.HMM(pi, a, b), pi, a, b, off, obs, comp, dtype)


def test_constrained_multi_position_sharded(gpu):
    from cviterbi import dist as cvdist

    pi, a, b, off, obs, comp = _multi_case(6, 9, nseq=30)
    h = cv.HMM(pi, a, b)
    ncomp = int(comp.max()) + 1
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, ncomp)
    pairs = cv.constrained_pairs(off, comp, ncomp)
    assert len(pairs) > 0
    part = 0
    for r in range(3):
        s0, s1, _ = cvdist.shard_range(len(off) - 1, 3, r)
        lo, hi = off[s0], off[s1]
        part = part + cv.constrained_partials(h, cvdist.shard_offsets(off, s0, s1), obs[lo:hi], comp[lo:hi], ncomp,
                                              pairs)
    got, _ = cv.constrained_select(h.nstates(), ncomp, part, pairs)
    assert np.array_equal(got, states)


def _cli_input(tmp_path, seed=2, unknown=0.0):
    rng = np.random.default_rng(seed)
    seqs, tags, test_tags = [], [], []
    for sid in range(8):
        T = int(rng.integers(2, 9))
        seqs += [f"{sid} {rng.integers(0, 4)} {rng.integers(0, 3)}" for _ in range(T)]
        tags += [f"{sid} {-1 if rng.random() < unknown else rng.integers(0, 6)}" for _ in range(T)]
        test_tags += [f"{sid} {rng.integers(0, 2) if t == 0 and sid % 2 == 0 else -1}" for t in range(T)]
    (tmp_path / "sequences").write_text("\n".join(seqs) + "\n")
    (tmp_path / "tags").write_text("\n".join(tags) + "\n")
    (tmp_path / "test_tags").write_text("\n".join(test_tags) + "\n")
    return len(seqs)


@pytest.mark.parametrize("supervised", [True, False])
def test_cli_train_then_decode(gpu, tmp_path, supervised):
    """main.rs:89-98 with -t [-s]: the model is fitted on the GPU, written to INPUT/hmm.json,
    and used for the decode; the written model equals a direct fit from the same start."""
    from cviterbi import cli

    # Baum-Welch on partly tagged data (a fully tagged corpus gives hard zero transitions,
    # which can make the constrained decode infeasible)
    n_el = _cli_input(tmp_path, unknown=0.0 if supervised else 0.5)
    args = ["-i", str(tmp_path), "-o", str(tmp_path / "out"), "-n", "6", "-b", "4", "3", "-p", "1", "-t",
            "--seed", "5"] + (["-s"] if supervised else [])
    assert cli.main(args) == 0
    lines = (tmp_path / "out" / "1_0").read_text().splitlines()
    assert len(lines) == 2 + n_el
    seqs = cv.load_sequences(tmp_path / "sequences", D=2)
    tags = cv.load_tags(tmp_path / "tags")
    pi0, a0, b0 = cli._random_start(6, (4, 3), np.random.default_rng(5))
    off, obs, tg = cli._flatten(seqs, tags, (4, 3))
    if supervised:
        lp, la, lb = cv.fit_mle(pi0, a0, b0, off, obs, tg)
    else:
        lp, la, lb, _ = cv.fit_train(pi0, a0, b0, off, obs, tg, max_iter=1000, tol=0.001)
    h = cv.HMM.from_json(tmp_path / "hmm.json")
    # MLE is exact (integer counts); the Baum-Welch E-step sums with f64 atomics, so two runs
    # may differ in the last bits
    tol = 0 if supervised else 1e-12
    for s in range(6):
        assert h.init_prob(s, 0) == pytest.approx(lp[s] + lb[s, 0], rel=tol, abs=tol)
        for o in range(12):
            assert h.emit_prob(s, o) == pytest.approx(lb[s, o], rel=tol, abs=tol)


def test_cli_train_config4_states(gpu, tmp_path):
    """main.rs:89-98 with -t at config 4's N = 256 and bdims [32, 32]: Baum-Welch beyond N = 128
    (the xi sums as a matrix-core GEMM, fit.hip bw_xi_gemm), the fitted model written and used
    by the decode; it equals a direct fit from the same start."""
    from cviterbi import cli

    rng = np.random.default_rng(11)
    seqs, tags, test_tags = [], [], []
    nxt = 0
    for sid in range(64):
        T = int(rng.integers(6, 14))
        seqs += [f"{sid} {rng.integers(0, 32)} {rng.integers(0, 32)}" for _ in range(T)]
        for t in range(T):
            # every state tagged at some non-final element (it keeps its a / b denominators
            # away from 0 -- hmm.rs:165-170 divides by them), 40% of the elements untagged
            if t < T - 1 and rng.random() < 0.6:
                tags.append(f"{sid} {nxt % 256}")
                nxt += 1
            else:
                tags.append(f"{sid} -1")
        test_tags += [f"{sid} -1" for _ in range(T)]
    assert nxt >= 256
    (tmp_path / "sequences").write_text("\n".join(seqs) + "\n")
    (tmp_path / "tags").write_text("\n".join(tags) + "\n")
    (tmp_path / "test_tags").write_text("\n".join(test_tags) + "\n")
    args = ["-i", str(tmp_path), "-o", str(tmp_path / "out"), "-n", "256", "-b", "32", "32", "-p", "0", "-t",
            "--seed", "3"]
    assert cli.main(args) == 0
    assert len((tmp_path / "out" / "0_0").read_text().splitlines()) == 2 + len(seqs)
    h = cv.HMM.from_json(tmp_path / "hmm.json")
    assert h.nstates() == 256
    # this EM does not settle (sum |new - old| oscillates: the 1,000 iterations all run), so
    # two GPU runs, whose f64 atomics add in different orders, drift apart: check the written
    # model is a proper log10 HMM (rows sum to 1, nothing NaN; the tiny-c_t steps it meets are
    # test_gpu_train_subnormal_xi_denominator's) -- parity vs the oracle is test_fit.py's
    a = np.stack([h.transitions_to(j) for j in range(256)], axis=1)  # a[i, j], log10
    assert not np.isnan(a).any()
    assert np.allclose((10.0 ** a).sum(axis=1), 1.0, rtol=1e-9)


def test_cli_cfn(gpu, tmp_path):
    """main.rs:116-118 (run_cfn): OUTPUT/problem_{prop}_0.cfn and the compile time in {prop}_0;
    the file equals the restatement of cfn.rs on the same super-sequence."""
    import cfn_oracle as CO
    from cviterbi import cli

    pi, a, b = synth.random_hmm(6, 12, seed=2)
    h = cv.HMM(pi, a, b.reshape(6, 4, 3))
    h.write(tmp_path / "hmm.json")
    _cli_input(tmp_path)
    assert cli.main(["-i", str(tmp_path), "-o", str(tmp_path / "out"), "-n", "6", "-b", "4", "3", "-p", "1",
                     "--cfn"]) == 0
    assert int((tmp_path / "out" / "1_0").read_text().strip()) >= 0
    seqs = cv.load_sequences(tmp_path / "sequences", D=2)
    control = cv.load_tags(tmp_path / "test_tags")
    ss = cv.SuperSequence(seqs, cv.Constraints.from_tags(control), h)
    ss.recompute_constraints(1.0)
    comp = np.where(ss.active == 1, ss.component, -1).tolist()
    ref = CO.write_cfn_text(pi.tolist(), a.tolist(), b.tolist(), ss.value.tolist(), comp,
                            (ss.t == 0).astype(int).tolist())
    assert (tmp_path / "out" / "problem_1_0.cfn").read_text() == ref


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("n,seed", [(7, 1), (64, 2), (256, 3)])
def test_device_exact_sums_equal_host(gpu, monkeypatch, n, seed, dtype):
    """The unary terms summed exactly on the device (kernels/exact.hip) give the same int64
    words as the host loop (tuning key host_sums = 1): single- and multi-position sequences, -inf
    terms, several components."""
    pi, a, b = synth.random_hmm(n, 13, seed=seed, zero_frac=0.05)
    rng = np.random.default_rng(seed)
    off = synth.offsets_from_lengths(rng.integers(1, 50, size=300))
    obs = rng.integers(0, 13, size=int(off[-1])).astype(np.int32)
    comp = np.full(len(obs), -1, np.int32)
    for s in range(len(off) - 1):  # 0, 1 or 3 constrained positions per sequence
        k = int(rng.choice([0, 1, 1, 3]))
        if k and off[s + 1] - off[s] >= k:
            pos = rng.choice(np.arange(off[s], off[s + 1]), size=k, replace=False)
            comp[pos] = rng.integers(0, 5, size=k)
    h = cv.HMM(pi, a, b)
    pairs = cv.constrained_pairs(off, comp, 5)
    dev = cv.constrained_partials(h, off, obs, comp, 5, pairs, dtype=dtype)
    h.set_tuning(host_sums=1)
    host = cv.constrained_partials(h, off, obs, comp, 5, pairs, dtype=dtype)
    assert np.array_equal(dev, host)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("n,seed", [(5, 11), (64, 12), (256, 13)])
def test_constrained_device_equals_host(gpu, n, seed, dtype):
    """cv_decode_constrained_device (inputs/outputs in HBM) == cv_decode_constrained, incl.
    several constrained positions per sequence and an unassignable component."""
    import torch
    pi, a, b = synth.random_hmm(n, 9, seed=seed)
    rng = np.random.default_rng(seed)
    off = synth.offsets_from_lengths(rng.integers(1, 48, size=40))
    obs = rng.integers(0, 9, size=int(off[-1])).astype(np.int32)
    comp = synth.constraint_components(off, seed=seed, ncomp=4, prob=0.7)
    h = cv.HMM(pi, a, b)
    ref = cv.decode_constrained(h, off, obs, comp, ncomp=5, dtype=dtype)  # component 4 has no element
    dev = torch.device("cuda", 0)
    path_d = torch.empty(int(off[-1]), dtype=torch.int32, device=dev)
    score_d = torch.empty(len(off) - 1, dtype=torch.float64, device=dev)
    status_d = torch.empty(len(off) - 1, dtype=torch.uint8, device=dev)
    states, obj = cv.decode_constrained_device(h, off, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev),
                                               comp, path_d, score_d, status_d, ncomp=5, dtype=dtype)
    assert np.array_equal(states, ref[3])
    assert np.array_equal(path_d.cpu().numpy(), ref[0])
    assert np.array_equal(score_d.cpu().numpy(), ref[1])
    assert np.array_equal(status_d.cpu().numpy(), ref[2])
    assert obj == ref[4]


def test_constrained_device_rejects_bad_obs(gpu):
    import torch
    pi, a, b = synth.random_hmm(8, 5, seed=1)
    off = np.array([0, 10, 20], np.int64)
    obs = np.zeros(20, np.int32)
    obs[13] = 5
    comp = np.full(20, -1, np.int32)
    comp[3] = 0
    dev = torch.device("cuda", 0)
    h = cv.HMM(pi, a, b)
    out = [torch.empty(20, dtype=torch.int32, device=dev), torch.empty(2, dtype=torch.float64, device=dev),
           torch.empty(2, dtype=torch.uint8, device=dev)]
    with pytest.raises(cv.CVError, match=r"obs\[13\]"):
        cv.decode_constrained_device(h, off, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev), comp, *out)


def _resume_case(n, seed, nseq=48, tmax=40, bad_obs=False):
    pi, a, b = synth.random_hmm(n, 9, seed=seed)
    if bad_obs:  # observation 8 is impossible in every state: sequences holding it are infeasible
        b = b.copy()
        b[:, 8] = -np.inf
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, tmax, size=nseq)
    lens[:3] = [1, 2, tmax]
    off = synth.offsets_from_lengths(lens)
    obs = rng.integers(0, 8, size=int(off[-1])).astype(np.int32)
    if bad_obs:
        obs[rng.integers(0, len(obs), size=3)] = 8
    comp = np.full(len(obs), -1, np.int32)
    for s in range(nseq):
        if rng.random() < 0.7:
            k = rng.integers(1, 4)
            pos = rng.choice(lens[s], size=min(k, lens[s]), replace=False)
            comp[off[s] + pos] = rng.integers(0, 4, size=len(pos))
    comp[off[0]] = 0          # t_1 = first element (length-1 sequence)
    comp[off[2] + lens[2] - 1] = 1  # t_1 = last element
    return pi, a, b, off, obs, comp


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("n,seed,bad", [(128, 1, False), (192, 2, False), (256, 3, False), (256, 4, True),
                                        (130, 5, True), (200, 6, False), (40, 7, True)])
def test_constrained_resume_equals_full(gpu, monkeypatch, n, seed, bad, dtype):
    """Resume flow (stored prefix rows, decode of [t_1, end), prefix backtrack from the forced
    state) == the full forced decode (tuning key no_resume = 1), host and device APIs, bit for bit;
    f32: N = 200 (NP 224) and N = 40 are outside the resume flow and run the full decode both
    times; f64 resumes at every N <= 256."""
    import torch
    pi, a, b, off, obs, comp = _resume_case(n, seed, bad_obs=bad)
    h = cv.HMM(pi, a, b)
    for f64 in ((False, True) if dtype == "f32" else (False,)):  # f32 scores see the resumed row itself
        h.set_tuning(no_resume=1)
        ref = cv.decode_constrained(h, off, obs, comp, ncomp=5, rescore_f64=f64, dtype=dtype)
        h.set_tuning(no_resume=0)
        got = cv.decode_constrained(h, off, obs, comp, ncomp=5, rescore_f64=f64, dtype=dtype)
        for x, y, what in zip(got, ref, ("path", "score", "status", "states", "objective")):
            assert np.array_equal(np.asarray(x), np.asarray(y)), (what, f64)
    if bad:
        assert (ref[2] == 1).any()
    dev = torch.device("cuda", 0)
    path_d = torch.full((int(off[-1]),), 7, dtype=torch.int32, device=dev)
    score_d = torch.empty(len(off) - 1, dtype=torch.float64, device=dev)
    status_d = torch.empty(len(off) - 1, dtype=torch.uint8, device=dev)
    states, obj = cv.decode_constrained_device(h, off, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev),
                                               comp, path_d, score_d, status_d, ncomp=5, dtype=dtype)
    assert np.array_equal(states, ref[3])
    assert np.array_equal(path_d.cpu().numpy(), ref[0])
    assert np.array_equal(score_d.cpu().numpy(), ref[1])
    assert np.array_equal(status_d.cpu().numpy(), ref[2])
    assert obj == ref[4] or (np.isinf(obj) and np.isinf(ref[4]))


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_constrained_resume_oracle(gpu, dtype):
    """Resume flow at N = 256 against the oracle spec directly."""
    pi, a, b, off, obs, comp = _resume_case(256, 9, nseq=24, tmax=30)
    for s in range(len(off) - 1):  # no component pairs (the oracle's search is brute force):
        e = off[s] + np.nonzero(comp[off[s]:off[s + 1]] >= 0)[0]  # later positions repeat the first's
        comp[e[1:]] = comp[e[0]] if len(e) else -1                # component (m >= 2, diagonal terms)
    _check(cv.HMM(pi, a, b), pi, a, b, off, obs, comp, dtype)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("nshards,resume", [(3, "0"), (3, "1"), (1, "0")])
def test_constrained_exchange_shards(gpu, monkeypatch, nshards, resume, dtype):
    """cv_decode_constrained_exchange per shard, the callback handing back the SUM of every
    shard's partials (what the all-reduce returns), == cv_decode_constrained's slice of that
    shard, with and without the resume flow; the callback sees exactly the shard's partials."""
    from cviterbi import dist as cvdist

    monkeypatch.setenv("CV_NO_RESUME", resume)
    pi, a, b, off, obs, comp = _resume_case(256, 21, nseq=60)
    h = cv.HMM(pi, a, b)
    ncomp = 5
    path, score, status, states, obj = cv.decode_constrained(h, off, obs, comp, ncomp, dtype=dtype)
    B = len(off) - 1
    pairs = cv.constrained_pairs(off, comp, ncomp)
    shards = [cvdist.shard_range(B, nshards, r)[:2] for r in range(nshards)]
    parts = [cv.constrained_partials(h, cvdist.shard_offsets(off, s0, s1), obs[off[s0]:off[s1]],
                                     comp[off[s0]:off[s1]], ncomp, pairs, dtype=dtype) for s0, s1 in shards]
    total = np.sum(parts, axis=0)
    for (s0, s1), own in zip(shards, parts):
        lo, hi = off[s0], off[s1]
        seen = []

        def exchange(w, own=own):
            seen.append(np.array_equal(w, own))
            return total

        p, s, st, got_states, explored, _ = cv.decode_constrained_exchange(
            h, cvdist.shard_offsets(off, s0, s1), obs[lo:hi], comp[lo:hi], ncomp, pairs, exchange, dtype=dtype)
        assert seen == [True]
        assert np.array_equal(got_states, states)
        assert np.array_equal(p, path[lo:hi]) and np.array_equal(s, score[s0:s1]) and np.array_equal(st, status[s0:s1])


def _sharded_worker(rank, world, port, q):
    import os
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
    import torch.distributed as dist
    from cviterbi import dist as cvd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pi, a, b, off, obs, comp = _resume_case(256, 31, nseq=50)
        h = cv.HMM(pi, a, b)
        got = cvd.constrained_decode_sharded(h, off, obs, comp, 5, dist)
        if rank == 0:
            ref = cv.decode_constrained(h, off, obs, comp, 5)
            q.put(all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(got, ref)))
    finally:
        dist.destroy_process_group()


def test_constrained_sharded_two_processes(gpu):
    """cviterbi.dist.constrained_decode_sharded in 2 processes (gloo for the exchange and the
    gather, both ranks on cuda:0) == the single-process decode on rank 0."""
    import torch.multiprocessing as mp
    from test_dist import _free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_sharded_worker, args=(2, _free_port(), q), nprocs=2, join=True, start_method="spawn")
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("nseq,T", [(4096, 64), (300, 33)])
def test_constrained_device_side_decode_bit_identical(gpu, monkeypatch, nseq, T):
    """The device API decodes the unconstrained sequences on a side stream beside the terms
    pass: bit-identical to the same call with tuning key no_side = 1 and to the host API
    (which does not use the side stream)."""
    import torch

    pi, a, b = synth.random_hmm(256, 40, seed=nseq)
    off = np.arange(nseq + 1, dtype=np.int64) * T
    rng = np.random.default_rng(nseq)
    obs = rng.integers(0, 40, size=nseq * T).astype(np.int32)
    comp = synth.constraint_components(off, seed=nseq, ncomp=5, prob=0.5)
    h = cv.HMM(pi, a, b)
    dev = torch.device("cuda", 0)
    o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
    res = []
    for side in ("0", "1"):
        h.set_tuning(no_side=int(side))
        outs = (torch.full((nseq * T,), 9, dtype=torch.int32, device=dev),
                torch.empty(nseq, dtype=torch.float64, device=dev), torch.empty(nseq, dtype=torch.uint8, device=dev))
        states, obj = cv.decode_constrained_device(h, off, o_d, ob_d, comp, *outs, ncomp=5, dtype="f64")
        res.append((outs[0].cpu().numpy(), outs[1].cpu().numpy(), outs[2].cpu().numpy(), states, obj))
    ref = cv.decode_constrained(h, off, obs, comp, ncomp=5, dtype="f64")
    for got in res:
        for x, y, what in zip(got, ref, ("path", "score", "status", "states", "objective")):
            assert np.array_equal(np.asarray(x), np.asarray(y)), what
    assert np.all(ref[2] == 0)


def test_full_config5_device_equals_host(gpu):
    """Config 5 at full size through the device API (side-stream decode of the unconstrained
    half, resume flow) == the host API, bit for bit."""
    import torch

    c = synth.config("c5")
    pi, a, b, off, obs, comp = c["pi"], c["a"], c["b"], c["offsets"], c["obs"], c["component"]
    h = cv.HMM(pi, a, b.reshape(256, 32, 32))
    ref = cv.decode_constrained(h, off, obs, comp, 7, dtype="f64")
    dev = torch.device("cuda", 0)
    outs = (torch.empty(len(obs), dtype=torch.int32, device=dev), torch.empty(len(off) - 1, dtype=torch.float64,
                                                                             device=dev),
            torch.empty(len(off) - 1, dtype=torch.uint8, device=dev))
    states, obj = cv.decode_constrained_device(h, off, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev),
                                               comp, *outs, ncomp=7, dtype="f64")
    got = (outs[0].cpu().numpy(), outs[1].cpu().numpy(), outs[2].cpu().numpy(), states, obj)
    for x, y, what in zip(got, ref, ("path", "score", "status", "states", "objective")):
        assert np.array_equal(np.asarray(x), np.asarray(y)), what


@pytest.mark.parametrize("n", [256, 192])
def test_constrained_ext_workgroup_units_bit_identical(gpu, tmp_path, n):
    """The constrained passes in eight-wave workgroups (the resume decode takes them from two
    rounds on; tuning key t64_wg_force = 1 forces them for every EXT launch: prefix, suffix,
    segment tables, resume decode) decode the same bits as one-wave workgroups: ragged
    lengths, multi-position sequences (segment tables), empty sequences."""
    import os
    import subprocess
    import sys

    pkg = os.path.dirname(os.path.dirname(os.path.abspath(cv.__file__)))
    pi, a, b = synth.random_hmm(n, 30, seed=300 + n)
    rng = np.random.default_rng(300 + n)
    lengths = rng.integers(0, 90, size=1500)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, 30, size=int(off[-1])).astype(np.int32)
    comp = synth.constraint_components(off, seed=300 + n, ncomp=4, prob=0.4)
    np.savez(tmp_path / "in.npz", pi=pi, a=a, b=b, off=off, obs=obs, comp=comp)
    h = cv.HMM(pi, a, b)
    ref = cv.decode_constrained(h, off, obs, comp, ncomp=4, dtype="f64")
    code = (
        "import sys, numpy as np; sys.path.insert(0, sys.argv[1]); import cviterbi as cv; "
        "d = np.load(sys.argv[2]); h = cv.HMM(d['pi'], d['a'], d['b']); "
        "p, s, st, states, obj = cv.decode_constrained(h, d['off'], d['obs'], d['comp'], ncomp=4, dtype='f64'); "
        "np.savez(sys.argv[3], p=p, s=s, st=st, states=np.asarray(states), obj=np.asarray(obj))")
    env = dict(os.environ, CV_T64_WG_FORCE="1", CV_T64_S="8")
    subprocess.run([sys.executable, "-c", code, pkg, str(tmp_path / "in.npz"), str(tmp_path / "out.npz")],
                   env=env, check=True, timeout=180)
    got = np.load(tmp_path / "out.npz")
    for key, x in zip(("p", "s", "st", "states", "obj"), ref):
        assert np.array_equal(np.asarray(x), got[key]), key


def test_one_handle_batch_and_constrained_on_two_streams(gpu):
    """one handle, cv_decode_batch_device enqueued on stream A and, with no
    synchronisation, cv_decode_constrained_device on stream B.  Both share the handle's
    workspace buffers (longest-first order, zero rows, statuses); the constrained call waits on
    its own stream for the batch call's workspace (ws_done) before writing them.  Each result
    equals the same call run alone, bit for bit (several interleavings)."""
    import torch

    dev = torch.device("cuda", 0)
    n = 256
    pi, a, b = synth.random_hmm(n, 40, seed=91)
    rng = np.random.default_rng(91)
    # batch A: 8,192 ragged sequences (a long forward pass: the constrained call starts while it runs)
    offa = synth.offsets_from_lengths(rng.integers(16, 96, size=8192))
    obsa = rng.integers(0, 40, size=int(offa[-1])).astype(np.int32)
    # constrained B: 600 sequences, 5 components
    offb = synth.offsets_from_lengths(rng.integers(1, 60, size=600))
    obsb = rng.integers(0, 40, size=int(offb[-1])).astype(np.int32)
    comp = synth.constraint_components(offb, seed=92, ncomp=5, prob=0.6)
    h = cv.HMM(pi, a, b)
    da = [torch.from_numpy(offa).to(dev), torch.from_numpy(obsa).to(dev)]
    db = [torch.from_numpy(offb).to(dev), torch.from_numpy(obsb).to(dev)]

    def outs(off):
        return (torch.full((int(off[-1]),), -1, dtype=torch.int32, device=dev),
                torch.full((len(off) - 1,), 7.0, dtype=torch.float64, device=dev),
                torch.full((len(off) - 1,), 9, dtype=torch.uint8, device=dev))

    def host(t):
        return tuple(x.cpu().numpy().copy() for x in t)

    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    oa = outs(offa)
    cv.decode_batch_device(h, da[0], da[1], *oa, offsets_host=offa, stream=sa.cuda_stream, dtype="f64")
    torch.cuda.synchronize()
    ref_a = host(oa)
    ob = outs(offb)
    ref_b = cv.decode_constrained_device(h, offb, db[0], db[1], comp, *ob, ncomp=5, stream=sb.cuda_stream)
    torch.cuda.synchronize()
    ref_bo = host(ob)
    for rep in range(3):
        oa, ob = outs(offa), outs(offb)
        torch.cuda.synchronize()
        cv.decode_batch_device(h, da[0], da[1], *oa, offsets_host=offa, stream=sa.cuda_stream, dtype="f64")
        got_b = cv.decode_constrained_device(h, offb, db[0], db[1], comp, *ob, ncomp=5, stream=sb.cuda_stream)
        torch.cuda.synchronize()
        for x, y, what in zip(host(oa), ref_a, ("path", "score", "status")):
            assert np.array_equal(x, y), (rep, "batch", what)
        for x, y, what in zip(host(ob), ref_bo, ("path", "score", "status")):
            assert np.array_equal(x, y), (rep, "constrained", what)
        assert np.array_equal(got_b[0], ref_b[0]) and got_b[1] == ref_b[1], rep
