"""GPU: the parallel CPSolver chain (cv_decode_superseq_cp, main.rs:120 / cp.rs:63-93 over the
super-sequence of utils.rs:62-103).  Every sequence is decoded on its own by the f64 trellis,
certified to be the chain's own path at the chain's running total, and folded on the host;
uncertified sequences re-run through the serial chain kernel.  The result must equal the serial
chain (tuning key chain_par = 0) and the C oracle's chained restatement (cvo_cp_superseq_f64) bit for bit:
every element of the path and the objective."""
import os

import numpy as np
import pytest

import c_oracle as O
import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu


def _serial(h, off, obs):
    with h.tuned(chain_par=0):  # tuning key (cviterbi.h): the serial chain kernel
        out = cv.decode_superseq_cp(h, off, obs)
        assert not cv.last_superseq_stats(h)["parallel"]
        return out


def _par(h, off, obs, force=None, spec=True):
    with h.tuned(chain_par_force=0 if force is None else int(force), chain_spec=1 if spec else 0):
        out = cv.decode_superseq_cp(h, off, obs)
        return out, cv.last_superseq_stats(h)


def _case(n, v, nseq, tlo, thi, seed, scale=1.0, zeros=(), ones=()):
    pi, a, b = synth.random_hmm(n, v, seed=seed)
    pi, a, b = pi * scale, a * scale, b * scale
    rng = np.random.default_rng(seed + 1)
    lengths = rng.integers(tlo, thi + 1, size=nseq)
    for k in zeros:
        lengths[k] = 0
    for k in ones:
        lengths[k] = 1
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    return pi, a, b, off, obs


@pytest.mark.parametrize("n", [1, 5, 64, 100, 128, 192, 256])
def test_chain_par_equals_oracle(gpu, n):
    """Random log10 models at every padded width, ragged lengths incl. empty and one-element
    sequences: the parallel chain equals the oracle's chained restatement element by element."""
    pi, a, b, off, obs = _case(n, 23, 60, 1, 90, seed=4000 + n, zeros=(3, 17), ones=(5, 40))
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs)
    assert st["parallel"], st
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj
    bad = np.nonzero(path != rp)[0]
    assert bad.size == 0, f"elements {bad[:10]} of {len(rp)}; {st}"


@pytest.mark.parametrize("spec", [True, False])
@pytest.mark.parametrize("n,force", [(64, 1), (64, 2), (64, 3), (256, 2), (256, 5), (7, 4)])
def test_chain_par_forced_runs(gpu, n, force, spec):
    """CV_CHAIN_PAR_FORCE=m takes every m-th sequence as uncertified.  With speculation they are
    re-decoded in parallel from their predicted offsets and taken where the offset was exact;
    without it (CV_CHAIN_SPEC=0) the serial chain kernel re-runs each from a synthetic start row
    (after a certified sequence) or from the previous sequence's last row (consecutive runs,
    m = 1: the whole chain in one run).  Either way: the oracle's chain."""
    pi, a, b, off, obs = _case(n, 19, 40, 1, 70, seed=4100 + n + force, zeros=(2,), ones=(7,))
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs, force=force, spec=spec)
    assert st["parallel"] and st["rerun"] + st["speculated"] >= 1, st
    if spec:
        assert st["spec_batches"] >= 1 and st["speculated"] >= 1, st
    else:
        assert st["speculated"] == 0 and st["rerun"] >= 1, st
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj and np.array_equal(path, rp), st


def test_chain_par_rounding_case(gpu):
    """The chain-rounding case of test_superseq_cp_chain_rounding with more sequences around it:
    at a running total of -2^40 two predecessors 2^-20 apart tie in the chain -- no certificate
    can hold there, so the serial chain kernel decides (first index), exactly as the reference."""
    big = 2.0 ** 40
    pi = np.array([-1.0, -1.0, -3.0])
    a = np.array([[-1.0] * 3, [-1.0 + 2.0 ** -20] * 3, [-5.0] * 3])
    b = np.array([[-0.5, -big], [-0.5, -big], [-0.5, -big]])
    lengths = np.array([1, 2, 3, 1, 2, 5, 2])
    off = synth.offsets_from_lengths(lengths)
    obs = np.zeros(int(off[-1]), np.int32)
    obs[0] = 1
    h = cv.HMM(pi, a, b)
    for spec in (True, False):
        (path, obj), st = _par(h, off, obs, spec=spec)
        rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
        assert np.array_equal(path, rp) and obj == robj, st
        assert st["parallel"] and st["rerun"] + st["speculated"] >= 1, st


@pytest.mark.parametrize("scale", [1.0, 1e3, 1e6])
def test_chain_par_large_totals(gpu, scale):
    """Scaled models (still log-probability-like: every entry <= 0) push the running total to
    1e7..1e13, where the chain's ulp reaches the path margins: certificates fail for some
    sequences, quantised folds take the rest, and the result is still the serial chain's."""
    pi, a, b, off, obs = _case(64, 31, 400, 50, 300, seed=4200, scale=scale)
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs)
    sp, sobj = _serial(h, off, obs)
    assert st["parallel"], st
    assert obj == sobj, (obj, sobj, st)
    (p2, o2), st2 = _par(h, off, obs, spec=False)
    assert o2 == sobj and np.array_equal(p2, sp), st2
    bad = np.nonzero(path != sp)[0]
    assert bad.size == 0, f"elements {bad[:10]} of {len(sp)}; {st}"
    if scale == 1.0:
        assert st["rerun"] == 0 and st["quantised"] > 300, st


def test_chain_par_1m_elements_vs_serial(gpu):
    """>= 1 M elements at N = 256 (config-4 model, 2,048 sequences of 512): the parallel chain
    equals the serial chain kernel bit for bit (every element and the objective), with nearly
    every sequence certified and folded by one quantised add."""
    c = synth.config("c4", 2048)
    h = cv.HMM(c["pi"], c["a"], c["b"])
    (path, obj), st = _par(h, c["offsets"], c["obs"])
    assert int(c["offsets"][-1]) >= 1 << 20
    sp, sobj = _serial(h, c["offsets"], c["obs"])
    assert st["parallel"] and st["certified"] + st["rerun"] + st["speculated"] == 2048, st
    assert st["certified"] >= 2000 and st["quantised"] >= 1900, st
    assert obj == sobj
    bad = np.nonzero(path != sp)[0]
    assert bad.size == 0, f"elements {bad[:10]}; {st}"


def test_chain_par_quantised_ties(gpu):
    """Dyadic (quantised) tables: exact ties at every step defeat every certificate, so every
    sequence re-runs through the serial chain kernel in one run -- equal to the oracle."""
    rng = np.random.default_rng(4300)
    n, v = 65, 9
    pi = np.round(rng.uniform(-2, 0, n) * 2) / 2
    a = np.round(rng.uniform(-2, 0, (n, n)) * 2) / 2
    b = np.round(rng.uniform(-2, 0, (n, v)) * 2) / 2
    off = synth.offsets_from_lengths(rng.integers(0, 50, size=30))
    obs = rng.integers(0, v, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    for spec in (True, False):
        (path, obj), st = _par(h, off, obs, spec=spec)
        rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
        assert obj == robj and np.array_equal(path, rp), st


def test_chain_par_not_applicable(gpu):
    """A positive entry (outside the certificate's [-2^80, 0] models) or an infeasible sequence:
    the serial chain runs (stats: parallel = False) with the same results / CV_EINFEASIBLE."""
    pi, a, b, off, obs = _case(16, 7, 12, 1, 30, seed=4400)
    a2 = a.copy()
    a2[0, 0] = 0.25
    h = cv.HMM(pi, a2, b)
    (path, obj), st = _par(h, off, obs)
    rp, robj = O.cp_superseq_f64(pi, a2, b, off, obs)
    assert not st["parallel"] and obj == robj and np.array_equal(path, rp)
    b3 = b.copy()
    b3[:, int(obs[off[4]])] = -np.inf  # sequence 4 cannot start
    h3 = cv.HMM(pi, a, b3)
    with pytest.raises(cv.CVError, match="INFEASIBLE"):
        cv.decode_superseq_cp(h3, off, obs)
    assert not cv.last_superseq_stats(h3)["parallel"]


# ---- N > 256 (round 5): the parallel chain on the batch path's own row-A0 decode ----------
# N = 300 / 600 (small batches) run the generic kernels' rows mode, N = 512 the NP = 512 f64
# trellis (split-plane rows), N = 1,024 the NP = 1,024 quads; speculation runs the generic CP
# kernel (cp_init / cp_last), the runs cp_superseq_chain with the segmented backtrack.

@pytest.mark.parametrize("n", [300, 512, 600, 1024])
def test_chain_par_large_n_equals_oracle(gpu, n):
    """Ragged lengths incl. empty and one-element sequences: the oracle's chain element by
    element and the objective, with the row-A0 kernel the batch path picks at this N."""
    pi, a, b, off, obs = _case(n, 17, 30, 1, 40, seed=4500 + n, zeros=(3, 17), ones=(5, 21))
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs)
    assert st["parallel"] and st["certified"] >= 20, st
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj
    bad = np.nonzero(path != rp)[0]
    assert bad.size == 0, f"elements {bad[:10]} of {len(rp)}; {st}"


@pytest.mark.parametrize("spec", [True, False])
@pytest.mark.parametrize("n,force", [(300, 2), (512, 3), (600, 1), (1024, 2)])
def test_chain_par_large_n_forced_runs(gpu, n, force, spec):
    """CV_CHAIN_PAR_FORCE=m above N = 256: speculation through the generic CP kernel (start
    offsets, last rows by sequence), or the serial runs of cp_superseq_chain from a synthetic or
    exact start row (m = 1: the whole chain in one run) -- the oracle's chain either way."""
    pi, a, b, off, obs = _case(n, 11, 16, 1, 30, seed=4600 + n + force, zeros=(2,), ones=(7,))
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs, force=force, spec=spec)
    assert st["parallel"] and st["rerun"] + st["speculated"] >= 1, st
    if spec:
        assert st["spec_batches"] >= 1 and st["speculated"] >= 1, st
    else:
        assert st["speculated"] == 0 and st["rerun"] >= 1, st
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj and np.array_equal(path, rp), st


@pytest.mark.parametrize("n", [512, 1024])
def test_chain_par_large_n_vs_serial(gpu, n):
    """1,024 sequences of 96 at N = 512 / 1,024 (a config-4-like model): the parallel chain equals
    the serial chain kernel (cp_superseq_chain) bit for bit, nearly every sequence certified."""
    pi, a, b = synth.random_hmm(n, 64, seed=4700 + n)
    off = synth.offsets_from_lengths(np.full(1024, 96))
    obs = synth.iid_obs(64, int(off[-1]), 4700 + n)
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs)
    sp, sobj = _serial(h, off, obs)
    assert st["parallel"] and st["certified"] + st["rerun"] + st["speculated"] == 1024, st
    assert st["certified"] >= 950, st
    assert obj == sobj
    bad = np.nonzero(path != sp)[0]
    assert bad.size == 0, f"elements {bad[:10]}; {st}"


def test_chain_serial_large_n_segmented_backtrack(gpu):
    """The serial chain above N = 256 now backtracks through the segmented passes (runtime row
    width, psi from global memory): > 256 elements per segment, several segments -- the oracle."""
    pi, a, b, off, obs = _case(300, 9, 12, 200, 400, seed=4800)
    h = cv.HMM(pi, a, b)
    sp, sobj = _serial(h, off, obs)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert sobj == robj and np.array_equal(sp, rp)


@pytest.mark.parametrize("n", [1100, 2500])
def test_chain_par_beyond_1024_equals_oracle(gpu, n):
    """N > 1,024: the row-A0 decode is the generic kernels' rows mode (states strided over the
    workgroup), the certificates read its plain rows, speculation / runs the generic CP kernel
    and cp_superseq_chain with states strided -- the oracle's chain element by element."""
    pi, a, b, off, obs = _case(n, 7, 10, 1, 12, seed=4900 + n, zeros=(1,), ones=(4,))
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs)
    assert st["parallel"], st
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj and np.array_equal(path, rp), st
    (p2, o2), st2 = _par(h, off, obs, force=1, spec=False)  # the whole chain as one serial run
    assert st2["rerun"] >= 1 and o2 == robj and np.array_equal(p2, rp), st2
    (p3, o3), st3 = _par(h, off, obs, force=2)  # speculation through the generic CP kernel
    assert st3["speculated"] >= 1 and o3 == robj and np.array_equal(p3, rp), st3


@pytest.mark.parametrize("n,force", [(300, 2), (600, 1), (1100, 3)])
def test_chain_par_wide_runs(gpu, monkeypatch, n, force):
    """The wide chain (cp_chain_wide_step: one launch per element, the states over workgroups,
    the rows in global memory; what runs above N = 10,240) as the parallel chain's serial runs
    from a start row (tuning key chain_wide_min = 1 brings it down to these N), and the whole serial chain
    with the segmented backtrack: the oracle's chain either way."""
    monkeypatch.setenv("CV_CHAIN_WIDE_MIN", "1")
    pi, a, b, off, obs = _case(n, 11, 16, 1, 30, seed=5000 + n + force, zeros=(2,), ones=(7,))
    h = cv.HMM(pi, a, b)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    (path, obj), st = _par(h, off, obs, force=force, spec=False)
    assert st["parallel"] and st["rerun"] >= 1, st
    assert obj == robj and np.array_equal(path, rp), st
    sp, sobj = _serial(h, off, obs)
    assert sobj == robj and np.array_equal(sp, rp)


@pytest.mark.parametrize("n", [300, 1100])
def test_chain_par_wide_speculation(gpu, monkeypatch, n):
    """Speculative re-decodes through the wide generic CP kernel (start offsets cp_init, last
    rows cp_last by sequence id; tuning key generic_wide_min = 1 -- the certificates keep the rows mode):
    the oracle's chain."""
    monkeypatch.setenv("CV_GENERIC_WIDE_MIN", "1")
    pi, a, b, off, obs = _case(n, 11, 16, 1, 30, seed=5100 + n, zeros=(2,), ones=(7,))
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs, force=2)
    assert st["parallel"] and st["speculated"] >= 1, st
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    assert obj == robj and np.array_equal(path, rp), st


@pytest.mark.parametrize("n,nseq", [(256, 2048), (300, 120)])
def test_chain_par_copy_overlap_knob(gpu, monkeypatch, n, nseq):
    """The paths' host copy runs on its own stream behind the last backtrack, beside the
    certificate pass (default); tuning key chain_copy_overlap = 0 copies after the certificates on the
    decode's stream.  Both return the same paths and objective (f64 trellis at N = 256, the
    generic rows mode's plain-row certificates at N = 300)."""
    if n == 256:
        c = synth.config("c4", nseq)
        pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    else:
        pi, a, b, off, obs = _case(n, 17, nseq, 1, 60, seed=4700)
    h = cv.HMM(pi, a, b)
    (path, obj), st = _par(h, off, obs)
    assert st["parallel"], st
    h.set_tuning(chain_copy_overlap=0)
    (p0, o0), st0 = _par(h, off, obs)
    assert st0["parallel"], st0
    assert obj == o0 and np.array_equal(path, p0)
    if n == 300:
        rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
        assert obj == robj and np.array_equal(path, rp)


@pytest.mark.parametrize("nseq,force", [(4096, None), (1024, 3)])
def test_chain_cert_fused_vs_pass(gpu, nseq, force):
    """The certificates computed inside the backtrack (backtrack_f64 CERT: estimated gap bounds,
    exact gaps below rho_cap) vs the separate cp_cert_f64 pass (tuning key chain_cert_fused = 0,
    exact gaps at every step): the same chain -- every element and the objective -- and the same
    certification decisions (rho_cap is above every U the walk tests)."""
    c = synth.config("c4", nseq)
    pi, a, b, off, obs = c["pi"], c["a"], c["b"], c["offsets"], c["obs"]
    h = cv.HMM(pi, a, b)
    (p1, o1), s1 = _par(h, off, obs, force=force)
    with h.tuned(chain_cert_fused=0):
        (p0, o0), s0 = _par(h, off, obs, force=force)
    assert s1["parallel"] and s0["parallel"], (s1, s0)
    assert o1 == o0 and np.array_equal(p1, p0)
    drop = ("gathered", "path_waits")
    assert {k: v for k, v in s1.items() if k not in drop} == {k: v for k, v in s0.items() if k not in drop}, (s1, s0)
    sp, sobj = _serial(h, off[:257], obs[:int(off[256])])
    (pp, op), _ = _par(h, off[:257], obs[:int(off[256])])
    assert op == sobj and np.array_equal(pp, sp)


@pytest.mark.parametrize("n,force", [(256, None), (256, 97), (100, 53), (150, 61), (40, 59)])
def test_chain_parts_schedules(gpu, n, force):
    """The parallel chain decodes a batch that spans more than a forward round (64 sequences per
    CU) in parts, each part's walk beside the next part's forward (tuning key chain_parts: 1 =
    one large part then chain_tail parts of a round / chain_tail_div, 2 = one round per part,
    0 = one part), with the later parts' observations and the path copy through pinned staging or
    pageable copies (chain_pin_obs / chain_pin_path).  Every schedule returns the serial chain's
    path and objective; forced runs (every 97th sequence uncertified) put speculative batches and
    runs on every part boundary; beside a forward the speculation runs cp_spec_psi (NP = 256,
    192, 128 and 64 here)."""
    nseq = 40000  # > 2 rounds on 256 CUs: three parts at the default schedule
    pi, a, b, off, obs = _case(n, 31, nseq, 4, 40, seed=5100 + n, zeros=(16383, 16384, 32767), ones=(24575, 24576))
    h = cv.HMM(pi, a, b)
    sp, sobj = _serial(h, off, obs)
    for keys in ({}, {"chain_parts": 0}, {"chain_parts": 2}, {"chain_tail": 3, "chain_tail_div": 4},
                 {"chain_pin_obs": 1, "chain_pin_path": 1}):
        with h.tuned(**keys):
            (path, obj), st = _par(h, off, obs, force=force)
        assert st["parallel"], (keys, st)
        if force:
            assert st["speculated"] + st["rerun"] >= nseq // 97 - 1, (keys, st)
        assert obj == sobj, (keys, obj, sobj)
        bad = np.nonzero(path != sp)[0]
        assert bad.size == 0, (keys, bad[:10], st)


@pytest.mark.parametrize("n", [3, 64, 100, 128, 150, 192, 256])
def test_chain_spec_batched_chain_kernel(gpu, n):
    """Speculative re-decodes after the forward passes run the serial chain kernel's layout
    batched, one sequence per workgroup (cp_chain_wg BATCH: row 0 at the predicted offset, the
    path backtracked through LDS-staged psi rows in the same workgroup), at every padded width;
    tuning key chain_spec_kernel = 2 keeps the generic CP kernel.  Every 2nd / 3rd sequence
    forced uncertified, ragged lengths with empty and one-element sequences and sequences longer
    than one psi staging block (> 296 rows at N = 256): both equal the oracle's chain."""
    pi, a, b, off, obs = _case(n, 21, 36, 1, 700, seed=5200 + n, zeros=(4,), ones=(9, 10))
    h = cv.HMM(pi, a, b)
    rp, robj = O.cp_superseq_f64(pi, a, b, off, obs)
    for force in (2, 3):
        for kern in (0, 2):
            with h.tuned(chain_spec_kernel=kern):
                (path, obj), st = _par(h, off, obs, force=force)
            assert st["parallel"] and st["speculated"] >= 1, (kern, st)
            assert obj == robj, (kern, force, obj, robj)
            bad = np.nonzero(path != rp)[0]
            assert bad.size == 0, (kern, force, bad[:10], st)


@pytest.mark.parametrize("n,nseq", [(64, 50), (256, 40000)])
def test_chain_bad_obs_rejected(gpu, n, nseq):
    """An observation outside [0, V) fails the call with CV_EINVAL naming the first bad element,
    on the parallel chain (range-checked by the trellis on the device: CV_SEQ_BADOBS, no host
    scan first; at 40,000 sequences the bad element sits in a later part) and on the serial chain
    (host scan), like the reference's index panic (hmm.rs:224)."""
    pi, a, b, off, obs = _case(n, 13, nseq, 2, 30, seed=5300 + n)
    h = cv.HMM(pi, a, b)
    for k in (nseq - 3, nseq // 2):
        bad = obs.copy()
        e = int(off[k]) + 1
        bad[e] = 13
        for par in (1, 0):
            with h.tuned(chain_par=par):
                with pytest.raises(cv.CVError, match=rf"obs\[{e}\] = 13 out of range"):
                    cv.decode_superseq_cp(h, off, bad)
    (path, obj), st = _par(h, off, obs)  # the handle still decodes
    assert st["parallel"]


def test_chain_config4_size(gpu):
    """The config-4-sized chain (65,536 x 512 = 33.5 M elements, N = 256: what main.rs:120 runs
    on BASELINE config 4's data) on the default schedule (parts, pinned copies through a ring of
    16 MiB chunks, speculation beside the forward passes and after them) equals the most
    conservative parallel schedule (one part, pageable copies, the generic speculation kernel,
    the separate certificate pass) bit for bit, and its first 2,048 sequences equal the serial
    chain's (the prefix's last element aside: the prefix ends its own chain there).
    CV_TEST_FULL_SERIAL=1 also runs the serial chain over the whole input (~2 minutes)."""
    c = synth.config("c4")
    off, obs = c["offsets"], c["obs"]
    h = cv.HMM(c["pi"], c["a"], c["b"])
    (p1, o1), s1 = _par(h, off, obs)
    assert s1["parallel"] and s1["certified"] > 60000, s1
    with h.tuned(chain_parts=0, chain_pin_obs=0, chain_pin_path=0, chain_spec_kernel=2, chain_cert_fused=0):
        (p0, o0), s0 = _par(h, off, obs)
    assert o1 == o0, (o1, o0)
    bad = np.nonzero(p1 != p0)[0]
    assert bad.size == 0, (bad[:10], s1, s0)
    k = 2048
    sp, _ = _serial(h, off[:k + 1], obs[:int(off[k])])
    assert np.array_equal(p1[:int(off[k]) - 1], sp[:-1])
    if os.environ.get("CV_TEST_FULL_SERIAL") == "1":
        fp, fo = _serial(h, off, obs)
        assert fo == o1 and np.array_equal(fp, p1)
