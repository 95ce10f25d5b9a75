"""GPU: the certified suffix trace of the constrained decode's resume flow (f64; DESIGN.md §3,
kernels/trellis64.hip suffix_trace_f64).  For one-position sequences the forced path after
t_1 is read off the terms pass's stored suffix rows, with a rounding-error margin that proves
it is the forced forward decode's own path; a step inside the margin (near ties) sends the
sequence to the forward pass.  Every case: bit-identical to the same call with the trace off
(CV_NO_TRACE=1: the second forward pass for every constrained sequence), host and device
APIs, and the trace must actually have run (cv_last_suffix_traced)."""
import numpy as np
import pytest

import cviterbi as cv
from cviterbi import synth

pytestmark = pytest.mark.gpu

FIELDS = ("path", "score", "status", "states", "objective")


def _case(n, seed, nseq=64, tmax=48, quant=None, bad_obs=False, multi=False):
    pi, a, b = synth.random_hmm(n, 9, seed=seed)
    if quant:  # dyadic grid: exact ties everywhere (the trace must fall back at those steps)
        pi, a, b = (np.where(np.isfinite(x), np.round(x * quant) / quant, x) for x in (pi, a, b))
    if bad_obs:
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
        if rng.random() < 0.75:
            k = rng.integers(1, 3) if multi else 1
            pos = rng.choice(lens[s], size=min(k, lens[s]), replace=False)
            comp[off[s] + pos] = rng.integers(0, 4, size=len(pos))
    comp[off[0]] = 0                # t_1 = first element (length-1 sequence)
    comp[off[2] + lens[2] - 1] = 1  # t_1 = last element
    comp[off[3]] = 2                # t_1 = 0 of a longer sequence
    return pi, a, b, off, obs, comp


def _one_position(off, comp):
    return sum(int((comp[off[s]:off[s + 1]] >= 0).sum() == 1) for s in range(len(off) - 1))


def _both(h, off, obs, comp, ncomp, monkeypatch):
    """(trace on, trace off) results of the host API, plus the trace count of the first."""
    h.set_tuning(no_trace=0)
    got = cv.decode_constrained(h, off, obs, comp, ncomp=ncomp, dtype="f64")
    traced = cv.last_suffix_traced(h)
    h.set_tuning(no_trace=1)
    ref = cv.decode_constrained(h, off, obs, comp, ncomp=ncomp, dtype="f64")
    assert cv.last_suffix_traced(h) == 0
    h.set_tuning(no_trace=0)
    return got, ref, traced


def _device(h, off, obs, comp, ncomp):
    import torch
    dev = torch.device("cuda", 0)
    outs = (torch.full((int(off[-1]),), 7, dtype=torch.int32, device=dev),
            torch.empty(len(off) - 1, dtype=torch.float64, device=dev),
            torch.empty(len(off) - 1, dtype=torch.uint8, device=dev))
    states, obj = cv.decode_constrained_device(h, off, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev),
                                               comp, *outs, ncomp=ncomp, dtype="f64")
    return (outs[0].cpu().numpy(), outs[1].cpu().numpy(), outs[2].cpu().numpy(), states, obj)


def _same(got, ref):
    for x, y, what in zip(got, ref, FIELDS):
        x, y = np.asarray(x), np.asarray(y)
        if what == "objective" and np.isinf(y):
            assert np.isinf(x) and x == y, what
        else:
            assert np.array_equal(x, y), what


@pytest.mark.parametrize("n,seed,bad", [(256, 1, False), (256, 2, True), (192, 3, False), (128, 4, False),
                                        (64, 5, False), (45, 6, True), (5, 7, False)])
def test_trace_equals_forward_pass(gpu, monkeypatch, n, seed, bad):
    pi, a, b, off, obs, comp = _case(n, seed, bad_obs=bad)
    h = cv.HMM(pi, a, b)
    got, ref, traced = _both(h, off, obs, comp, 5, monkeypatch)
    _same(got, ref)
    assert 0 < traced <= _one_position(off, comp)
    if bad:
        assert (ref[2] == 1).any()
    _same(_device(h, off, obs, comp, 5), ref)
    assert cv.last_suffix_traced(h) == traced


@pytest.mark.parametrize("quant", [4, 16])
def test_trace_ties_fall_back(gpu, monkeypatch, quant):
    """Dyadic models: exact ties on the paths send sequences to the forward pass (first-index
    rule); the mix of traced and re-decoded sequences is still bit-identical."""
    pi, a, b, off, obs, comp = _case(48, 11 + quant, nseq=96, quant=quant)
    h = cv.HMM(pi, a, b)
    got, ref, traced = _both(h, off, obs, comp, 5, monkeypatch)
    _same(got, ref)
    assert traced < _one_position(off, comp)  # some sequences fell back
    _same(_device(h, off, obs, comp, 5), ref)


def test_trace_multi_position_untouched(gpu, monkeypatch):
    """Sequences with several constrained elements keep the forward pass; the one-position
    ones beside them are traced."""
    pi, a, b, off, obs, comp = _case(256, 21, nseq=80, multi=True)
    h = cv.HMM(pi, a, b)
    got, ref, traced = _both(h, off, obs, comp, 5, monkeypatch)
    _same(got, ref)
    assert 0 < traced <= _one_position(off, comp)


def test_trace_positive_model_off(gpu, monkeypatch):
    """A model with a positive entry is outside the trace's bound (all terms <= 0): no trace."""
    pi, a, b, off, obs, comp = _case(64, 31)
    b = b.copy()
    b[0, 0] = 0.5
    h = cv.HMM(pi, a, b)
    got, ref, traced = _both(h, off, obs, comp, 5, monkeypatch)
    assert traced == 0
    _same(got, ref)


def test_trace_vs_oracle(gpu):
    """The traced decode against the oracle spec directly (N = 256, one position each):
    component states, paths and statuses equal, scores bit for bit (test_gpu_constrained._check)."""
    from test_gpu_constrained import _check
    pi, a, b, off, obs, comp = _case(256, 41, nseq=24, tmax=30)
    h = cv.HMM(pi, a, b)
    _check(h, pi, a, b, off, obs, comp, "f64")
    assert cv.last_suffix_traced(h) > 0


def test_trace_config5_full(gpu, monkeypatch):
    """Config 5 at full size, device API: trace on == trace off bit for bit, and nearly every
    constrained sequence is traced."""
    c = synth.config("c5")
    pi, a, b, off, obs, comp = c["pi"], c["a"], c["b"], c["offsets"], c["obs"], c["component"]
    h = cv.HMM(pi, a, b.reshape(256, 32, 32))
    h.set_tuning(no_trace=1)
    ref = _device(h, off, obs, comp, 7)
    h.set_tuning(no_trace=0)
    got = _device(h, off, obs, comp, 7)
    traced = cv.last_suffix_traced(h)
    _same(got, ref)
    ncon = _one_position(off, comp)
    assert traced >= 0.99 * ncon, (traced, ncon)
