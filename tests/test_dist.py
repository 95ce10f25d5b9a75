"""CPU, world_size 2 (gloo): the batch-shard + gather-to-rank-0 path of bench.py.

Each rank decodes its contiguous shard (here with the CPU oracle standing in for the GPU
decode -- the collective logic is what is under test) and gathers paths, scores and
statuses to rank 0, which must reassemble exactly the single-process result.  On the
GPU node the same code runs with the "nccl" (RCCL over xGMI) backend.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

B, T_MAX, N, V = 37, 25, 9, 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data():
    sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
    from cviterbi import synth

    pi, a, b = synth.random_hmm(N, V, seed=3)
    rng = np.random.default_rng(3)
    off = synth.offsets_from_lengths(rng.integers(1, T_MAX, size=B))
    obs = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
    return pi, a, b, off, obs


def _worker(rank, world, port, q):
    for p in (os.path.join(ROOT, "consistent-viterbi_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import c_oracle
    from cviterbi import dist as cvd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pi, a, b, off, obs = _data()
    s0, s1, per = cvd.shard_range(B, world, rank)
    loff = cvd.shard_offsets(off, s0, s1)
    lobs = obs[off[s0]:off[s1]]
    path, score, status = c_oracle.decode_batch(pi, a, b, loff, lobs, c_oracle.VITERBI, np.float32)
    # paths are ragged: gather with the per-rank element capacity
    cap = int(max(off[min((r + 1) * per, B)] - off[min(r * per, B)] for r in range(world)))
    got = cvd.gather_to_root([torch.from_numpy(path), torch.from_numpy(score), torch.from_numpy(status)],
                             [cap, per, per], dist)
    # the packed single-collective form bench.py uses (u8 states, raw f64 scores, u8 status)
    packed = cvd.gather_packed_to_root(torch.from_numpy(path), torch.from_numpy(score),
                                       torch.from_numpy(status), N, cap, per, dist)
    if rank == 0:
        nel = [int(off[min((r + 1) * per, B)] - off[min(r * per, B)]) for r in range(world)]
        nsq = [min((r + 1) * per, B) - min(r * per, B) for r in range(world)]
        res = (cvd.assemble(got[0], nel).numpy(), cvd.assemble(got[1], nsq).numpy(),
               cvd.assemble(got[2], nsq).numpy())
        res2 = (cvd.assemble([x[0] for x in packed], nel).numpy(), cvd.assemble([x[1] for x in packed], nsq).numpy(),
                cvd.assemble([x[2] for x in packed], nsq).numpy())
        for x, y in zip(res, res2):
            assert np.array_equal(x, y.astype(x.dtype))
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shard_and_gather_matches_single_process(world):
    import c_oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pi, a, b, off, obs = _data()
    ref = c_oracle.decode_batch(pi, a, b, off, obs, c_oracle.VITERBI, np.float32)
    for x, y in zip(res, ref):
        assert np.array_equal(x, y)


def test_shard_range_covers_batch():
    sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
    from cviterbi import dist as cvd

    for total in (1, 7, 64, 65536):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s0, s1, per = cvd.shard_range(total, world, r)
                assert 0 <= s1 - s0 <= per
                seen.extend(range(s0, s1))
            assert seen == list(range(total))


# ---- config 5 exchange step: exact partials, all-reduce SUM, select -----------------------
NC = 4


def _pack_partials(mu_rows, comps, n, ncomp):
    """Test-side packing of include/cviterbi.h's partial layout from oracle max-marginals."""
    part = np.zeros((ncomp, 5 * n + 1), np.int64)
    M = (1 << 32) - 1
    for mu, c in zip(mu_rows, comps):
        part[c, 5 * n] += 1
        for s in range(n):
            if not np.isfinite(mu[s]):
                part[c, 4 * n + s] += 1
                continue
            import np_oracle as NO

            v = NO.exact_units(float(mu[s]))
            part[c, 4 * s:4 * s + 4] += [v & M, (v >> 32) & M, (v >> 64) & M, v >> 96]
    return part


def _constrained_data():
    sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
    from cviterbi import synth

    pi, a, b = synth.random_hmm(N, V, seed=11, zero_frac=0.2)
    rng = np.random.default_rng(11)
    lengths = rng.integers(1, T_MAX, size=B)
    off = synth.offsets_from_lengths(lengths)
    obs = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
    comp = np.full(len(obs), -1, np.int32)
    for k in range(B):
        if rng.random() < 0.8:
            comp[off[k] + rng.integers(0, lengths[k])] = rng.integers(0, NC)
    return pi, a, b, off, obs, comp


def _shard_mu(pi, a, b, off, obs, comp, s0, s1):
    import c_oracle

    rows, comps = [], []
    for k in range(s0, s1):
        lo, hi = off[k], off[k + 1]
        pos = np.nonzero(comp[lo:hi] >= 0)[0]
        for t in pos:
            rows.append(c_oracle.max_marginal(pi, a, b, obs[lo:hi], int(t), np.float32))
            comps.append(int(comp[lo + t]))
    return rows, comps


def _partials_worker(rank, world, port, q):
    for p in (os.path.join(ROOT, "consistent-viterbi_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    from cviterbi.decode import constrained_select
    from cviterbi import dist as cvd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pi, a, b, off, obs, comp = _constrained_data()
    s0, s1, _ = cvd.shard_range(B, world, rank)
    part = _pack_partials(*_shard_mu(pi, a, b, off, obs, comp, s0, s1), N, NC)
    red = cvd.allreduce_partials(part, dist)
    states, explored = constrained_select(N, NC, red.reshape(-1))  # host-only C-ABI call
    q.put((rank, states.tolist(), explored))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_constrained_partials_allreduce_matches_spec(world):
    """Shard partials + all-reduce + cv_constrained_select == the single-process spec's
    component states (np_oracle.constrained_decode, exact 2^-64 sums) on every rank."""
    import c_oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_partials_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pi, a, b, off, obs, comp = _constrained_data()
    spec, _ = c_oracle.constrained_forced(pi, a, b, off, obs, comp, np.float32)
    want = [spec.get(c, -1) for c in range(NC)]
    for _, states, explored in res:
        assert states == want
        assert explored == N * sum(1 for c in range(NC) if (comp == c).any())


def test_constrained_select_limb_carries():
    """cv_constrained_select reconstructs sums whose limbs carry (values near +-2^88)."""
    sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
    from cviterbi.decode import constrained_select

    M = (1 << 32) - 1
    rng = np.random.default_rng(0)
    n, ncomp = 5, 3
    part = np.zeros((ncomp, 5 * n + 1), np.int64)
    exact = np.zeros((ncomp, n), object)
    for c in range(ncomp):
        part[c, 5 * n] = 1
        for s in range(n):
            for _ in range(50):
                v = int(rng.integers(-(1 << 62), 1 << 62)) * int(rng.integers(1, 1 << 24)) - (1 << 80) * (c % 2)
                exact[c, s] += v
                part[c, 4 * s:4 * s + 4] += [v & M, (v >> 32) & M, (v >> 64) & M, v >> 96]
    part[1, 4 * n + 2] = 1  # state 2 of component 1 infeasible
    states, ex = constrained_select(n, ncomp, part.reshape(-1))
    for c in range(ncomp):
        cand = [s for s in range(n) if not (c == 1 and s == 2)]
        best = max(cand, key=lambda s: (exact[c, s], -s))
        assert states[c] == best
    assert ex == n * ncomp


def _preflight_worker(rank, world, port, corrupt, q):
    sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
    import torch.distributed as dist

    from cviterbi import dist as cvd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg = cvd.preflight(dist, None, 256, corrupt=corrupt)
    q.put((rank, ok, msg))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, None), (3, None), (8, None), (2, "gather"), (3, "allreduce")])
def test_collective_preflight(world, corrupt):
    """bench.py's RCCL first-run check (cviterbi.dist.preflight) over gloo: known values through
    the packed gather and an int64 all-reduce (incl. words above 2^53); a perturbed contribution
    on rank 1 makes EVERY rank report failure, the message naming the collective.  World 8 is
    the driver's SCALE node (round 5: a 2^60-based word overflowed int64 there)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_preflight_worker, args=(r, world, port, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get() for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(ok == (corrupt is None) for _, ok, _ in res), res
    if corrupt == "gather":
        assert "gather_packed_to_root: rank 1" in res[0][2], res
    if corrupt == "allreduce":
        assert all("all_reduce" in m or "another rank" in m for _, _, m in res), res
