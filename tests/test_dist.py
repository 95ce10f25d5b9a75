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
    if rank == 0:
        nel = [int(off[min((r + 1) * per, B)] - off[min(r * per, B)]) for r in range(world)]
        nsq = [min((r + 1) * per, B) - min(r * per, B) for r in range(world)]
        q.put((cvd.assemble(got[0], nel).numpy(), cvd.assemble(got[1], nsq).numpy(),
               cvd.assemble(got[2], nsq).numpy()))
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
