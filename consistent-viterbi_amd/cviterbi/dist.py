"""Batch sharding across GPUs and the gather of decoded paths.

The unconstrained decode is independent per sequence, so the batch is split into
contiguous shards of ceil(B/world) sequences, one per rank (one process per GPU); the
HMM is replicated.  The only collective is the gather of paths, scores and statuses to
rank 0 -- RCCL over xGMI with the "nccl" backend on the GPU node, gloo in CPU tests.

The consistency-constrained decode (config 5) has one real exchange step: the unary and
pairwise component terms.  Every rank derives the same pair layout from the full batch
(cv_constrained_pairs), reduces its shard to exact integer partials (int64 words,
include/cviterbi.h CV_PARTIAL_WORDS), one all-reduce SUM combines them -- bit-identical to
the single-process choice whatever the shard boundaries -- and every rank runs the same
exact search and decodes its own shard.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from contextlib import contextmanager
from datetime import timedelta

import numpy as np

# collective timeout of bench.py's process group: well inside the driver's 600 s bench limit,
# far above any legitimate wait (rank 0's verify decode is a few seconds)
COLLECTIVE_TIMEOUT_S = 180.0


def init_process_group(dist, backend, device=None, timeout_s=COLLECTIVE_TIMEOUT_S, **kw):
    """init_process_group with a finite collective timeout and, for "nccl" (RCCL), async error
    handling on: a collective that never completes raises (gloo) or tears the process down
    (the RCCL watchdog) after `timeout_s` instead of the default 10 minutes."""
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group("nccl", device_id=device, timeout=timedelta(seconds=timeout_s), **kw)
    else:
        dist.init_process_group(backend, timeout=timedelta(seconds=timeout_s), **kw)


class CollectiveWatch:
    """Names the collective a rank is stuck in and ends the process when it overruns.

    `with watch.phase("gather_packed_to_root (step results)"):` marks the code between as one
    collective phase; a daemon thread checks every `poll_s`, and when a phase has run longer
    than `timeout_s` it prints "<who> rank R: collective '<phase>' did not complete within N s"
    to stderr and exits the process with `exit_code` (os._exit: a rank blocked inside a
    collective cannot unwind).  A collective that FAILS instead raises inside the phase; the
    phase re-raises it as RuntimeError with the same naming.  Works for gloo and nccl alike,
    independent of the backend's own timeout (which `init_process_group` above also sets)."""

    def __init__(self, rank, timeout_s=COLLECTIVE_TIMEOUT_S, who="bench.py", exit_code=4, poll_s=1.0):
        self.rank, self.timeout_s, self.who, self.exit_code = rank, float(timeout_s), who, exit_code
        self._cur = None  # (name, start, limit)
        self._lock = threading.Lock()
        self._t = threading.Thread(target=self._run, args=(poll_s,), daemon=True)
        self._t.start()

    def _run(self, poll_s):
        while True:
            time.sleep(poll_s)
            with self._lock:
                cur = self._cur
            if cur and time.monotonic() - cur[1] > cur[2]:
                print(f"{self.who} rank {self.rank}: collective '{cur[0]}' did not complete within "
                      f"{cur[2]:.0f} s (a peer rank never entered it or the transport hangs); exiting",
                      file=sys.stderr, flush=True)
                os._exit(self.exit_code)

    @contextmanager
    def phase(self, name, timeout_s=None):
        """timeout_s: this phase's own limit (default: the watch's)."""
        with self._lock:
            self._cur = (name, time.monotonic(), float(timeout_s or self.timeout_s))
        try:
            yield
        except Exception as e:  # a backend error (gloo timeout, RCCL abort): say which collective
            raise RuntimeError(f"{self.who} rank {self.rank}: collective '{name}' failed: {e}") from e
        finally:
            with self._lock:
                self._cur = None


def shard_range(total: int, world: int, rank: int):
    """Contiguous shard [s0, s1) of `total` sequences for `rank` (last shards may be short)."""
    per = (total + world - 1) // world
    return min(rank * per, total), min((rank + 1) * per, total), per


def shard_offsets(offsets, s0, s1):
    """Rebase the CSR offsets of sequences [s0, s1) to start at 0."""
    offsets = np.asarray(offsets, np.int64)
    return offsets[s0:s1 + 1] - offsets[s0]


def gather_to_root(tensors, per_sizes, dist, device=None):
    """Gather each rank's tensors to rank 0, padded to the per-rank capacity `per_sizes`
    (one entry per tensor).  Returns, on rank 0, lists of per-rank tensors trimmed by
    the caller; None elsewhere."""
    import torch

    world = dist.get_world_size()
    rank = dist.get_rank()
    out = []
    for x, cap in zip(tensors, per_sizes):
        if x.numel() != cap:
            y = torch.zeros(cap, dtype=x.dtype, device=x.device)
            y[: x.numel()] = x
            x = y
        lst = [torch.empty(cap, dtype=x.dtype, device=x.device) for _ in range(world)] if rank == 0 else None
        dist.gather(x, lst, dst=0)
        out.append(lst)
    return out if rank == 0 else None


def gather_packed_to_root(path, score, status, nstates, elem_cap, seq_cap, dist):
    """ONE gather of a rank's decode result to rank 0: states as u8 when nstates <= 256 (else
    int32), f64 scores as raw bytes, u8 statuses, packed into one byte buffer padded to the
    per-rank capacities (elem_cap path entries, seq_cap sequences).  At config 4 / 8 ranks
    that is 4.2 MB per rank instead of 16.8 MB of int32 paths in three collectives.
    Returns on rank 0 a list over ranks of (path int32, score f64, status u8) padded to the
    capacities (trim with `assemble`); None elsewhere."""
    import torch

    pdt = torch.uint8 if nstates <= 256 else torch.int32
    psz = 1 if pdt == torch.uint8 else 4
    dev = path.device
    nbytes = seq_cap * 8 + elem_cap * psz + seq_cap  # [scores | paths | statuses], views stay aligned
    buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    buf[: score.numel() * 8] = score.contiguous().view(torch.uint8)
    o = seq_cap * 8
    buf[o: o + path.numel() * psz] = path.to(pdt).view(torch.uint8)
    o += elem_cap * psz
    buf[o: o + status.numel()] = status.to(torch.uint8)
    rank = dist.get_rank()
    # gloo gathers host tensors only (CPU tests, the 1-GPU rehearsal of bench.py)
    host = dist.get_backend() == "gloo" and buf.device.type != "cpu"
    src = buf.cpu() if host else buf
    lst = [torch.empty(nbytes, dtype=torch.uint8, device=src.device) for _ in range(dist.get_world_size())] \
        if rank == 0 else None
    dist.gather(src, lst, dst=0)
    if rank != 0:
        return None
    if host:
        lst = [b.to(dev) for b in lst]
    out = []
    for b in lst:
        sc = b[: seq_cap * 8].view(torch.float64)
        p = b[seq_cap * 8: seq_cap * 8 + elem_cap * psz].view(pdt).to(torch.int32)
        st = b[seq_cap * 8 + elem_cap * psz:]
        out.append((p, sc, st))
    return out


def assemble(parts, lengths):
    """Concatenate per-rank gathered buffers, keeping the first lengths[r] entries of each."""
    import torch

    return torch.cat([p[:n] for p, n in zip(parts, lengths)])


def allreduce_partials(partials, dist, device=None):
    """All-reduce SUM of int64 constrained partials (CV_PARTIAL_WORDS); returns numpy int64.
    Integer sums: exact and independent of reduction order."""
    import torch

    t = torch.from_numpy(np.ascontiguousarray(partials, np.int64)).to(device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def constrained_decode_sharded(hmm, offsets, obs, component, ncomp, dist, device=None, dtype="f64"):
    """Config 5 across ranks: shard sequences, exact partials, one all-reduce, select,
    per-shard final decode (cv_decode_constrained_exchange), gather to rank 0.  Returns (path, score, status, comp_state,
    objective) on rank 0 and (None, None, None, comp_state, None) elsewhere."""
    import torch

    from .decode import constrained_pairs, decode_constrained_exchange

    offsets = np.asarray(offsets, np.int64)
    world, rank = dist.get_world_size(), dist.get_rank()
    B = len(offsets) - 1
    s0, s1, per = shard_range(B, world, rank)
    lo, hi = int(offsets[s0]), int(offsets[s1])
    off = shard_offsets(offsets, s0, s1)
    ob = np.asarray(obs, np.int32)[lo:hi]
    cp = np.asarray(component, np.int32)[lo:hi]
    pairs = constrained_pairs(offsets, component, ncomp)  # full batch: the same layout on every rank
    # partials -> all-reduce SUM (the callback) -> search -> final decode, in one library call,
    # so the shard's decode reuses its terms pass's prefix rows (the resume flow)
    path, score, status, states, _, _ = decode_constrained_exchange(
        hmm, off, ob, cp, ncomp, pairs, exchange=lambda w: allreduce_partials(w, dist, device), dtype=dtype)
    # gather: sequence counts and element counts differ per rank -> pad to capacities
    counts = torch.tensor([s1 - s0, hi - lo], dtype=torch.int64, device=device or "cpu")
    allc = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(allc, counts)
    ecap = max(int(c[1]) for c in allc)
    dev = device or "cpu"
    # ONE packed collective (u8 states when N <= 256, raw f64 scores, u8 statuses), as bench.py
    g = gather_packed_to_root(torch.from_numpy(path).to(dev), torch.from_numpy(score).to(dev),
                              torch.from_numpy(status.astype(np.uint8)).to(dev), hmm.nstates(), ecap, per, dist)
    if rank != 0:
        return None, None, None, states, None
    ns = [int(c[0]) for c in allc]
    ne = [int(c[1]) for c in allc]
    path = assemble([x[0] for x in g], ne).cpu().numpy()
    score = assemble([x[1] for x in g], ns).cpu().numpy()
    status = assemble([x[2] for x in g], ns).cpu().numpy().astype(np.uint8)
    # sequential sum in sequence order, as cv_decode_constrained does (CV_SEQ_INFEASIBLE = 1)
    objective = float(np.cumsum(np.where(status == 1, -np.inf, score))[-1]) if B else 0.0
    return path, score, status, states, objective


def preflight(dist, device=None, nstates=256, corrupt=None):
    """First-run check of the two collectives bench.py relies on, right after
    init_process_group: ONE packed gather (gather_packed_to_root, the decode's result path) of
    known per-rank values, and ONE int64 all-reduce SUM (allreduce_partials, the config-5
    exchange) of known words incl. values above 2^53.  Every rank learns the outcome (an
    all-reduce MIN of the per-rank verdicts), so all ranks fail together.  Returns
    (True, "") or (False, message naming the collective and the rank that saw it fail).
    corrupt: test hook ("gather" / "allreduce") that perturbs rank 1's contribution.
    Contract: main.rs:129-133 writes one output line per element; a gather that silently
    dropped or reordered a rank would break it, so the bench exits before timing anything."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    dev = device or "cpu"
    seq_cap, elem_cap = 3, 7
    n_el = elem_cap - (rank % 2)  # ragged: odd ranks one element short (padded by the gather)
    path = torch.tensor([(rank * 13 + k) % nstates for k in range(n_el)], dtype=torch.int32, device=dev)
    score = torch.tensor([-(rank + 0.25) * 10.0 ** k for k in range(seq_cap)], dtype=torch.float64, device=dev)
    status = torch.tensor([(rank + k) % 4 for k in range(seq_cap)], dtype=torch.uint8, device=dev)
    if corrupt == "gather" and rank == 1:
        path = path.clone()
        path[0] += 1
    problems = []
    g = gather_packed_to_root(path, score, status, nstates, elem_cap, seq_cap, dist)
    if rank == 0:
        for r, (p, sc, st) in enumerate(g):
            ne = elem_cap - (r % 2)
            want_p = torch.tensor([(r * 13 + k) % nstates for k in range(ne)], dtype=torch.int32)
            want_s = torch.tensor([-(r + 0.25) * 10.0 ** k for k in range(seq_cap)], dtype=torch.float64)
            want_st = torch.tensor([(r + k) % 4 for k in range(seq_cap)], dtype=torch.uint8)
            if not (torch.equal(p[:ne].cpu(), want_p) and torch.equal(sc.cpu().view(torch.int64), want_s.view(torch.int64))
                    and torch.equal(st.cpu(), want_st)):
                problems.append(f"gather_packed_to_root: rank {r}'s part arrived wrong at rank 0")
    # above 2^53 (not representable in f64) but summing within int64 for up to 32 ranks
    words = np.array([rank + 1, (1 << 57) + rank, -(1 << 55) - rank, 7 * rank - 3], np.int64)
    if corrupt == "allreduce" and rank == 1:
        words[1] += 1
    got = allreduce_partials(words, dist, dev if dev != "cpu" else None)
    rs = np.arange(world, dtype=np.int64)
    want = np.array([(rs + 1).sum(), (1 << 57) * world + rs.sum(), -(1 << 55) * world - rs.sum(), (7 * rs - 3).sum()],
                    np.int64)
    if not np.array_equal(got, want):
        problems.append(f"all_reduce(int64 SUM): rank {rank} got {got.tolist()}, expected {want.tolist()}")
    ok = torch.tensor([0 if problems else 1], dtype=torch.int64, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 1:
        return True, ""
    return False, "; ".join(problems) if problems else f"rank {rank}: another rank's collective check failed"
