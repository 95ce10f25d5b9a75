"""bench.py -- trellis cells/s of the MI355X Viterbi decode path (BASELINE.json metric).

Workload (BASELINE.json configs[3]): synthetic HMM with N=256
states, V=1,024 observations (bdims [32,32]), Dirichlet(1) rows in log10, iid uniform
observations from splitmix64; T=512, B=65,536 sequences per batch.  The headline `value` is
the EXACT-f64 decode (--dtype f64, the default): the reference's own arithmetic (hmm.rs:10-18
stores f64; viterbi.rs:13-18 / cp.rs:70-79), so every path and score is bit-identical to the
f64 recurrence -- the north star's "decoded state paths identical to CPU".  The f32 trellis
(BASELINE's "f32 log-prob", paths differ from f64 on ~3.7% of config-4 sequences) is timed in the same
run and reported as the extra key `f32_trellis`.
Sequences are independent, so the batch shards across ranks with no data-path collective.
For N>1 the default is strong scaling (--scaling strong: ONE 65,536-sequence batch, B/N per
GPU, BASELINE config 4 read literally); --scaling weak gives every rank its own 65,536
sequences.  One step = decode of the rank's shard (forward trellis kernel + backtrack) and,
for N>1, ONE RCCL gather (torch.distributed "nccl") of the paths (u8 states), scores and
statuses to rank 0 over xGMI -- issued on a second stream so that step k's gather overlaps
step k+1's decode (double-buffered outputs; the closing synchronize waits for the last
one).  Inputs are resident in HBM before the timed region.

After the timed region (never inside it):
* N>1: rank 0 assembles the LAST step's gathered result and compares it bit for bit (paths,
  scores, statuses) with its own single-GPU decode of the same global batch -> "verified";
* rank 0: the CPU baseline (the oracle, test infrastructure, timed on this host) whose leg
  also checks the GPU's first sequences against the oracle's f64 row-A0 decode;
* rank 0: configs 2, 3 and 5 (BASELINE.json configs[1], [2], [4]) on its GPU, inputs
  resident, as the extra key `configs` (--no-configs skips them).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak] [--dtype f64|f32]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))

N_STATES, V_OBS, T_LEN, B_TOTAL, SEED = 256, 1024, 512, 65536, 20261015
HBM_PEAK = 8.0e12            # B/s, MI355X_MICROARCH.md chip table (spec)
VALU_PAIR_PEAK = 3.93e13     # f32 (from,to) pairs/s: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / 2 VALU slots per pair
F64_PAIR_PEAK = 1.966e13     # f64 (from,to) pairs/s: 256 CU x 64 lanes x 2.4 GHz / (v_add_f64 + v_max_f64)
NOMINAL_GHZ = 2.4
# measured f64 VALU roof (tools/microbench/valu_roof_f64.hip, profiles/r06_valu_roof.txt): lane-
# pairs per clock per SIMD, each SIMD timed from its first wave's start to its last wave's end
# (s_memtime), clock from s_memtime / s_memrealtime; pure add+max pairs at 2 waves / SIMD (the
# forward's occupancy) and at 4, and the forward's own issue mix (2 dwordx4 A-row loads + 4
# ds_read_b128 broadcasts per 32 pairs) at 2 waves
VALU_ROOF_F64 = {"pairs_2w": 7.772, "pairs_4w": 7.884, "fwd_mix_2w": 7.006, "nominal": 8.0,
                 "clock_ghz": 2.393, "source": "profiles/r06_valu_roof.txt"}
SIMDS = 1024
WORKSPACE = 48 << 30         # delta workspace cap: one forward launch per step at N=1 (34.4 GB)
WORKSPACE_F64 = 80 << 30     # f64: one launch per step too (68.7 GB of f64 delta rows)
PMC_F64 = "profiles/pmc_trellis_fwd_f64_c4.json"   # committed rocprofv3 PMC summary (traffic, clock)
PMC_F32 = "profiles/pmc_trellis_fwd_c4.json"
PMC_F64_RS = "profiles/pmc_trellis_fwd_f64_rs_8192.json"  # the 8,192-sequence shard's kernel (N = 8, strong)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=B_TOTAL,
                   help="sequences per rank (weak) or in total (strong); default 65,536")
    p.add_argument("--scaling", choices=("weak", "strong"), default="strong")
    p.add_argument("--dtype", choices=("f64", "f32"), default="f64",
                   help="f64 (default): the exact-f64 trellis, paths and scores bit-identical to the "
                        "f64 reference recurrence; f32: the f32 trellis + f64 re-score of each path")
    p.add_argument("--no-f32-extra", action="store_true", help="skip the f32-trellis extra measurement")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-configs", action="store_true", help="skip the configs 2/3/5 extra measurements")
    p.add_argument("--no-verify", action="store_true", help="N>1: skip rank 0's re-decode of the global batch")
    p.add_argument("--c5-batch", type=int, default=B_TOTAL, help="N>1: sequences of the sharded config-5 leg")
    p.add_argument("--no-c5-sharded", action="store_true", help="N>1: skip the sharded config-5 leg")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="collective backend for N>1 (nccl = RCCL over xGMI; gloo only to rehearse the "
                        "multi-rank path with several ranks on one GPU)")
    return p.parse_args()


def cpu_baseline(pi, a, b, obs_rank, budget_s, gpu_first):
    """Oracle (C restatement of the reference's CPSolver forward + backtrack, f64, CP
    association = what main.rs:120 runs) timed on this host on the first k sequences of this
    rank's shard; k grows until ~budget_s of CPU work.  `value` is the single-thread rate
    (the reference is single-threaded); `all_cores` repeats it with OpenMP across sequences
    on this process's CPU share.  As the checker, the leg also decodes the
    first sequences of the shard with the oracle's f64 row-A0 recurrence (viterbi.rs:13-18)
    and compares the GPU's result for them bit for bit (`gpu_first` = (path, score, status)
    of those sequences)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import c_oracle

    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    nth = max(1, min(share, int(os.environ.get("OMP_NUM_THREADS", share)), 16))

    def run(k, threads, assoc=c_oracle.CP):
        off = np.arange(k + 1, dtype=np.int64) * T_LEN
        t0 = time.perf_counter()
        r = c_oracle.decode_batch(pi, a, b, off, obs_rank[: k * T_LEN], assoc, np.float64, nthreads=threads)
        return time.perf_counter() - t0, r

    def sample(threads, budget):
        k = 2 * threads
        dt, _ = run(k, threads)
        k = max(2 * threads, min(int(budget / max(dt / k, 1e-6)), 4096 * threads))
        return k, run(k, threads)[0]

    k, dt = sample(1, budget_s)
    cells = k * T_LEN * N_STATES
    km, dtm = sample(nth, budget_s / 2)
    check = None
    if gpu_first is not None:  # f64 decode: the oracle's f64 row-A0 result, bit for bit
        kc = len(gpu_first[1])
        _, (rp, rs, rst) = run(kc, nth, c_oracle.VITERBI)
        gp, gs, gst = gpu_first
        check = {"sequences": kc, "what": "GPU f64 decode vs oracle f64 row-A0 (viterbi.rs:13-18): paths, "
                                          "scores (bits), statuses",
                 "bit_exact": bool(np.array_equal(rp, gp) and np.array_equal(rs.view(np.int64), gs.view(np.int64))
                                   and np.array_equal(rst, gst))}
    return {"value": cells / dt, "unit": "trellis cells/s", "cores": 1, "kind": "port",
            "sample": f"first {k} sequences of config 4 (N=256, T=512), f64 CP association "
                      f"(cp.rs:63-93), oracle/cv_oracle.c single thread, {dt:.1f} s",
            "seconds": dt,
            "all_cores": {"value": km * T_LEN * N_STATES / dtm, "cores": nth, "sequences": km, "seconds": dtm,
                          "cpu": _cpu_model()},
            "check": check}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def load_pmc(f64, row_split=False):
    """The committed rocprofv3 PMC summary of the forward kernel that ran (f64: one
    65,536-sequence launch of trellis_fwd_f64, or with row_split one 8,192-sequence launch of
    trellis_fwd_f64_rs, the strong-scaling shard's kernel; f32: one 8,192-sequence launch):
    HBM bytes per decoded ELEMENT (the traffic is the delta rows written, proportional to the
    elements a launch decodes) and the effective clock (GRBM_GUI_ACTIVE over the kernel)."""
    rel = (PMC_F64_RS if row_split else PMC_F64) if f64 else PMC_F32
    p = os.path.join(ROOT, rel)
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        seqs = d.get("sequences_per_launch", B_TOTAL if f64 else 8192)
        return {"per_elem": float(d["hbm_bytes_per_launch"]) / (seqs * T_LEN),
                "clock_ghz": d.get("clock_ghz"), "source": rel + (" (" + d["source"] + ")" if "source" in d else "")}
    except Exception:
        return None


def bench_configs(dev, stream):
    """Configs 2, 3 (plain decode) and 5 (consistency-constrained decode, K=7) on this GPU in
    the default mode (exact f64), inputs resident in HBM (device APIs), wall time per decode
    after one warmup call.  Roofline fractions of the forward kernel: HBM on SURVEY.md §8(d)'s
    (9N+8) B per step, f64 VALU on N^2 pairs per step."""
    import torch

    import cviterbi as cv
    from cviterbi import synth

    out = {}
    for name, reps in (("c2", 20), ("c3", 10), ("c5", 3)):
        c = synth.config(name)
        n = c["pi"].shape[0]
        off, obs = c["offsets"], c["obs"]
        B = len(off) - 1
        elems = int(off[-1])
        h = cv.HMM(c["pi"], c["a"], c["b"], device=dev.index)
        o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
        p_d = torch.empty(elems, dtype=torch.int32, device=dev)
        s_d = torch.empty(B, dtype=torch.float64, device=dev)
        st_d = torch.empty(B, dtype=torch.uint8, device=dev)
        if name == "c5":
            comp = c["component"]

            def run():
                cv.decode_constrained_device(h, off, o_d, ob_d, comp, p_d, s_d, st_d, ncomp=7,
                                             stream=stream.cuda_stream, dtype="f64")
        else:
            def run():
                cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                                       dtype="f64", workspace_bytes=WORKSPACE_F64)
        run()
        torch.cuda.synchronize(dev)
        if int((st_d != 0).sum().item()):
            raise SystemExit(f"{name}: sequences did not decode cleanly")
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        t = cv.last_timing(h)
        pairs = n * n * (elems - B)
        d = {"workload": {"c2": "config2: N=45, V=50,000 Zipf emissions, 4,096 sequences, T in [1,128]",
                          "c3": "config3: N=64, V=256, 16,384 sequences, T in [32,1024] (length-sorted schedule)",
                          "c5": "config5: config 4 + one constrained position in half the sequences, K=7 "
                                "components, exact f64 constrained decode"}[name],
             "ms_per_decode": dt * 1e3, "cells_per_s": elems * n / dt, "seqs_per_s": B / dt, "reps": reps,
             "valu_frac_end_to_end": pairs / dt / F64_PAIR_PEAK}
        if name != "c5":
            fwd = t["fwd_ms"] * 1e-3
            d.update({"kernel": "trellis_wave_f64" if n <= 64 else "trellis_fwd_f64",
                      "kernel_ms": t["fwd_ms"], "backtrack_ms": t["bt_ms"],
                      "hbm_frac_8d": ((9 * n + 8) * elems + 8 * B) / fwd / HBM_PEAK,
                      "valu_frac": pairs / fwd / F64_PAIR_PEAK})
        else:
            d["kernel"] = ("trellis_fwd_f64 EXT (prefix + suffix passes, suffix rows kept) + exact search + "
                           "certified suffix trace (suffix_trace_f64) + backtracks")
            d["suffix_traced"] = cv.last_suffix_traced(h)  # constrained sequences needing no 2nd forward pass
        out[name] = d
        del h, o_d, ob_d, p_d, s_d, st_d
        torch.cuda.empty_cache()
    out["c4_superseq_cp"] = bench_superseq_cp(dev)
    return out


def bench_superseq_cp(dev):
    """What main.rs:120 runs on config 4's data: CPSolver over the WHOLE batch as one chained
    super-sequence (cv_decode_superseq_cp = solver kind gpu-cp, the CLI default; 33.5 M
    elements, N = 256): the parallel chain (per-sequence f64 trellis decode certified to be the
    chain's own path at the running total, host fold, serial-chain re-runs of the uncertified
    sequences), bit-identical to the serial chain.  Host arrays in and out (the host API)."""
    import cviterbi as cv
    from cviterbi import synth

    c = synth.config("c4")
    h = cv.HMM(c["pi"], c["a"], c["b"].reshape(N_STATES, 32, 32), device=dev.index)
    cv.decode_superseq_cp(h, c["offsets"][:3], c["obs"][:2 * T_LEN])  # tables
    times = []
    path = None
    for _ in range(5):  # the first full-size call also sizes the handle's chain buffers
        path = None  # the previous call's 134 MB path is the caller's to free, before the clock
        t0 = time.perf_counter()
        path, obj = cv.decode_superseq_cp(h, c["offsets"], c["obs"])
        times.append(time.perf_counter() - t0)
    st = cv.last_superseq_stats(h)
    L = int(c["offsets"][-1])
    del h
    return {"workload": "config4's 65,536 x 512 elements as ONE CPSolver super-sequence (main.rs:120, "
                        "cp.rs:63-93 over utils.rs:62-103), N=256, exact f64; host arrays (PCIe included)",
            "ms_per_solve": min(times) * 1e3, "elements_per_s": L / min(times), "objective": obj,
            "stats": st, "serial_chain_us_per_element": 3.48,
            "note": "serial chain kernel: 3.48 us/element at N=256 (profiles/r03_cp_chain.txt), i.e. ~117 s "
                    "for this input"}


def c5_sharded(dev, world, rank, dist, backend, nseq, reps, ph):
    """BASELINE config 5 (consistency-constrained decode, "8x MI355X") across the ranks:
    cviterbi.dist.constrained_decode_sharded -- each rank's contiguous shard through
    cv_decode_constrained_exchange (terms pass, ONE all-reduce of exact integer partials, the
    search, the certified-trace resume decode), then the packed gather of paths/scores/statuses
    to rank 0.  Host arrays in and out (PCIe and the host's pair scan included): end-to-end wall
    time per call, max over ranks -- not the device-API figure of configs.c5.  Rank 0 checks the
    gathered result bit for bit against its own single-process cv_decode_constrained of the
    global batch (cp.rs:95-126 semantics, main.rs:129-133 output)."""
    import torch

    import cviterbi as cv
    from cviterbi import dist as cvd
    from cviterbi import synth

    c = synth.config("c5", nseq)
    h = cv.HMM(c["pi"], c["a"], c["b"].reshape(N_STATES, 32, 32), device=dev.index)
    device = dev if backend == "nccl" else None
    call = (h, c["offsets"], c["obs"], c["component"], 7, dist)
    with ph("c5_sharded: all_reduce of the exact partials + packed gather (warmup call)"):
        got = cvd.constrained_decode_sharded(*call, device=device)  # warmup
        dist.barrier()
    with ph("c5_sharded: all_reduce of the exact partials + packed gather (timed calls)"):
        el = 0.0
        for _ in range(reps):
            got = None  # the previous call's gathered arrays are the caller's to free, before the clock
            dist.barrier()
            t0 = time.perf_counter()
            got = cvd.constrained_decode_sharded(*call, device=device)
            dist.barrier()
            el += time.perf_counter() - t0
    el /= reps
    traced = cv.last_suffix_traced(h)  # this rank's shard, before rank 0's reference decode below
    tt = torch.tensor([el], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
    with ph("c5_sharded: all_reduce MAX of the call times"):
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el = float(tt.item())
    out = None
    if rank == 0:
        ref = cv.decode_constrained(h, c["offsets"], c["obs"], c["component"], 7, dtype="f64")
        equal = all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(got, ref))
        B = len(c["offsets"]) - 1
        out = {"workload": f"config5: N=256, T=512, batch={B} sharded over {world} ranks, one constrained "
                           "position in half the sequences, K=7, exact f64; host arrays (PCIe included)",
               "ms_per_decode": el * 1e3, "cells_per_s": B * T_LEN * N_STATES / el, "seqs_per_s": B / el,
               "reps": reps, "suffix_traced_rank0": traced,
               "check": {"what": "gathered paths/scores/statuses, component states and objective == rank 0's "
                                 "single-process cv_decode_constrained of the global batch, bit for bit",
                         "equal": bool(equal)}}
    with ph("c5_sharded: barrier after rank 0's single-process check"):
        dist.barrier()
    del h
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import cviterbi as cv
    from cviterbi import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (MI355X); none visible")
    local = local % max(torch.cuda.device_count(), 1)  # == LOCAL_RANK on a node with one GPU per rank
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from cviterbi import dist as cvd

    watch = None
    if world > 1:
        # finite collective timeout (180 s, async error handling for RCCL) and a watchdog that
        # names the collective a rank is stuck in: a hang exits non-zero with that message well
        # inside the driver's 600 s limit instead of being killed there silently
        cvd.init_process_group(dist, args.backend, dev if args.backend == "nccl" else None)
        watch = cvd.CollectiveWatch(rank)

    def ph(name, timeout_s=None):
        return watch.phase(name, timeout_s) if watch else contextlib.nullcontext()

    if world > 1:  # RCCL first-run readiness: one known-value gather + one int64 all-reduce
        with ph("preflight: gather_packed_to_root + int64 all_reduce"):
            ok, msg = cvd.preflight(dist, dev if args.backend == "nccl" else None, N_STATES)
        if not ok:
            print(f"bench.py rank {rank}: collective pre-flight failed ({args.backend}): {msg}", file=sys.stderr, flush=True)
            dist.destroy_process_group()
            raise SystemExit(3)

    if args.scaling == "weak":  # every rank: its own full batch of the global N x B
        B = args.batch * world
        s0, s1, per = rank * args.batch, (rank + 1) * args.batch, args.batch
    else:
        B = args.batch
        s0, s1, per = cvd.shard_range(B, world, rank)
    nloc = s1 - s0
    f64 = args.dtype == "f64"
    pi, a, b = synth.random_hmm(N_STATES, V_OBS, seed=SEED)
    obs = synth.iid_obs(V_OBS, nloc * T_LEN, SEED, start=s0 * T_LEN)
    off = np.arange(nloc + 1, dtype=np.int64) * T_LEN

    h = cv.HMM(pi, a, b.reshape(N_STATES, 32, 32), device=local)
    stream = torch.cuda.Stream(dev)  # the decode
    comm = torch.cuda.Stream(dev)    # the gathers (RCCL waits on it), overlapping the next decode
    torch.cuda.set_stream(stream)
    off_d = torch.from_numpy(off).to(dev)
    obs_d = torch.from_numpy(obs).to(dev)
    nbuf = 2 if world > 1 else 1
    outs = [(torch.empty(nloc * T_LEN, dtype=torch.int32, device=dev),
             torch.empty(nloc, dtype=torch.float64, device=dev),
             torch.empty(nloc, dtype=torch.uint8, device=dev)) for _ in range(nbuf)]
    gathered = [None] * nbuf  # event: that buffer's gather has read it
    k_step = [0]
    last = {}  # the last step's buffer index and, on rank 0, its gathered result

    def step(dtype):
        i = k_step[0] % nbuf
        k_step[0] += 1
        path_d, score_d, status_d = outs[i]
        if gathered[i] is not None:
            stream.wait_event(gathered[i])
        cv.decode_batch_device(h, off_d, obs_d, path_d, score_d, status_d, offsets_host=off,
                               stream=stream.cuda_stream, dtype=dtype,
                               workspace_bytes=WORKSPACE_F64 if dtype == "f64" else WORKSPACE)
        last["buf"] = i
        if world > 1:  # RCCL over xGMI: decoded paths (u8 states), scores, statuses to rank 0, one gather
            done = torch.cuda.Event()
            done.record(stream)
            comm.wait_event(done)
            with torch.cuda.stream(comm):
                for t in outs[i]:
                    t.record_stream(comm)
                last["gather"] = cvd.gather_packed_to_root(path_d, score_d, status_d, N_STATES, per * T_LEN, per,
                                                           dist)
                ev = torch.cuda.Event()
                ev.record(comm)
                gathered[i] = ev

    def timed(dtype, steps, warmup):
        for _ in range(warmup):
            step(dtype)
        torch.cuda.synchronize(dev)
        bad = int(sum(int((o[2] != 0).sum().item()) for o in outs))
        if bad:
            raise SystemExit(f"rank {rank}: {bad} sequences did not decode cleanly")
        # timed region: barrier + sync on both sides, exactly K steps; kernel times summed from
        # HIP events recorded around each launch on the decode stream (read after the region)
        if world > 1:
            with ph("barrier before the timed region"):
                dist.barrier()
        torch.cuda.synchronize(dev)
        cv.timing_begin(h)
        with ph("timed steps: per-step gather_packed_to_root to rank 0 + closing barrier"):
            t0 = time.perf_counter()
            for _ in range(steps):
                step(dtype)
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            el = time.perf_counter() - t0
        kt = cv.timing_end(h)
        per_rank = [el]
        if world > 1:  # every rank's time (the SCALE record shows imbalance); the max is the job's
            per_rank = [r[0] for r in all_gather_floats([el])]
            el = max(per_rank)
        return el, kt, per_rank

    def all_gather_floats(vals):
        t = torch.tensor(vals, dtype=torch.float64, device="cpu" if args.backend == "gloo" else dev)
        parts = [torch.zeros_like(t) for _ in range(world)]
        with ph("all_gather of per-rank timings"):
            dist.all_gather(parts, t)
        return [p.cpu().tolist() for p in parts]

    el, kt, per_rank_s = timed(args.dtype, args.steps, args.warmup)
    fwd_ms, bt_ms, launches = kt["fwd_ms"], kt["bt_ms"], kt["launches"]
    # every rank's shard kernel times (HIP events on its decode stream): a SCALE line's gap to
    # linear shows up here as forward / backtrack vs host and gather time
    kms = [fwd_ms / args.steps, bt_ms / args.steps]
    kms_ranks = all_gather_floats(kms) if world > 1 else [kms]
    spw = kt.get("seqs_per_wave", 8)  # the layout of the timed run (before the f32 extra)
    # this rank's first sequences as the timed run decoded them (for the CPU baseline's check)
    kc = min(64, nloc)
    pb, sb, stb = outs[last["buf"]]
    first = (pb[: kc * T_LEN].cpu().numpy(), sb[:kc].cpu().numpy(), stb[:kc].cpu().numpy()) if f64 else None

    # ---- rank 0 re-decodes the global batch on its own GPU: the gathered last step must equal it
    verify = None
    if world > 1 and not args.no_verify:
        ok = True
        if rank == 0:
            parts = last["gather"]
            ns = [cvd.shard_range(B, world, r)[1] - cvd.shard_range(B, world, r)[0] if args.scaling == "strong"
                  else args.batch for r in range(world)]
            gp = cvd.assemble([x[0] for x in parts], [n * T_LEN for n in ns])
            gs = cvd.assemble([x[1] for x in parts], ns)
            gst = cvd.assemble([x[2] for x in parts], ns)
            obs_g = torch.from_numpy(synth.iid_obs(V_OBS, B * T_LEN, SEED)).to(dev)
            off_gh = np.arange(B + 1, dtype=np.int64) * T_LEN
            rp = torch.empty(B * T_LEN, dtype=torch.int32, device=dev)
            rs = torch.empty(B, dtype=torch.float64, device=dev)
            rst = torch.empty(B, dtype=torch.uint8, device=dev)
            # its own handle: the global batch's workspace (68.7 GB of f64 rows) is freed with it
            hv = cv.HMM(pi, a, b.reshape(N_STATES, 32, 32), device=local)
            cv.decode_batch_device(hv, torch.from_numpy(off_gh).to(dev), obs_g, rp, rs, rst, offsets_host=off_gh,
                                   stream=stream.cuda_stream, dtype=args.dtype,
                                   workspace_bytes=WORKSPACE_F64 if f64 else WORKSPACE)
            torch.cuda.synchronize(dev)
            del hv
            ok = bool(torch.equal(gp.to(dev), rp) and torch.equal(gs.to(dev).view(torch.int64), rs.view(torch.int64))
                      and torch.equal(gst.to(dev), rst))
            verify = {"what": "last step's gathered paths/scores/statuses (all ranks) == rank 0's single-GPU "
                              "decode of the same global batch, bit for bit", "sequences": B, "equal": ok}
            del obs_g, rp, rs, rst
        with ph("barrier after rank 0's verify decode"):
            dist.barrier()

    f32_extra = None
    if f64 and not args.no_f32_extra:
        p64 = outs[last["buf"]][0].clone()  # the f64 (reference-exact) paths of this rank's shard
        el32, kt32, _ = timed("f32", args.steps, args.warmup)
        # measured, not quoted: the share of this rank's sequences whose f32 path differs from
        # the f64 one (the f32 mode's cost in parity; the f64 headline is the reference's)
        p32 = outs[last["buf"]][0]
        differ = (p32.view(nloc, T_LEN) != p64.view(nloc, T_LEN)).any(dim=1)
        ndiff = int(differ.sum().item())
        del p64
        f32_extra = {"value": B * T_LEN * N_STATES * args.steps / el32, "unit": "trellis cells/s",
                     "ms_per_step": el32 * 1e3 / args.steps,
                     "kernel": "trellis_fwd2_f32<256>", "kernel_ms_per_launch": kt32["fwd_ms"] / max(kt32["launches"], 1),
                     "paths_differ_frac": ndiff / max(nloc, 1), "paths_differ": ndiff, "sequences_compared": nloc,
                     "note": "f32 log-probs (BASELINE config 4 literally), f64 re-score of each path; "
                             "paths_differ_frac = share of this rank's sequences whose f32 path differs from the "
                             "f64 (reference-exact) path of the same batch"}

    c5s = None
    if world > 1 and not args.no_c5_sharded:
        c5s = c5_sharded(dev, world, rank, dist, args.backend, args.c5_batch, 2, ph)

    # per-rank peak device memory: torch's tensors + the library's tables and workspaces
    mem = [torch.cuda.max_memory_allocated(dev) / 1e9, cv.device_memory()["peak"] / 1e9]
    mem_ranks = all_gather_floats(mem) if world > 1 else [mem]

    cells_total = B * T_LEN * N_STATES * args.steps
    value = cells_total / el
    ms_step = el * 1e3 / args.steps
    # roofline of the dominant kernel (forward trellis) on THIS rank, per launch
    steps_rank = nloc * T_LEN
    lps = launches / args.steps  # forward launches per step
    fwd_launch_s = fwd_ms / max(launches, 1) * 1e-3
    # read obs 4 B + emission column 4N, write delta column 4N + psi column N
    # (u8) + path 4 B = (9N + 8) B per sequence step, + 8 B of score per sequence
    alg_8d = ((9 * N_STATES + 8) * steps_rank + 8 * nloc) / lps
    alg_read_8d = (4 * N_STATES + 4) * steps_rank / lps
    # the f64 path's own bytes: f64 emission column 8N in, f64 delta column 8N out
    alg_f64 = ((16 * N_STATES + 8) * steps_rank + 8 * nloc) / lps
    achieved = alg_8d / fwd_launch_s
    pairs_per_launch = N_STATES * N_STATES * (T_LEN - 1) * nloc / lps
    # spw 4 = the pair-of-waves small-batch layout with S = 8, run as the row split
    # (trellis_fwd_f64_rs, four pairs per workgroup) on equal-length batches like this one
    row_split = f64 and spw == 4
    pmc = load_pmc(f64, row_split)
    traffic = pmc["per_elem"] * steps_rank / lps if pmc else None
    kname = ("trellis_fwd_f64<C=4,S=8>" if spw == 8 else "trellis_fwd_f64_rs<8> (row-split pairs, S=8)" if row_split
             else "trellis_fwd_f64<C=2,S=%d,W=2>" % (2 * spw)) if f64 else "trellis_fwd2_f32<256>"
    pair_peak = F64_PAIR_PEAK if f64 else VALU_PAIR_PEAK
    valu_frac = pairs_per_launch / fwd_launch_s / pair_peak
    valu = {"achieved_pairs_per_s": pairs_per_launch / fwd_launch_s, "peak_pairs_per_s": pair_peak,
            "frac": valu_frac, "peak_basis": f"nominal {NOMINAL_GHZ} GHz"}
    if pmc and pmc.get("clock_ghz"):
        valu.update({"clock_ghz_pmc": pmc["clock_ghz"], "frac_at_pmc_clock": valu_frac * NOMINAL_GHZ / pmc["clock_ghz"],
                     "clock_source": pmc["source"] + ": GRBM_GUI_ACTIVE / 8 XCDs over the kernel duration"})
        if f64:  # against the MEASURED roof, per clock
            per_clk = pairs_per_launch / fwd_launch_s / (SIMDS * pmc["clock_ghz"] * 1e9)
            valu["measured_roof"] = {
                "achieved_lane_pairs_per_clk_per_simd": per_clk,
                "roof_lane_pairs_per_clk_per_simd": VALU_ROOF_F64["pairs_2w"],
                "frac": per_clk / VALU_ROOF_F64["pairs_2w"],
                "frac_of_4_wave_roof": per_clk / VALU_ROOF_F64["pairs_4w"],
                "frac_of_fwd_mix_roof": per_clk / VALU_ROOF_F64["fwd_mix_2w"],
                "basis": "pure v_add_f64 + v_max_f64 pairs at 2 waves per SIMD (the forward's occupancy), per-SIMD "
                         "first-start to last-end s_memtime spans; the kernel's rate per clock at the PMC clock",
                "source": VALU_ROOF_F64["source"]}
    out = {
        "metric": "trellis cells/s (N*T*batch), N=256 T=512 batch=65536",
        "value": value,
        "unit": "trellis cells/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (Dirichlet(1) log10 HMM, splitmix64 iid observations; SURVEY.md §8d config 4)",
        "config": {"workload": "config4: N=256 states, V=1024, T=512, " +
                               (f"batch={args.batch} per rank (weak scaling, global {B})" if args.scaling == "weak" else
                                f"batch={B} sharded over {world} ranks (strong scaling)") +
                               (", exact-f64 row-A0 trellis + backtrack (paths/scores bit-identical to the f64 "
                                "reference recurrence)" if f64 else
                                ", f32 row-A0 trellis + backtrack + f64 re-score") +
                               ((", RCCL gather to rank 0 (overlapped with the next step)" if args.backend == "nccl" else
                                 ", gloo gather to rank 0 (rehearsal: ranks may share a GPU)") if world > 1 else ""),
                   "global_batch": B, "seq_len": T_LEN, "states": N_STATES, "parallelism": f"batch-shard x{world}"},
        "seqs_per_s": B * args.steps / el,
        "roofline": {"bound": "valu",
                     "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
                     "traffic": traffic,
                     "traffic_source": (pmc["source"] + ": rocprofv3 FETCH_SIZE x2 (gfx950) + WRITE_SIZE, scaled "
                                        "per decoded element") if pmc else None,
                     "basis": "achieved/frac: HBM roof on SURVEY.md §8(d)'s algorithmic bytes ((9N+8) B per "
                              "sequence step + 8 B per sequence) / the kernel's HIP-event time per launch; the "
                              "binding roof is the f64 VALU one (roofs.valu)" if f64 else
                              "achieved/frac: HBM roof on SURVEY.md §8(d)'s algorithmic bytes; binding roof: VALU",
                     "kernel": kname,
                     "kernel_ms_per_launch": fwd_launch_s * 1e3,
                     "alg_bytes_per_launch": alg_8d,
                     "read_only_frac": alg_read_8d / fwd_launch_s / HBM_PEAK,
                     "frac_f64_bytes": alg_f64 / fwd_launch_s / HBM_PEAK if f64 else None,
                     "roofs": {"hbm": {"achieved_GBps": achieved / 1e9, "peak_GBps": HBM_PEAK / 1e9,
                                       "frac": achieved / HBM_PEAK},
                               "valu": valu}},
        "kernel_ms_per_step": {"forward": fwd_ms / args.steps, "backtrack_rescore": bt_ms / args.steps},
        "per_rank": {"ms_per_step": [x * 1e3 / args.steps for x in per_rank_s],
                     "min_ms_per_step": min(per_rank_s) * 1e3 / args.steps,
                     "max_ms_per_step": max(per_rank_s) * 1e3 / args.steps,
                     "kernel_ms_per_step": [{"forward": k[0], "backtrack": k[1]} for k in kms_ranks],
                     "preflight": "gather_packed_to_root + int64 all_reduce checked" if world > 1 else None,
                     "peak_device_gb": [{"torch": m[0], "library": m[1]} for m in mem_ranks],
                     "note": "timed region of the headline dtype; peak device memory over the whole run so far "
                             "(decode workspaces, rank 0's verify decode, the sharded config-5 leg)"},
    }
    if f32_extra is not None:
        out["f32_trellis"] = f32_extra
    if verify is not None:
        out["multi_gpu_check"] = verify
    if c5s is not None:
        out["c5_sharded"] = c5s
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pi, a, b, obs, args.cpu_seconds, first)
        out["cpu_baseline"]["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0 and not args.no_configs:
        out["configs"] = bench_configs(dev, stream)
    checks = []
    if verify is not None:
        checks.append(verify["equal"])
    if c5s is not None:
        checks.append(c5s["check"]["equal"])
    if out.get("cpu_baseline", {}).get("check"):
        checks.append(out["cpu_baseline"]["check"]["bit_exact"])
    out["verified"] = bool(checks) and all(checks)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        with ph("final barrier (rank 0's CPU baseline and configs)"):
            dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and checks and not all(checks):
        raise SystemExit("bench.py: the decoded result failed its check (see multi_gpu_check / cpu_baseline.check)")


if __name__ == "__main__":
    main()
