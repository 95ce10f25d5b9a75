"""Throughput of the other BASELINE.json configs on one MI355X (documentation lines for
DESIGN.md; bench.py keeps config 4 as the headline):
  c2  N=45,  V=50,000, T~U[1,128], B=4,096          (plain decode, f32 + f64 re-score)
  c3  N=64,  V=256,    T~U[32,1024], B=16,384       (plain decode, length-sorted schedule)
  c4f64, c2f64, c3f64  the same decodes in exact f64 (trellis_fwd_f64: paths and scores
      bit-identical to the f64 reference recurrence)
  c5  config 4 + one constrained position in half the sequences, K=7, exact f64 (the
      reference's precision; cv_decode_constrained_device; "c5f32": the f32 trellis;
      "c5host": the host-pointer cv_decode_constrained in f64)
Inputs resident in HBM (device APIs) except c5host, whose line includes PCIe transfers.
Prints one JSON line per config."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))
which = sys.argv[1:] or ["c2", "c3", "c5"]
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)

for name in which:
    f64 = name.endswith("f64")
    base = name.replace("f64", "").replace("f32", "").replace("host", "")
    c = synth.config(base)
    n = c["pi"].shape[0]
    off, obs = c["offsets"], c["obs"]
    B = len(off) - 1
    cells = int(off[-1]) * n
    h = cv.HMM(c["pi"], c["a"], c["b"])
    if name in ("c2", "c3") or f64:
        o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
        p_d = torch.empty(len(obs), dtype=torch.int32, device=dev)
        s_d = torch.empty(B, dtype=torch.float64, device=dev)
        st_d = torch.empty(B, dtype=torch.uint8, device=dev)

        def run():
            cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                                   dtype="f64" if f64 else "f32", workspace_bytes=80 << 30 if f64 else 0)
    elif name == "c5host":
        comp = c["component"]

        def run():
            cv.decode_constrained(h, off, obs, comp, 7)
    else:
        comp = c["component"]
        o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
        p_d = torch.empty(len(obs), dtype=torch.int32, device=dev)
        s_d = torch.empty(B, dtype=torch.float64, device=dev)
        st_d = torch.empty(B, dtype=torch.uint8, device=dev)

        def run():
            cv.decode_constrained_device(h, off, o_d, ob_d, comp, p_d, s_d, st_d, ncomp=7,
                                         stream=stream.cuda_stream, dtype="f32" if name == "c5f32" else "f64",
                                         workspace_bytes=int(os.environ.get("WS_GB", "0")) << 30)
    run()
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / REPS
    t = cv.last_timing(h)
    out = {"config": name, "states": n, "sequences": B, "elements": int(off[-1]), "ms_per_decode": dt * 1e3,
           "cells_per_s": cells / dt, "seqs_per_s": B / dt, "last_call_timing": t}
    if f64:
        npad = 64 * ((n + 63) // 64)
        # exact f64: read obs 4 B + emission column 8N, write delta column 8*NP + path 4 B
        alg = (8 * n + 8 * npad + 8) * int(off[-1]) + 8 * B
        out["alg_hbm_frac"] = alg / (t["fwd_ms"] * 1e-3) / 8.0e12 if t["fwd_ms"] else None
        out["f64_valu_frac"] = 2 * n * n * (int(off[-1]) - B) / (t["fwd_ms"] * 1e-3) / (64 * 256 * 2.4e9)
    elif name in ("c2", "c3"):
        alg = (9 * n + 8) * int(off[-1]) + 8 * B
        out["alg_hbm_frac"] = alg / (t["fwd_ms"] * 1e-3) / 8.0e12 if t["fwd_ms"] else None
        out["valu_pairs_frac"] = n * n * (int(off[-1]) - B) / (t["fwd_ms"] * 1e-3) / 3.93e13 if t["fwd_ms"] else None
    print(json.dumps(out), flush=True)
