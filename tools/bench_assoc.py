"""Config-4 shape decode time per reference-solver association in f64 (SURVEY.md §8a A0
notes): viterbi (row A0: trellis_fwd_f64), cp (CPSolver cp.rs:70-79), dp (DPSolver
dp.rs:127-177), decode (viterbi.rs:5-32).  NSEQ sequences of T=512 (default 8,192), device
API, one JSON line per association (sha16: digest of paths, scores and statuses: knobs
that must be bit-identical print the same digest)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

nseq = int(os.environ.get("NSEQ", "8192"))
c = synth.config("c4", nseq)
if os.environ.get("NSTATES"):  # config-4 shape with another state count (T = 512, V = 1,024)
    ns = int(os.environ["NSTATES"])
    c["pi"], c["a"], c["b"] = synth.random_hmm(ns, 1024, seed=20261015)
if os.environ.get("TRANGE"):  # ragged lengths: T ~ U[lo, hi] (seeded), iid observations
    import numpy as np
    lo, hi = (int(x) for x in os.environ["TRANGE"].split(","))
    lengths = np.random.default_rng(5).integers(lo, hi + 1, size=nseq)
    c["offsets"] = synth.offsets_from_lengths(lengths)
    c["obs"] = synth.iid_obs(1024, int(c["offsets"][-1]), 20261015)
off, obs = c["offsets"], c["obs"]
B = len(off) - 1
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
h = cv.HMM(c["pi"], c["a"], c["b"])
o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
p_d = torch.empty(len(obs), dtype=torch.int32, device=dev)
s_d = torch.empty(B, dtype=torch.float64, device=dev)
st_d = torch.empty(B, dtype=torch.uint8, device=dev)
for assoc in sys.argv[1:] or ["viterbi", "cp", "dp", "decode"]:
    def run():
        cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                               dtype="f64", assoc=assoc, rescore_f64=False, workspace_bytes=40 << 30)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = cv.last_timing(h)
    import hashlib
    digest = hashlib.sha256(p_d.cpu().numpy().tobytes() + s_d.cpu().numpy().tobytes() +
                            st_d.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"assoc": assoc, "nseq": B, "states": int(c["pi"].shape[0]), "ms": dt * 1e3,
                      "cells_per_s": B * 512 * int(c["pi"].shape[0]) / dt,
                      "kernel": t["kernel"], "fwd_ms": t["fwd_ms"], "bt_ms": t["bt_ms"], "sha16": digest}), flush=True)
