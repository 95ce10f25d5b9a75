"""Config-4 exact-f64 decode (trellis_fwd_f64) under tuning knobs: sequences per wave
(CV_T64_S, set by the caller's environment) and pipelined vs serial chunks.  Prints one JSON
line per schedule; results are bit-identical for every knob (tests/test_gpu_f64.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

nseq = int(os.environ.get("NSEQ", "65536"))
c = synth.config("c4", nseq)
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
for serial in (False, True):
    def run():
        cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                               dtype="f64", workspace_bytes=80 << 30, serial=serial)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    t = cv.last_timing(h)
    print(json.dumps({"S": os.environ.get("CV_T64_S", "auto"), "serial": serial, "nseq": B, "ms": dt * 1e3,
                      "fwd_ms": t["fwd_ms"], "bt_ms": t["bt_ms"], "launches": t["launches"],
                      "spw": t["seqs_per_wave"]}), flush=True)
