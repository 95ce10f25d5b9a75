"""Interleaved A/B timing of trellis variants on config 4 (one process, rule 24 of the
HIP guide): every variant must produce bit-identical paths/scores; prints per-variant
median wall ms and kernel ms."""
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

B = int(os.environ.get("TUNE_B", "65536"))
ROUNDS = int(os.environ.get("TUNE_ROUNDS", "3"))
VARIANTS = [
    dict(name="valu1-serial", variant="valu1", serial=True),
    dict(name="valu1-overlap", variant="valu1", serial=False),
    dict(name="valu-serial", variant="valu", serial=True),
    dict(name="valu-overlap", variant="valu", serial=False),
]
if os.environ.get("TUNE_ONLY"):
    keep = os.environ["TUNE_ONLY"].split(",")
    VARIANTS = [v for v in VARIANTS if v["name"] in keep]

c = synth.config("c4", nseq=B)
h = cv.HMM(c["pi"], c["a"], c["b"])
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
off, obs = c["offsets"], c["obs"]
o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
p_d = torch.empty(len(obs), dtype=torch.int32, device=dev)
s_d = torch.empty(B, dtype=torch.float64, device=dev)
st_d = torch.empty(B, dtype=torch.uint8, device=dev)
ref = None
res = {v["name"]: [] for v in VARIANTS}
for r in range(ROUNDS + 1):
    for v in VARIANTS:
        kw = {k: v[k] for k in v if k != "name"}
        # one untimed call first: the host-side checks below leave the GPU idle long
        # enough to drop its clocks, which would bias the next call
        cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                               workspace_bytes=48 << 30, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                               workspace_bytes=48 << 30, **kw)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        t = cv.last_timing(h)
        out = (p_d.cpu().numpy(), s_d.cpu().numpy(), st_d.cpu().numpy())
        if ref is None:
            ref = out
        else:
            for x, y in zip(out, ref):
                assert np.array_equal(x, y), f"variant {v['name']} differs"
        if r > 0:
            res[v["name"]].append((wall, t["fwd_ms"], t["bt_ms"], t["launches"], t["seqs_per_wave"], t["total_ms"]))
summary = {}
for name, rows in res.items():
    a = np.array(rows)
    summary[name] = dict(wall_ms=float(np.median(a[:, 0])), fwd_ms=float(np.median(a[:, 1])),
                         bt_ms=float(np.median(a[:, 2])), total_ms=float(np.median(a[:, 5])), launches=int(a[0, 3]), seqs_per_wave=int(a[0, 4]))
    print(f"{name:16s} wall {summary[name]['wall_ms']:8.2f} ms  fwd {summary[name]['fwd_ms']:8.2f}  "
          f"bt {summary[name]['bt_ms']:7.2f}  gpu-total {summary[name]['total_ms']:7.2f}  launches {summary[name]['launches']}", flush=True)
print(json.dumps(dict(B=B, rounds=ROUNDS, results=summary)))
