"""f64 batch decode (forward + backtrack) of the first n config-4 sequences, per launch, for the
parallel chain's part sizing: python tools/bench_batch_sizes.py n1[:key=v,...] n2 ...
(tuning keys per size after a colon, e.g. 16384:t64_s=4).  Prints fwd / bt ms (HIP events,
median of REPS) and the forward's microseconds per sequence."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
c = synth.config("c4")
h = cv.HMM(c["pi"], c["a"], c["b"])
off_all, obs_all = c["offsets"], c["obs"]
for arg in sys.argv[1:]:
    n, _, kv = arg.partition(":")
    n = int(n)
    keys = {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}
    off = off_all[:n + 1]
    obs = obs_all[:int(off[-1])]
    o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
    p_d = torch.empty(len(obs), dtype=torch.int32, device=dev)
    s_d = torch.empty(n, dtype=torch.float64, device=dev)
    st_d = torch.empty(n, dtype=torch.uint8, device=dev)
    f, b = [], []
    with h.tuned(**keys):
        for r in range(REPS + 1):
            cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream,
                                   dtype="f64", workspace_bytes=80 << 30)
            stream.synchronize()
            t = cv.last_timing(h)
            if r:
                f.append(t["fwd_ms"])
                b.append(t["bt_ms"])
    fm, bm = float(np.median(f)), float(np.median(b))
    print(f"n={n:6d} {keys} fwd {fm:8.3f} ms bt {bm:6.3f} ms  {fm / n * 1e3:6.3f} us/seq fwd  kernel {t.get('kernel')}",
          flush=True)
