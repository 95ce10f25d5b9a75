"""Config-4 decode throughput with consecutive batches in flight: P handles (each its own delta
workspace) on P streams, step k on handle k % P, so one batch's backtrack (HBM-bound) can run
beside the next batch's forward (f64 VALU-bound).  Prints ms per step for P = 1 and P = 2 on
the same inputs, and checks every step's result against the P = 1 decode bit for bit.

  python tools/bench_pipeline.py [steps=8]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

N, V, T, B, SEED = 256, 1024, 512, 65536, 20261015


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    pi, a, b = synth.random_hmm(N, V, seed=SEED)
    obs = synth.iid_obs(V, B * T, SEED, start=0)
    off = np.arange(B + 1, dtype=np.int64) * T
    off_d, obs_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
    res = {}
    for P in (1, 2, 1, 2):
        hs = [cv.HMM(pi, a, b.reshape(N, 32, 32)) for _ in range(P)]
        ss = [torch.cuda.Stream(dev) for _ in range(P)]
        outs = [(torch.empty(B * T, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.float64, device=dev),
                 torch.empty(B, dtype=torch.uint8, device=dev)) for _ in range(P)]

        def step(k):
            i = k % P
            cv.decode_batch_device(hs[i], off_d, obs_d, *outs[i], offsets_host=off, stream=ss[i].cuda_stream,
                                   dtype="f64", workspace_bytes=80 << 30)

        for k in range(P):  # warmup
            step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            step(k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        got = [tuple(x.cpu().numpy() for x in o) for o in outs]
        if "ref" not in res:
            res["ref"] = got[0]
        same = all(all(np.array_equal(x, y) for x, y in zip(g, res["ref"])) for g in got)
        print(f"P={P}: {ms:.2f} ms per step ({steps} steps), results equal the P=1 decode: {same}", flush=True)
        del hs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
