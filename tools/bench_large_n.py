"""Decode throughput of the generic kernels beyond N = 256 (trellis cells/s = N*T*batch / time),
f64 row-A0, synthetic model and observations.  Usage: python tools/bench_large_n.py [N ...]"""
import sys
import time

import numpy as np

sys.path.insert(0, "consistent-viterbi_amd")
import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402


def run(n, nseq, T, reps=3):
    pi, a, b = synth.random_hmm(n, 64, seed=n)
    off = synth.offsets_from_lengths(np.full(nseq, T))
    obs = synth.iid_obs(64, nseq * T, n)
    h = cv.HMM(pi, a, b)
    cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    t0 = time.perf_counter()
    for _ in range(reps):
        cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    dt = (time.perf_counter() - t0) / reps
    tm = cv.last_timing(h)
    print(f"N={n} nseq={nseq} T={T}: {dt * 1e3:.1f} ms/decode, {n * T * nseq / dt:.3e} cells/s, "
          f"{n * n * T * nseq / dt:.3e} pairs/s, kernel {tm.get('kernel')} fwd {tm.get('fwd_ms', 0):.1f} ms "
          f"bt {tm.get('bt_ms', 0):.1f} ms", flush=True)


if __name__ == "__main__":
    import os
    nseq = int(os.environ.get("NSEQ", "4096"))
    for n in [int(x) for x in sys.argv[1:]] or [256, 300, 512, 1024]:
        run(n, nseq, 128)
