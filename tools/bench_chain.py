"""CPSolver chained super-sequence decode (cv_decode_superseq_cp, kind gpu-cp, what main.rs:120
runs): wall time per element at several N.  CV_CHAIN_OLD=1 selects the one-thread-per-state
kernel for comparison (N <= 256 otherwise runs kernels/chain.hip)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import numpy as np  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

sizes = [(12, 200000), (64, 200000), (126, 100000), (256, 100000)]
if os.environ.get("CV_CHAIN_OLD") == "1":
    sizes = [(12, 200000), (64, 50000), (126, 20000), (256, 5000)]
for n, L in sizes:
    pi, a, b = synth.random_hmm(n, 50, seed=1)
    lengths = np.full(L // 25, 25)
    off = synth.offsets_from_lengths(lengths)
    obs = np.random.default_rng(0).integers(0, 50, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    cv.decode_superseq_cp(h, off[:3], obs[:off[2]])
    t0 = time.perf_counter()
    cv.decode_superseq_cp(h, off, obs)
    el = time.perf_counter() - t0
    print(f"N={n} elements={off[-1]} {el*1e3:.1f} ms  {el/off[-1]*1e6:.3f} us/element", flush=True)
