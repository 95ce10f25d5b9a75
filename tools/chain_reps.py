"""The config-4-sized gpu-cp chain solved REPS times in one process (the first call sizes the
handle's buffers); prints every time and the median of the rest -- for interleaved A/B runs:
  python tools/chain_reps.py [nseq=65536]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
c = synth.config("c4", n)
h = cv.HMM(c["pi"], c["a"], c["b"])
ts = []
keep = os.environ.get("KEEP", "1") == "1"  # 1: the previous result is freed outside the timed call
out = None
for r in range(int(os.environ.get("REPS", "6"))):
    if keep:
        out = None  # the caller's previous 134 MB path array, released before the clock starts
    t0 = time.perf_counter()
    out = cv.decode_superseq_cp(h, c["offsets"], c["obs"])
    if not keep:
        out = None
    ts.append(1e3 * (time.perf_counter() - t0))
print(f"chain ms: {' '.join(f'{t:.1f}' for t in ts)}  median(rest) {np.median(ts[1:]):.1f}  min {min(ts[1:]):.1f}",
      flush=True)
