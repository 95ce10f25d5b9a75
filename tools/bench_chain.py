import sys, time, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import numpy as np, cviterbi as cv
from cviterbi import synth
for n, L in [(12, 200000), (64, 50000), (126, 20000), (256, 5000)]:
    pi, a, b = synth.random_hmm(n, 50, seed=1)
    lengths = np.full(L // 25, 25)
    off = synth.offsets_from_lengths(lengths)
    obs = np.random.default_rng(0).integers(0, 50, size=int(off[-1])).astype(np.int32)
    h = cv.HMM(pi, a, b)
    cv.decode_superseq_cp(h, off[:3], obs[:off[2]])
    t0 = time.perf_counter(); cv.decode_superseq_cp(h, off, obs); el = time.perf_counter() - t0
    print(f"N={n} elements={off[-1]} {el*1e3:.1f} ms  {el/off[-1]*1e6:.2f} us/element", flush=True)
