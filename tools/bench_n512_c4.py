import sys, time
import numpy as np
sys.path.insert(0, "consistent-viterbi_amd")
import cviterbi as cv
from cviterbi import synth
n, nseq, T = 512, 65536, 512
pi, a, b = synth.random_hmm(n, 1024, seed=4)
off = synth.offsets_from_lengths(np.full(nseq, T))
obs = synth.iid_obs(1024, nseq * T, 4)
h = cv.HMM(pi, a, b)
cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
t0 = time.perf_counter()
cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
dt = time.perf_counter() - t0
t = cv.last_timing(h)
print(f"N=512 config-4 shape (65,536 x 512, host arrays): {dt*1e3:.0f} ms, {n*T*nseq/dt:.3e} cells/s, {n*n*T*nseq/dt:.3e} pairs/s, kernel {t['kernel']} fwd {t['fwd_ms']:.1f} ms bt {t['bt_ms']:.1f} ms launches {t['launches']}", flush=True)
