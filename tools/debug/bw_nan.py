"""Debug: Baum-Welch at N = 256 (GEMM xi path) over many iterations -- first iteration with a
NaN and the distance to the oracle at a few early iterations."""
import sys
import numpy as np
sys.path[:0] = ["consistent-viterbi_amd", "oracle"]
import fit_oracle as FO  # noqa: E402
import cviterbi as cv  # noqa: E402
from cviterbi import cli  # noqa: E402

rng = np.random.default_rng(11)
lens, obs, tg = [], [], []
nxt = 0
for sid in range(64):
    T = int(rng.integers(6, 14))
    lens.append(T)
    for t in range(T):
        obs.append(int(rng.integers(0, 32)) * 32 + int(rng.integers(0, 32)))
    for t in range(T):
        if t < T - 1 and rng.random() < 0.6:
            tg.append(nxt % 256)
            nxt += 1
        else:
            tg.append(-1)
off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
obs = np.array(obs, np.int32)
tg = np.array(tg, np.int32)
pi0, a0, b0 = cli._random_start(256, (32, 32), np.random.default_rng(3))
for it in (1, 2, 3, 5, 8, 12, 20, 40, 80, 160, 320, 640, 1000):
    gp, ga, gb, r = cv.fit_train(pi0, a0, b0, off, obs, tg, max_iter=it, tol=0.0)
    line = f"iters {it}: nan pi {np.isnan(gp).sum()} a {np.isnan(ga).sum()} b {np.isnan(gb).sum()}"
    if it <= 5:
        rp, ra, rb, _ = FO.train(pi0, a0, b0, off, obs, tg, it, 0.0)
        fin = np.isfinite(ra) & np.isfinite(ga)
        line += f"; max |a - oracle| {np.abs(ga[fin] - ra[fin]).max():.3e}, inf mismatch {(np.isinf(ga) != np.isinf(ra)).sum()}"
    print(line, flush=True)
    if np.isnan(gp).any() or np.isnan(ga).any():
        break
