"""Throughput of HMM fitting on one MI355X, with a CPU baseline.

Corpus: config-2 shape (N=45 states, V=50,000 observations, B=4,096 sequences,
T ~ U[1,128]), or with SHAPE=c4 config 4's (N=256, V=1,024, B=65,536, T=512; B from
BATCH=...); initial parameters = random row-normalised probabilities (the reference
draws them in HMM::new, hmm.rs:22-28).
  mle    cv_hmm_fit_mle, every element tagged (hmm.rs:30-62)
  train  cv_hmm_fit_train, 20% of elements tagged, tol = 0 (hmm.rs:69-190): ms per EM
         iteration and elements/s per iteration, from a 1- and an (ITERS+1)-iteration call
CPU baseline: the numpy restatement (oracle/fit_oracle.py train_step, 1 thread) on the
first k sequences, scaled per element.  Prints one JSON line per mode."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import cviterbi as cv  # noqa: E402

SHAPE = os.environ.get("SHAPE", "c2")
if SHAPE == "c4":
    N, V, B, TMAX, SEED = 256, 1024, int(os.environ.get("BATCH", "65536")), 512, 2
else:
    N, V, B, TMAX, SEED = 45, 50000, 4096, 128, 2
ITERS = int(os.environ.get("ITERS", "20" if SHAPE != "c4" else "5"))
rng = np.random.default_rng(SEED)
lengths = rng.integers(1, TMAX + 1, size=B) if SHAPE != "c4" else np.full(B, TMAX)
off = np.zeros(B + 1, np.int64)
np.cumsum(lengths, out=off[1:])
E = int(off[-1])
obs = rng.integers(0, V, size=E).astype(np.int32)
tags_full = rng.integers(0, N, size=E).astype(np.int32)
tags = np.where(rng.random(E) < 0.2, tags_full, -1).astype(np.int32)
a = rng.random((N, N))
a /= a.sum(axis=1, keepdims=True)
b = rng.random((N, V))
b /= b.sum(axis=1, keepdims=True)
pi = rng.random(N)
pi /= pi.sum()

cv.fit_mle(pi, a, b, off, obs, tags_full)  # warm-up (code objects, allocations)
t0 = time.perf_counter()
cv.fit_mle(pi, a, b, off, obs, tags_full)
dt = time.perf_counter() - t0
print(json.dumps({"mode": "mle", "states": N, "nobs": V, "sequences": B, "elements": E, "ms": dt * 1e3,
                  "elements_per_s": E / dt}), flush=True)

cv.fit_train(pi, a, b, off, obs, tags, max_iter=1, tol=0.0)
t0 = time.perf_counter()
cv.fit_train(pi, a, b, off, obs, tags, max_iter=1, tol=0.0)
t1 = time.perf_counter()
_, _, _, it = cv.fit_train(pi, a, b, off, obs, tags, max_iter=ITERS + 1, tol=0.0)
t2 = time.perf_counter()
# per iteration = difference of a 1-iteration and an (ITERS+1)-iteration call, so the one-off
# upload of the corpus and parameters and the final download / log-map are not counted
dt = ((t2 - t1) - (t1 - t0)) / ITERS
out = {"mode": "train", "states": N, "nobs": V, "sequences": B, "elements": E, "tagged_frac": 0.2,
       "iterations": it, "ms_per_iteration": dt * 1e3, "ms_one_iteration_call": (t1 - t0) * 1e3,
       "elements_per_s": E / dt}
# f64 arithmetic per element and iteration: forward N^2 and backward N^2 FMAs (VALU), the
# xi sum N^2 FMAs (MFMA at N > 128); roofs: 256 CU x 64 lanes x 2.4 GHz f64 FMA (VALU)
fma = 3.0 * N * N * E
out["gflop_per_iteration"] = 2 * fma / 1e9
out["tflops"] = 2 * fma / dt / 1e12
# CPU baseline: numpy restatement, one EM iteration on the first k sequences
import fit_oracle as FO  # noqa: E402

k = 64 if SHAPE != "c4" else 2
t0 = time.perf_counter()
FO.train_step(pi, a, b, off[: k + 1], obs, tags)
cdt = time.perf_counter() - t0
ce = int(off[k])
out["cpu_baseline"] = {"elements_per_s": ce / cdt, "cores": 1, "kind": "port",
                       "sample": f"one EM iteration on the first {k} sequences ({ce} elements), oracle/fit_oracle.py"}
out["gpu_over_cpu"] = out["elements_per_s"] / out["cpu_baseline"]["elements_per_s"]
print(json.dumps(out), flush=True)
