"""Per-wave timing of the constrained decode's suffix pass at config 5 (debug build with
-DCV_T64_PROBE copied over the package library): wave start / end times and how many waves
were resident over time -- the occupancy of the ragged-length EXT pass.  Usage:
python tools/debug/ext_probe.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import cviterbi as cv  # noqa: E402
from cviterbi import _lib, synth  # noqa: E402

c = synth.config("c5")
h = cv.HMM(c["pi"], c["a"], c["b"])
off, obs, comp = c["offsets"], c["obs"], c["component"]
ncomp = int(comp.max()) + 1
for _ in range(2):
    cv.constrained_partials(h, off, obs, comp, ncomp)
nc = int(sum(1 for k in range(len(off) - 1) if (comp[off[k]:off[k + 1]] >= 0).any()))
nwaves = (nc + 7) // 8
buf = (ctypes.c_uint64 * (6 * nwaves))()
rc = ctypes.CDLL(_lib.LIB_PATH).cv_debug_t64_probe(buf, ctypes.c_int(nwaves))
assert rc == 0, rc
p = np.frombuffer(buf, dtype=np.uint64).reshape(nwaves, 6).astype(np.int64)
rt0, rt1, c0, c1, hw, xcc = p.T
t0 = rt0.min()
s, e = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0  # microseconds
d = e - s
span = e.max()
print(f"constrained sequences {nc}, waves {nwaves}, span {span / 1e3:.2f} ms")
q = [0, 1, 10, 50, 90, 99, 100]
print("start us pct", dict(zip(q, np.percentile(s, q).round(1))))
print("end us   pct", dict(zip(q, np.percentile(e, q).round(1))))
print("dur us   pct", dict(zip(q, np.percentile(d, q).round(1))))
print(f"sum of wave durations / (span x 2048 slots) = {d.sum() / (span * 2048):.3f}")
grid = np.linspace(0, span, 41)
live = [int(((s <= x) & (e > x)).sum()) for x in grid]
print("live waves over time:", live)
# per wave: slot order index (longest first) vs duration
print("duration of waves by launch index (deciles):", [round(float(np.median(d[i * nwaves // 10:(i + 1) * nwaves // 10])), 1) for i in range(10)])
print("start of waves by launch index (deciles):", [round(float(np.median(s[i * nwaves // 10:(i + 1) * nwaves // 10])), 1) for i in range(10)])
