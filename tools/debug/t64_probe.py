"""Per-wave timing of the f64 forward (debug build with -DCV_T64_PROBE, tools/_ab/lib_probe.so
copied over the package library): decodes a config-4-shaped batch of B sequences and prints
the distribution of wave start / end times (s_memrealtime, 100 MHz), durations, and how the
waves were placed (HW_ID: SIMD, CU, SE; XCC_ID).  Usage: python tools/debug/t64_probe.py B"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import _lib, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N, V, T = 256, 1024, 512
pi, a, b = synth.random_hmm(N, V, seed=20261015)
obs = synth.iid_obs(V, B * T, 20261015, start=0)
off = np.arange(B + 1, dtype=np.int64) * T
dev = torch.device("cuda", 0)
h = cv.HMM(pi, a, b.reshape(N, 32, 32), device=0)
off_d = torch.from_numpy(off).to(dev)
obs_d = torch.from_numpy(obs).to(dev)
path = torch.empty(B * T, dtype=torch.int32, device=dev)
score = torch.empty(B, dtype=torch.float64, device=dev)
st = torch.empty(B, dtype=torch.uint8, device=dev)
for _ in range(3):
    cv.decode_batch_device(h, off_d, obs_d, path, score, st, offsets_host=off, dtype="f64",
                           workspace_bytes=80 << 30)
torch.cuda.synchronize()
tm = cv.last_timing(h)
spw = tm.get("seqs_per_wave", 8)
nwaves = B // spw if spw == 8 else 2 * (B // (2 * spw))
buf = (ctypes.c_uint64 * (6 * nwaves))()
lib = ctypes.CDLL(_lib.LIB_PATH)
rc = lib.cv_debug_t64_probe(buf, ctypes.c_int(nwaves))
assert rc == 0, rc
p = np.frombuffer(buf, dtype=np.uint64).reshape(nwaves, 6).astype(np.int64)
rt0, rt1, c0, c1, hw, xcc = p.T
t0 = rt0.min()
s, e = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0  # microseconds
d = e - s
print(f"B={B} waves={nwaves} fwd_ms={tm['fwd_ms']:.3f} seqs_per_wave={spw}")
q = [0, 1, 10, 50, 90, 99, 100]
print("start us  pct", dict(zip(q, np.percentile(s, q).round(1))))
print("end us    pct", dict(zip(q, np.percentile(e, q).round(1))))
print("dur us    pct", dict(zip(q, np.percentile(d, q).round(1))))
print("cycles/us (s_memtime)", np.median((c1 - c0) / np.maximum(d, 1e-9)).round(1))
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
xc = xcc & 15
key = ((xc * 8 + se) * 2 + sh) * 16 + cu
ck = key * 4 + simd
u, cnt = np.unique(ck, return_counts=True)
print("distinct SIMDs used", len(u), "waves per SIMD histogram", dict(zip(*np.unique(cnt, return_counts=True))))
uc, ccnt = np.unique(key, return_counts=True)
print("distinct CUs used", len(uc), "waves per CU histogram", dict(zip(*np.unique(ccnt, return_counts=True))))
# duration by waves sharing the SIMD
per = {k: c for k, c in zip(u, cnt)}
for n in sorted(set(cnt)):
    m = np.array([per[k] == n for k in ck])
    print(f"  SIMDs holding {n} waves: wave dur median {np.median(d[m]):.1f} us, max {d[m].max():.1f}")
# pair partners (W=2): same SIMD or not
if spw != 8:
    same = (ck[0::2] == ck[1::2]).mean()
    print("W2 partners on the same SIMD:", round(float(same), 3), " same CU:", round(float((key[0::2] == key[1::2]).mean()), 3))
