"""Per-wave timeline of trellis_wave48_f64 at config 2 (probe build: CVK_W48_PROBE, loaded with
CV_LIB_PATH=tools/_ab/lib_probe.so).  Each sequence's wave records s_memrealtime (100 MHz) and
s_memtime at start and end, HW_ID and XCC_ID; this groups them by SIMD and prints where the
makespan goes: the longest sequences' per-step time, alone and shared.
Build the probe library first (in this container; it travels to the GPU box with the tree):
  make -C consistent-viterbi_amd/csrc BUILD=build_probe OUT=../../tools/_ab/lib_probe.so \
       T64FLAGS="-fno-honor-nans -DCVK_W48_PROBE"
(the `build_probe` objects are git- and gpurun-ignored; `tools/_ab/` is git-ignored)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
import torch  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import _lib, synth  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
c = synth.config("c2")
off, obs = c["offsets"], c["obs"]
B = len(off) - 1
h = cv.HMM(c["pi"], c["a"], c["b"])
o_d, ob_d = torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev)
p_d = torch.empty(len(obs), dtype=torch.int32, device=dev)
s_d = torch.empty(B, dtype=torch.float64, device=dev)
st_d = torch.empty(B, dtype=torch.uint8, device=dev)
for _ in range(int(os.environ.get("REPS", "10"))):
    cv.decode_batch_device(h, o_d, ob_d, p_d, s_d, st_d, offsets_host=off, stream=stream.cuda_stream, dtype="f64",
                           workspace_bytes=80 << 30)
torch.cuda.synchronize()
print("last_timing", cv.last_timing(h))
lib = ctypes.CDLL(_lib.LIB_PATH)
buf = np.zeros((8192, 8), dtype=np.uint64)
rc = lib.cvk_w48_probe_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
assert rc == 0, rc
p = buf[:B].astype(np.int64)
r0, r1, re, rd0, hw, xcc, T, rb1 = (p[:, i] for i in range(8))
assert (T == np.diff(off)).all(), "probe lengths do not match"
base = r0.min()
print(f"makespan (realtime, 10 ns): first start -> last end {(r1.max() - base) * 10 / 1e3:.2f} us;"
      f" start spread {(r0.max() - base) * 10 / 1e3:.2f} us")
us = lambda x: np.median(x) * 10 / 1e3  # noqa: E731
print(f"startup (median over waves): entry at {us(re - base):.2f} us; offsets read +{us(r0 - re):.2f} us;"
      f" delta_0 +{us(rd0 - r0):.2f} us; first {os.environ.get('PD', '4')}-step block"
      f" +{us((rb1 - rd0)[rb1 > 0]):.2f} us (waves with T >= 5)")
L = T >= 100
print(f"T >= 100: entry {us(re[L] - base):.2f}, offsets +{us(r0[L] - re[L]):.2f}, delta_0 +{us(rd0[L] - r0[L]):.2f},"
      f" block 1 +{us(rb1[L] - rd0[L]):.2f} us; rest {us(r1[L] - rb1[L]):.2f} us over T-5 steps ="
      f" {np.median((r1[L] - rb1[L]) * 10 / np.maximum(T[L] - 5, 1)):.1f} ns/step")
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = ((xcc & 15) << 16) | (se << 8) | (sh << 6) | (cu << 2) | simd
dur = (r1 - r0) * 10 / 1e3  # us
per_step = dur / np.maximum(T, 1) * 1e3  # ns per step
print("per-step ns by length decile (duration / T):")
order = np.argsort(T)
for q in range(10):
    idx = order[q * B // 10:(q + 1) * B // 10]
    print(f"  T {T[idx].min():4d}-{T[idx].max():4d}: {np.median(per_step[idx]):7.1f} ns/step,"
          f" duration {np.median(dur[idx]):6.2f} us, start {np.median((r0[idx] - base) * 10 / 1e3):6.2f} us")
uk, inv = np.unique(key, return_inverse=True)
print(f"distinct SIMDs {len(uk)}; waves per SIMD: {np.bincount(np.bincount(inv))}")
spans, sums, longest, ends = [], [], [], []
for i in range(len(uk)):
    m = inv == i
    spans.append((r1[m].max() - r0[m].min()) * 10 / 1e3)
    sums.append(T[m].sum())
    longest.append(T[m].max())
    ends.append((r1[m].max() - base) * 10 / 1e3)
spans, sums, longest, ends = map(np.asarray, (spans, sums, longest, ends))
print(f"SIMD end time us: p50 {np.median(ends):.2f} p90 {np.percentile(ends, 90):.2f} max {ends.max():.2f}")
print(f"SIMD total steps: min {sums.min()} p50 {np.median(sums)} max {sums.max()}; longest-per-SIMD max {longest.max()}")
w = np.argsort(ends)[-5:]
for i in w:
    m = np.where(inv == i)[0]
    print(f"  late SIMD key {uk[i]:#x}: end {ends[i]:.2f} us, steps {sums[i]}, waves",
          [(int(T[j]), round(float((r0[j] - base) * 10 / 1e3), 2), round(float((r1[j] - base) * 10 / 1e3), 2)) for j in m])
# alone vs shared: the longest wave of each SIMD, time after its last mate ended
alone = []
for i in range(len(uk)):
    m = np.where(inv == i)[0]
    j = m[np.argmax(T[m])]
    mates = [k for k in m if k != j]
    if not mates:
        continue
    last_mate = max(r1[k] for k in mates)
    if r1[j] > last_mate:
        alone.append(((r1[j] - last_mate) * 10, T[j]))
print(f"longest waves running alone at their end: {len(alone)} SIMDs, median alone time"
      f" {np.median([a for a, _ in alone]) / 1e3 if alone else 0:.2f} us")
# SIMD end time by its composition (sorted lengths of its four waves)
comp = []
for i in range(len(uk)):
    m = np.where(inv == i)[0]
    comp.append((tuple(sorted((int(T[j]) for j in m), reverse=True)), ends[i]))
comp.sort(key=lambda c: c[1])
print("SIMD compositions, earliest and latest ends:")
for c, e in comp[:6] + comp[-6:]:
    print(f"  {c}: end {e:.2f} us")
lmax = np.array([c[0][0] for c in comp]); l2 = np.array([c[0][1] for c in comp]); en = np.array([c[1] for c in comp])
for lo, hi in ((0, 100), (100, 116), (116, 129)):
    for a, b in ((0, 48), (48, 80), (80, 129)):
        sel = (lmax >= lo) & (lmax < hi) & (l2 >= a) & (l2 < b)
        if sel.any():
            print(f"  longest [{lo},{hi}) second [{a},{b}): {sel.sum():4d} SIMDs, end p50 {np.median(en[sel]):.2f} max {en[sel].max():.2f} us")
