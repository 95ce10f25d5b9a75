"""Time the generic decode at large N: one workgroup per sequence (rows in LDS, generic_fwd /
generic_fwd_ms) against the wide kernel (generic_wide_step: each step over ceil(N / 256)
workgroups, rows in global memory; CV_GENERIC_WIDE_MIN), and the serial super-sequence chain
both ways (CV_CHAIN_WIDE_MIN).  Results bit-identical between modes (checked here too).

  python tools/bench_wide.py [--n 4096,10240,16384] [--nseq 4,64,1024] [--T 8]
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "consistent-viterbi_amd"))
import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402


def _beat():
    while True:
        time.sleep(30)
        print("  ... running", flush=True)


def _time(fn, reps=2):
    fn()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="4096,10240,16384")
    ap.add_argument("--nseq", default="4,64,1024")
    ap.add_argument("--T", type=int, default=8)
    ap.add_argument("--chain-len", type=int, default=64)
    ap.add_argument("--wide-s", default="auto", help="tuning key wide_s values for the wide runs, e.g. auto,1,2,4")
    ap.add_argument("--assocs", default="viterbi,cp")
    args = ap.parse_args()
    threading.Thread(target=_beat, daemon=True).start()
    for n in [int(x) for x in args.n.split(",")]:
        pi, a, b = synth.random_hmm(n, 16, seed=n)
        h = cv.HMM(pi, a, b)
        for nseq in [int(x) for x in args.nseq.split(",")]:
            off = synth.offsets_from_lengths(np.full(nseq, args.T))
            obs = synth.iid_obs(16, int(off[-1]), n + nseq)
            res = {}
            modes = (["lds"] if n <= 10240 else []) + ["wide" + x for x in args.wide_s.split(",")]
            for mode in modes:
                h.set_tuning(wide_s=0 if mode in ("lds", "wideauto") else int(mode[4:]),
                             generic_wide_min=1 if mode.startswith("wide") else 0)
                for assoc in args.assocs.split(","):
                    ms, out = _time(lambda: cv.decode_batch(h, off, obs, dtype="f64", assoc=assoc, kernel="generic",
                                                            rescore_f64=False))
                    t = cv.last_timing(h)
                    res[(mode, assoc)] = out
                    steps = nseq * (args.T - 1)
                    gbs = steps * n * n * 8 / (t["fwd_ms"] * 1e-3) / 1e9
                    print(f"N={n} nseq={nseq} T={args.T} {mode:8s} {assoc:7s} wall {ms:9.2f} ms  fwd {t['fwd_ms']:9.2f} ms "
                          f"bt {t['bt_ms']:6.2f} ms  table stream {gbs:7.1f} GB/s", flush=True)
            h.set_tuning(wide_s=0, generic_wide_min=0)
            for (mode, assoc), out in res.items():
                for x, y in zip(res[(modes[0], assoc)], out):
                    assert np.array_equal(x, y), (n, nseq, mode, assoc)
        # the serial chain
        off = synth.offsets_from_lengths(np.full(max(args.chain_len // 8, 1), 8))
        obs = synth.iid_obs(16, int(off[-1]), n)
        h.set_tuning(chain_par=0)
        outs = {}
        for mode in (("lds", "wide") if n <= 10240 else ("wide",)):
            h.set_tuning(chain_wide_min=1 if mode == "wide" else 0)
            ms, outs[mode] = _time(lambda: cv.decode_superseq_cp(h, off, obs), reps=1)
            print(f"N={n} chain L={int(off[-1])} {mode:4s} {ms:9.2f} ms  ({ms / int(off[-1]):.3f} ms per element)", flush=True)
        h.set_tuning(chain_wide_min=0, chain_par=1)
        if len(outs) == 2:
            assert outs["lds"][1] == outs["wide"][1] and np.array_equal(outs["lds"][0], outs["wide"][0])
        del h


if __name__ == "__main__":
    main()
