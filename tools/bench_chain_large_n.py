"""The parallel CPSolver chain above N = 256 (cv_decode_superseq_cp = solver kind gpu-cp, what
main.rs:120 runs; cp.rs:63-93 over utils.rs:24-38): wall time of the parallel chain vs the
serial chain kernel (cp_superseq_chain, tuning key chain_par = 0) on config-4-shaped inputs at N states
(Dirichlet(1) log10 model, V = 1,024, T = 512), bit for bit (every element and the objective).

  python tools/bench_chain_large_n.py N [nseq=4096] [nseq_par_only=0]

nseq_par_only > 0 adds a parallel-only run over that many sequences (config-4 size: 65,536);
SERIAL=0 skips the serial comparison (and that run).
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import numpy as np  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402


def run(h, off, obs, serial=False):
    h.set_tuning(chain_par=0 if serial else 1)  # tuning key: the serial chain kernel
    stop = threading.Event()

    def beat():  # the serial chain runs minutes in one library call (ctypes releases the GIL)
        t0 = time.perf_counter()
        while not stop.wait(30.0):
            print(f"    ... {time.perf_counter() - t0:.0f} s", flush=True)

    hb = threading.Thread(target=beat, daemon=True)
    hb.start()
    try:
        t0 = time.perf_counter()
        path, obj = cv.decode_superseq_cp(h, off, obs)
        el = time.perf_counter() - t0
    finally:
        stop.set()
        hb.join()
        h.set_tuning(chain_par=1)
    return path, obj, el, cv.last_superseq_stats(h)


def main():
    n = int(sys.argv[1])
    nseq = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    nbig = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    T, V = 512, 1024
    pi, a, b = synth.random_hmm(n, V, seed=20261015 + n)
    tot = max(nseq, nbig)
    off_all = synth.offsets_from_lengths(np.full(tot, T))
    obs_all = synth.iid_obs(V, tot * T, 20261015)
    h = cv.HMM(pi, a, b)
    run(h, off_all[:3], obs_all[:off_all[2]])  # tables, first-call setup
    off, obs = off_all[:nseq + 1], obs_all[:off_all[nseq]]
    L = int(off[-1])
    p1, o1, t1, s1 = run(h, off, obs)
    print(f"N={n} {nseq} seqs x {T} = {L} elements: parallel {t1*1e3:.1f} ms ({t1/L*1e9:.1f} ns/element), "
          f"objective {o1!r}, stats {s1}", flush=True)
    p2, o2, t2, _ = run(h, off, obs)
    print(f"  again: {t2*1e3:.1f} ms, same result {bool(np.array_equal(p1, p2) and o1 == o2)}", flush=True)
    if os.environ.get("SERIAL", "1") == "0":
        print("  (serial comparison skipped: SERIAL=0)", flush=True)
    else:
        print(f"  serial chain (cp_superseq_chain, one thread per state) over the same {L} elements ...", flush=True)
        p0, o0, t0, s0 = run(h, off, obs, serial=True)
        same = bool(np.array_equal(p1, p0) and o1 == o0)
        print(f"  serial chain {t0:.2f} s ({t0/L*1e6:.2f} us/element), objective {o0!r}, parallel == serial: {same}, "
              f"speedup {t0/t1:.1f}x", flush=True)
        if not same:
            bad = np.nonzero(p1 != p0)[0]
            raise SystemExit(f"parallel chain differs from the serial chain: {bad.size} elements, first {bad[:5]}")
    if nbig > 0:
        ob, bb = off_all[:nbig + 1], obs_all[:off_all[nbig]]
        Lb = int(ob[-1])
        for rep in range(2):
            p, o, t, s = run(h, ob, bb)
            print(f"N={n} {nbig} seqs x {T} = {Lb} elements (config-4-sized gpu-cp solve): {t*1e3:.1f} ms "
                  f"({t/Lb*1e9:.1f} ns/element), objective {o!r}, stats {s}", flush=True)
        ok = bool(np.array_equal(p[:L][:-T], p1[:-T]))
        print(f"  prefix of {nseq} sequences equals the checked run (all but its last sequence): {ok}", flush=True)
        if not ok:
            raise SystemExit("prefix differs")


if __name__ == "__main__":
    main()
