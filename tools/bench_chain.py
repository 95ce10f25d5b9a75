"""CPSolver chained super-sequence decode (cv_decode_superseq_cp = solver kind gpu-cp, what
main.rs:120 runs): wall time of the PARALLEL chain (per-sequence f64 trellis + certificates +
host fold + serial re-runs of the uncertified sequences) on config-4-shaped inputs, with the
serial chain kernel (tuning key chain_par = 0) on a smaller slice for comparison; every parallel result
is checked against the serial chain where both run.

  python tools/bench_chain.py [nseq_full=65536] [nseq_cmp=2048]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import numpy as np  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402


def run(h, off, obs, serial=False):
    with h.tuned(chain_par=0 if serial else 1):  # tuning key: the serial chain kernel
        t0 = time.perf_counter()
        path, obj = cv.decode_superseq_cp(h, off, obs)
        el = time.perf_counter() - t0
    return path, obj, el, cv.last_superseq_stats(h)


def main():
    nfull = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    ncmp = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    c = synth.config("c4", nfull)
    h = cv.HMM(c["pi"], c["a"], c["b"])
    off, obs = c["offsets"], c["obs"]
    run(h, off[:3], obs[:off[2]])  # tables, first-call setup
    # comparison slice: parallel vs serial, bit for bit
    oc, bc = off[:ncmp + 1], obs[:off[ncmp]]
    p1, o1, t1, s1 = run(h, oc, bc)
    p0, o0, t0, _ = run(h, oc, bc, serial=True)
    same = bool(np.array_equal(p1, p0) and o1 == o0)
    L = int(oc[-1])
    print(f"N=256 {ncmp} seqs x 512 = {L} elements: parallel {t1*1e3:.1f} ms ({t1/L*1e9:.1f} ns/element), "
          f"serial chain {t0*1e3:.1f} ms ({t0/L*1e6:.3f} us/element), equal={same}, stats {s1}", flush=True)
    if not same:
        raise SystemExit("parallel chain differs from the serial chain")
    for rep in range(2):
        p, o, t, s = run(h, off, obs)
        L = int(off[-1])
        print(f"N=256 {nfull} seqs x 512 = {L} elements (config-4-sized gpu-cp solve): {t*1e3:.1f} ms "
              f"({t/L*1e9:.1f} ns/element), objective {o!r}, stats {s}", flush=True)
    # the full chain's prefix slice must agree with the comparison run's serial chain
    assert np.array_equal(p[:int(oc[-1])][:-512], p0[:-512]), "prefix of the full chain differs"
    if os.environ.get("FULL_SERIAL") == "1":  # the whole input through the serial chain (~2 min)
        ps, os_, ts, _ = run(h, off, obs, serial=True)
        same = bool(np.array_equal(ps, p) and os_ == o)
        print(f"serial chain over all {int(off[-1])} elements: {ts:.1f} s, objective {os_!r}, "
              f"parallel == serial: {same}", flush=True)
        if not same:
            raise SystemExit("parallel chain differs from the serial chain at full size")


if __name__ == "__main__":
    main()
