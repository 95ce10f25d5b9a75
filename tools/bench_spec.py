"""The parallel chain's speculative batch in isolation: a CP-association batch decode of a few
hundred config-4 sequences (N = 256, T = 512), as superseq_cp_par's speculate() launches it,
timed per kernel choice (forward / backtrack ms from the library's own events).

  python tools/bench_spec.py [nseq ...]      (default 573: config 4's batch)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "consistent-viterbi_amd"))
import numpy as np  # noqa: E402

import cviterbi as cv  # noqa: E402
from cviterbi import synth  # noqa: E402

VARIANTS = [
    ("generic s=auto", "generic", {}),
    ("generic s=1", "generic", {"generic_s": 1}),
    ("generic s=2", "generic", {"generic_s": 2}),
    ("generic s=4", "generic", {"generic_s": 4}),
    ("generic split k=2", "generic", {"generic_split": 1, "generic_split_k": 2}),
    ("generic split k=4", "generic", {"generic_split": 1, "generic_split_k": 4}),
    ("trellis_cp auto", "trellis_f64", {}),
    ("trellis_cp w=1", "trellis_f64", {"t64_cp_w": 1}),
]


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [573, 143]
    c = synth.config("c4", max(sizes))
    h = cv.HMM(c["pi"], c["a"], c["b"])
    off, obs = c["offsets"], c["obs"]
    for n in sizes:
        o, b = off[:n + 1], obs[:off[n]]
        ref = None
        for name, kern, keys in VARIANTS:
            with h.tuned(**keys):
                best = None
                for _ in range(3):
                    p, s, st = cv.decode_batch(h, o, b, dtype="f64", assoc="cp", kernel=kern, rescore_f64=False)
                    t = cv.last_timing(h)
                    best = t if best is None or t["fwd_ms"] < best["fwd_ms"] else best
            same = ref is None or (np.array_equal(p, ref[0]) and np.array_equal(s, ref[1]))
            if ref is None:
                ref = (p, s)
            print(f"n={n} {name:18s} fwd {best['fwd_ms']:8.3f} ms  bt {best['bt_ms']:7.3f} ms  "
                  f"launches {best.get('launches')}  equal={same}", flush=True)


if __name__ == "__main__":
    main()
