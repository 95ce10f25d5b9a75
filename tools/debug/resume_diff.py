import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cviterbi as cv
from test_gpu_constrained import _resume_case
pi, a, b, off, obs, comp = _resume_case(256, 4, bad_obs=True)
h = cv.HMM(pi, a, b)
os.environ["CV_NO_RESUME"] = "1"
ref = cv.decode_constrained(h, off, obs, comp, ncomp=5)
os.environ["CV_NO_RESUME"] = "0"
got = cv.decode_constrained(h, off, obs, comp, ncomp=5)
print("states", ref[3], got[3])
d = np.nonzero(ref[0] != got[0])[0]
seqs = np.unique(np.searchsorted(off, d, side="right") - 1)
for s in seqs:
    e0, e1 = off[s], off[s + 1]
    cp = np.nonzero(comp[e0:e1] >= 0)[0]
    print("seq", s, "len", e1 - e0, "constrained at", cp, "comps", comp[e0:e1][cp], "bad at", np.nonzero(obs[e0:e1] == 8)[0],
          "status ref/got", ref[2][s], got[2][s], "score", ref[1][s], got[1][s])
    print("  ref", ref[0][e0:e1].tolist())
    print("  got", got[0][e0:e1].tolist())
