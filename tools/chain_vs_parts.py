"""One process: the f64 batch decode of the chain's part sizes alone (49,152 and 8,192 config-4
sequences, and all 65,536), then the config-4-sized chain twice -- run under rocprofv3
--kernel-trace to compare each part's forward / backtrack inside the chain with the same launch
alone (tools/kt_overlap.py)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consistent-viterbi_amd"))
sys.argv = [sys.argv[0]] + (sys.argv[1:] or ["65536", "49152", "8192"])
exec(open(os.path.join(ROOT, "tools", "bench_batch_sizes.py")).read())  # noqa: S102 (our own tool)
for rep in range(2):
    t0 = time.perf_counter()
    cv.decode_superseq_cp(h, off_all, obs_all)
    print(f"chain {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
