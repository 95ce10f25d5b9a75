"""CPU, world_size 2 (gloo): a rank that never enters a collective must not hang the job.

bench.py (N > 1) initialises its process group through cviterbi.dist.init_process_group (a
finite collective timeout; async error handling for RCCL) and wraps every collective in a
CollectiveWatch phase.  Here rank 1 never enters the packed gather of the step results (it
sleeps far past the timeout); rank 0 must exit non-zero within the timeout with a message that
names the collective and its rank -- the driver's SCALE run would otherwise sit at its 600 s
limit with no output.  Contract: main.rs:129-133 (one output line per element): a gather that
never completes must fail loudly.
"""
import os
import subprocess
import sys
import time

from conftest import ROOT

from test_dist import _free_port

RANK_SCRIPT = r"""
import os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "consistent-viterbi_amd"))
import torch
import torch.distributed as dist
from cviterbi import dist as cvd

rank, mode, timeout = int(sys.argv[2]), sys.argv[3], float(sys.argv[4])
cvd.init_process_group(dist, "gloo", timeout_s=timeout if mode == "backend" else 120.0)
watch = cvd.CollectiveWatch(rank, timeout_s=timeout, who="test", poll_s=0.2)
with watch.phase("preflight: gather_packed_to_root + int64 all_reduce"):
    ok, msg = cvd.preflight(dist)
assert ok, msg
if rank == 1:
    time.sleep(60)  # never enters the gather below
    os._exit(0)
path = torch.zeros(5, dtype=torch.int32)
score = torch.zeros(2, dtype=torch.float64)
status = torch.zeros(2, dtype=torch.uint8)
try:
    with watch.phase("timed steps: per-step gather_packed_to_root to rank 0"):
        cvd.gather_packed_to_root(path, score, status, 256, 5, 2, dist)
except RuntimeError as e:
    print(e, file=sys.stderr, flush=True)
    os._exit(5)
print("gather returned", flush=True)
"""


def _run(mode, timeout):
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = []
    t0 = time.monotonic()
    for r in (0, 1):
        procs.append(subprocess.Popen([sys.executable, "-c", RANK_SCRIPT, ROOT, str(r), mode, str(timeout)],
                                      env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    try:
        out, err = procs[0].communicate(timeout=90)
        el = time.monotonic() - t0
        return procs[0].returncode, out, err, el
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.communicate()


def test_watch_names_stuck_collective():
    """The watch fires first (backend timeout 120 s): exit code 4, the phase named."""
    rc, out, err, el = _run("watch", 4.0)
    assert rc == 4, (rc, out, err)
    assert "test rank 0: collective 'timed steps: per-step gather_packed_to_root to rank 0' did not complete " \
           "within 4 s" in err, err
    assert el < 45, el  # import + rendezvous + 4 s, far from a 10-minute default


def test_backend_timeout_names_collective():
    """gloo's own timeout fires first (watch 4 s, process group 4 s; gloo raises): the phase
    re-raises with the collective named, the rank exits non-zero."""
    rc, out, err, el = _run("backend", 4.0)
    assert rc in (4, 5), (rc, out, err)
    assert "collective 'timed steps: per-step gather_packed_to_root to rank 0'" in err, err
    assert el < 45, el
