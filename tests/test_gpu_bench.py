"""GPU: bench.py's multi-rank path (strong-scaling shards, per-rank decode, barriers, the
max-over-ranks timing, the packed gather to rank 0, the JSON line) rehearsed with 2 ranks on
one GPU over gloo -- RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the
RCCL gather itself runs only on a multi-GPU node (the driver's scaling runs)."""
import json
import os
import signal
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_two_rank_rehearsal(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "2048", "--backend", "gloo",
           "--no-f32-extra", "--no-configs", "--cpu-seconds", "1", "--c5-batch", "2048"]
    # own session: on a timeout the launcher AND its ranks are killed (process group)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=ROOT,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=240)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        raise
    assert p.returncode == 0, out[-3000:] + err[-3000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]  # rank 0 prints ONE line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["dtype"] == "f64"
    assert d["config"]["global_batch"] == 2048 and "sharded over 2 ranks" in d["config"]["workload"]
    assert d["value"] > 0 and d["roofline"]["kernel"].startswith("trellis_fwd_f64")
    # self-verification: rank 0 re-decoded the global batch and the gathered last step equals it
    # bit for bit (main.rs:129-133's per-element output), and the CPU-baseline leg's oracle check
    assert d["multi_gpu_check"]["equal"] is True and d["multi_gpu_check"]["sequences"] == 2048
    assert d["cpu_baseline"]["check"]["bit_exact"] is True and d["cpu_baseline"]["check"]["sequences"] == 64
    assert d["verified"] is True
    # config 5 sharded over the 2 ranks (exchange + gather) == rank 0's single-process decode
    c5 = d["c5_sharded"]
    assert c5["check"]["equal"] is True and c5["ms_per_decode"] > 0 and "sharded over 2 ranks" in c5["workload"]
    r = d["roofline"]
    assert r["bound"] == "valu" and 0 < r["frac"] < 1 and r["frac_f64_bytes"] > r["frac"]
    assert r["roofs"]["valu"]["frac"] > 0
