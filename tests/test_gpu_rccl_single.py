"""GPU: the RCCL ("nccl" backend) branches of the multi-GPU path, exercised with ONE rank on this
GPU (RCCL refuses two ranks on one device, so the multi-rank runs are the driver's): the
collective pre-flight on device tensors, the packed gather of a real decode's device result, the
device-tensor all-reduce of the constrained partials, and the sharded config-5 decode -- each
against the single-process result, bit for bit.  Contract: main.rs:129-133 (one output per
element), dp.rs:153-165 (the component choice)."""
import os
import signal
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = textwrap.dedent(r"""
    import os, sys
    sys.path.insert(0, os.path.join(sys.argv[1], "consistent-viterbi_amd"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import cviterbi as cv
    from cviterbi import dist as cvd, synth

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # bench.py's init: 180 s collective timeout, RCCL async error handling, a named-phase watch
    cvd.init_process_group(dist, "nccl", dev, rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    watch = cvd.CollectiveWatch(0, who="rccl-single")
    with watch.phase("preflight: gather_packed_to_root + int64 all_reduce"):
        ok, msg = cvd.preflight(dist, dev, 256)
    assert ok, msg
    # a real decode on the device, gathered as bench.py does (its own stream)
    pi, a, b = synth.random_hmm(256, 64, seed=11)
    nseq, T = 300, 40
    off = np.arange(nseq + 1, dtype=np.int64) * T
    obs = synth.iid_obs(64, nseq * T, 11)
    h = cv.HMM(pi, a, b)
    path = torch.empty(nseq * T, dtype=torch.int32, device=dev)
    score = torch.empty(nseq, dtype=torch.float64, device=dev)
    status = torch.empty(nseq, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    cv.decode_batch_device(h, torch.from_numpy(off).to(dev), torch.from_numpy(obs).to(dev), path, score, status,
                           offsets_host=off, stream=stream.cuda_stream, dtype="f64")
    comm = torch.cuda.Stream(dev)
    done = torch.cuda.Event()
    done.record(stream)
    comm.wait_event(done)
    with torch.cuda.stream(comm):
        g = cvd.gather_packed_to_root(path, score, status, 256, nseq * T, nseq, dist)
    torch.cuda.synchronize(dev)
    rp, rs, rst = cv.decode_batch(h, off, obs, dtype="f64", rescore_f64=False)
    gp, gs, gst = g[0]
    assert np.array_equal(gp[: nseq * T].cpu().numpy(), rp)
    assert np.array_equal(gs[:nseq].cpu().numpy().view(np.int64), rs.view(np.int64))
    assert np.array_equal(gst[:nseq].cpu().numpy(), rst)
    # the config-5 exchange on device tensors, and the sharded constrained decode
    w = cvd.allreduce_partials(np.array([1, -(1 << 60), 3], np.int64), dist, dev)
    assert w.tolist() == [1, -(1 << 60), 3]
    c = synth.config("c5", 512)
    hc = cv.HMM(c["pi"], c["a"], c["b"])
    got = cvd.constrained_decode_sharded(hc, c["offsets"], c["obs"], c["component"], 7, dist, device=dev)
    ref = cv.decode_constrained(hc, c["offsets"], c["obs"], c["component"], 7, dtype="f64")
    for x, y in zip(got, ref):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    dist.destroy_process_group()
    print("RCCL-SINGLE-OK")
""")


def test_rccl_single_rank_paths(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29571", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.Popen([sys.executable, "-c", SCRIPT, ROOT], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         env=env, cwd=ROOT, start_new_session=True)
    try:
        out, err = p.communicate(timeout=240)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        raise
    assert p.returncode == 0 and "RCCL-SINGLE-OK" in out, out[-3000:] + err[-3000:]
