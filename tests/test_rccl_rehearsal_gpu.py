"""RCCL with more than one rank, on a one-GPU box.

RCCL refuses two ranks on one device; giving every rank its own NCCL_HOSTID
(scripts/rccl_rehearsal_launch.py) lets them build real RCCL communicators over loopback
sockets. That runs the same c10d/RCCL code the multi-GPU job runs: the torchrun-style headline
bench with the hand-written direct all-to-all all-reduce, and the elastic trainer's
per-generation communicators with ncclCommAbort when a peer is SIGKILLed inside the collective.
Numbers from these runs are not xGMI numbers; only correctness is asserted.
"""
import ast
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port(kind=socket.SOCK_STREAM):
    s = socket.socket(socket.AF_INET, kind)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(text):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise AssertionError(f"no JSON line in output:\n{text[-3000:]}")


@pytest.mark.gpu
def test_bench_two_ranks_rccl(gpu, tmp_path):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "scripts", "rccl_rehearsal_launch.py"), "--nproc", "2",
           "--timeout", "150", "--log-dir", str(tmp_path), "--", sys.executable, "-u", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "4", "--batch", "2", "--seq", "128", "--algo", "direct"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=180)
    out = (tmp_path / "rank0.out").read_text()
    assert r.returncode == 0, r.stderr[-3000:] + (tmp_path / "rank1.err").read_text()[-3000:]
    rec = _last_json(out)
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 4
    assert "allreduce=direct" in rec["config"]["parallelism"]
    assert rec["final_loss"] == rec["final_loss"]  # not NaN


@pytest.mark.gpu
def test_elastic_rccl_peer_killed_inside_collective(gpu, tmp_path):
    out = tmp_path / "drop.json"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench_drop.py"), "--peers", "3", "--backend", "nccl",
           "--model", "gpt2-tiny", "--batch", "2", "--seq", "64", "--steps", "12", "--warmup", "4",
           "--fault", "collective", "--lease", "1.5", "--graph", "0", "--timeout", "150", "--json-out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = json.loads(out.read_text())
    assert rec["config"]["backend"] == "nccl"
    assert rec["rounds_aborted_and_redone"] >= 1  # the survivors aborted the RCCL round and redid it
    assert rec["regroup_step"] is not None
    assert rec["drop_stall_ms"] < 30_000  # abort + regroup, not a collective timeout


@pytest.mark.gpu
def test_video_node_job_rccl_pairs(gpu, tmp_path):
    """The one-node video job (control/node_job.py) with 3 volunteers, chunks moving between
    GPU volunteers over RCCL pair communicators (requester -> worker -> requester send/recv)."""
    out_dir = tmp_path / "out"
    out_dir.mkdir()
    cmd = [sys.executable, "-u", os.path.join(ROOT, "scripts", "rccl_rehearsal_launch.py"), "--nproc", "3",
           "--timeout", "170", "--log-dir", str(tmp_path), "--", sys.executable, "-u", "-m",
           "distributedvolunteercomputing_amd.cli.main", "video", "--source", "synthetic:240:640x360",
           "--out-dir", str(out_dir), "--out-ext", ".npy", "--chunk", "40", "--port", str(_free_port(socket.SOCK_DGRAM)),
           "--store-port", str(_free_port())]
    env = dict(os.environ, VCX_P2P_BACKEND="nccl")  # (the default is gloo when volunteers share a GPU)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=200, env=env)
    log = (tmp_path / "rank0.out").read_text()
    assert r.returncode == 0, log[-2000:] + (tmp_path / "rank0.err").read_text()[-3000:]
    res = ast.literal_eval(log.strip().splitlines()[-1])
    assert res["frames"] == 240 and res["chunks"] == 6, res
    req = res["requester"]
    assert req.get("p2p_pairs_nccl", 0) >= 2 and not req.get("p2p_pairs_gloo"), req
    import numpy as np

    assert np.load(res["out"], mmap_mode="r").shape[0] == 240
