"""Training-peer CLI on CPU: multi-peer local-SGD / sharded runs, checkpoint and resume onto
a different peer count, fault injection."""
import json
import os
import subprocess
import sys

import pytest

from tests import _mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(n, args, port, timeout=180, extra_env=None, ids=None):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    env.update(extra_env or {})
    procs = []
    for r in (ids if ids is not None else range(n)):
        cmd = [sys.executable, "-m", "distributedvolunteercomputing_amd.cli.main", "train", "--peer-id", str(r),
               "--world", str(n), "--store-port", str(port), *args]
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out))
    return outs


def _records(out):
    recs = []
    for line in out.splitlines():
        if line.startswith("{"):
            try:
                recs.append(json.loads(line))
            except json.JSONDecodeError:
                pass
    return recs


def test_localsgd_cli_checkpoint_and_resume_on_more_peers(tmp_path):
    ck = str(tmp_path / "ck")
    outs = _launch(2, ["--model", "mlp", "--steps", "8", "--H", "2", "--batch", "32", "--lr", "0.05",
                       "--ckpt-dir", ck, "--ckpt-every", "4", "--log-every", "4"], _mp.free_port())
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    assert open(os.path.join(ck, "LATEST")).read().strip() == "step_00000008"
    man = json.load(open(os.path.join(ck, "step_00000008", "manifest.json")))
    assert man["format"] == "vcx-ckpt-v1" and len(man["shards"]) == 2 and man["step"] == 8
    # resume on 3 peers (different shard layout) and keep training
    outs = _launch(3, ["--model", "mlp", "--steps", "12", "--H", "2", "--batch", "32", "--lr", "0.05",
                       "--ckpt-dir", ck, "--resume", "--log-every", "2"], _mp.free_port())
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "resumed from" in out
        recs = _records(out)
        assert recs and recs[0]["step"] == 10 and recs[-1]["step"] == 12


def test_sharded_cli_with_fault_injection(tmp_path):
    outs = _launch(3, ["--model", "mlp", "--trainer", "sharded", "--steps", "10", "--batch", "32", "--lr", "0.01",
                       "--elastic", "--lease", "1.0", "--log-every", "2", "--drop-at", "-1"], _mp.free_port())
    for rc, out in outs:
        assert rc == 0, out[-3000:]


def test_localsgd_cli_peer_crash_survivors_continue(tmp_path):
    port = _mp.free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    procs = []
    for r in range(3):
        args = ["--model", "mlp", "--steps", "16", "--H", "2", "--batch", "32", "--elastic", "--lease", "1.0",
                "--log-every", "2"]
        if r == 2:
            args += ["--drop-at", "5"]
        procs.append(subprocess.Popen([sys.executable, "-m", "distributedvolunteercomputing_amd.cli.main", "train",
                                       "--peer-id", str(r), "--world", "3", "--store-port", str(port), *args],
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=180) for p in procs]
    for (out, _), p in zip(outs, procs):
        assert p.returncode == 0, out[-3000:]
    assert "fault injection" in outs[2][0]
    for r in (0, 1):
        recs = _records(outs[r][0])
        assert recs[-1]["step"] == 16 and recs[-1]["members"] == 2 and recs[-1]["gen"] == 1


def test_coordinator_hosted_store_survives_peer0_crash():
    """With the coordinator hosting the rendezvous store, even peer 0 may crash."""
    from distributedvolunteercomputing_amd.control.coordinator import coordinator

    c = coordinator("127.0.0.1", 0, ephemeral_ports=True, train_store_port=0)
    try:
        env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
        procs = []
        for r in range(3):
            args = ["--model", "mlp", "--steps", "16", "--H", "2", "--batch", "32", "--elastic", "--lease", "1.0",
                    "--log-every", "2", "--coordinator", f"127.0.0.1:{c.control_port}"]
            if r == 0:
                args += ["--drop-at", "5"]
            procs.append(subprocess.Popen([sys.executable, "-m", "distributedvolunteercomputing_amd.cli.main",
                                           "train", "--peer-id", str(r), "--world", "3", *args], cwd=ROOT, env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        outs = [p.communicate(timeout=180)[0] for p in procs]
        for out, p in zip(outs, procs):
            assert p.returncode == 0, out[-3000:]
        for r in (1, 2):
            recs = _records(outs[r])
            assert recs[-1]["step"] == 16 and recs[-1]["members"] == 2, recs[-1]
    finally:
        c.exit_threads()
