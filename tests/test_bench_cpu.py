"""bench.py under the driver's contract, on CPU/gloo with a tiny model: the single-process run and
the torchrun launch with world_size 2 (the multi-GPU command line, RCCL replaced by gloo). Checks
the one JSON line rank 0 prints: whole-job value, N, steps/warmup echo, weak scaling."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "4", "--warmup", "2", "--model", "gpt2-tiny", "--batch", "2", "--seq", "32", "--H", "2"]


def _env():
    return dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")


def _json_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def _check(rec: dict, n: int):
    assert rec["n_gpus"] == n and rec["steps"] == 4 and rec["warmup"] == 2
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["higher_is_better"] is True
    assert rec["scaling"] == "weak" and rec["config"]["global_batch"] == 2 * n
    # value is the whole-job rate: N x per-peer batch x steps / max-over-ranks time
    assert abs(rec["value"] - n * 2 * 4 / (rec["ms_per_step"] * 4 / 1e3)) / rec["value"] < 1e-2


def test_bench_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *ARGS], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_json_line(r.stdout), 1)


@pytest.mark.slow
def test_bench_gpus_flag_spawns_ranks_without_torchrun():
    """The driver's literal `python bench.py --gpus 4` (no launcher): bench.py starts 4 ranks itself
    (a child torch.distributed.run, never an exec) and the JSON reports the group that formed."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", *ARGS], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    _check(rec, 4)
    assert rec["rccl_world"] == 4 and rec["backend"] == "gloo" and len(rec["devices"]) == 4
    assert rec["sync_rounds_timed"] == 2 and rec["sync_ms_timed_mean"] > 0  # H = 2, 4 timed steps


def test_bench_mismatched_launch_fails_loudly():
    """--gpus 4 under a 2-rank launch must not report a 2-rank number as a 4-GPU run."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "4", *ARGS]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE=2" in r.stderr


def _torchrun(n, extra=()):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(n), *ARGS, *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    _check(rec, n)
    assert f"dp{n}" in rec["config"]["parallelism"]
    return rec


@pytest.mark.slow
def test_bench_torchrun_two_ranks():
    rec = _torchrun(2)
    assert "allreduce=direct" in rec["config"]["parallelism"]  # the default averaging schedule


@pytest.mark.slow
@pytest.mark.parametrize("n,algo", [(4, "direct"), (4, "butterfly"), (4, "ring"), (4, "rs_ag"), (4, "rccl"),
                                    (8, "direct"), (8, "butterfly")])
def test_bench_torchrun_more_ranks(n, algo):
    """The driver's multi-GPU command line at 4 and 8 ranks, each averaging algorithm (gloo)."""
    rec = _torchrun(n, ["--algo", algo])
    assert f"allreduce={algo}" in rec["config"]["parallelism"]
    assert rec["sync_ms"] > 0


def test_rehearsal_launcher_propagates_a_failed_rank(tmp_path):
    """scripts/rccl_rehearsal_launch.py: every rank gets the torchrun env and its own NCCL_HOSTID;
    one rank failing ends the job with that rank's exit status (the others are killed)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "assert os.environ['WORLD_SIZE'] == '3' and os.environ['NCCL_HOSTID'] == f'vcx-rehearsal-{r}'\n"
            "sys.exit(7) if r == 1 else time.sleep(60)\n")
    cmd = [sys.executable, os.path.join(root, "scripts", "rccl_rehearsal_launch.py"), "--nproc", "3", "--timeout", "50",
           "--", sys.executable, "-c", prog]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=90)
    assert r.returncode == 7, r.stderr
