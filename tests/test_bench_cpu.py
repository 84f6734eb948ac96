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
def test_bench_gpus_flag_spawns_ranks_without_torchrun(tmp_path):
    """The driver's literal `python bench.py --gpus 4` (no launcher): bench.py starts 4 ranks itself
    (a child torch.distributed.run, never an exec) and the JSON reports the group that formed. The
    spawning parent loads neither torch nor the HIP runtime, and the JSON carries
    the averaging round's bytes, time and bandwidth."""
    libs = tmp_path / "parent_libs.txt"
    env = dict(_env(), VCX_BENCH_PARENT_LIBS=str(libs))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", *ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    _check(rec, 4)
    assert rec["rccl_world"] == 4 and rec["backend"] == "gloo" and len(rec["devices"]) == 4
    assert rec["sync_rounds_timed"] == 2 and rec["sync_ms_timed_mean"] > 0  # H = 2, 4 timed steps
    loaded = libs.read_text().split()
    assert loaded and not [x for x in loaded if "amdhip64" in x or "libtorch" in x or "hsa-runtime" in x], loaded
    assert rec["avg_bytes_per_rank"] > 0 and rec["avg_collective_ms_mean"] > 0
    assert rec["avg_algbw_GBps"] > 0 and abs(rec["avg_busbw_GBps"] / rec["avg_algbw_GBps"] - 1.5) < 5e-2
    assert rec["rccl_transports"] is None  # gloo: no RCCL connection lines


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


def test_rccl_transport_parse_and_gpu_count(tmp_path, monkeypatch):
    """The transport counts come from RCCL's connection lines; the parent's GPU count from the
    visible-devices lists (intersection = the shortest) without any HIP call."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("vcx_bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    log = tmp_path / "rank0.log"
    log.write_text("host:1:2 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n"
                   "host:1:2 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC\n"
                   "host:1:2 [0] NCCL INFO Channel 00/1 : 0[0] -> 2[2] via SHM/direct/direct\n"
                   "host:1:2 [0] NCCL INFO Using network Socket\n")
    assert b._rccl_transports(str(log)) == {"P2P/IPC": 2, "SHM/direct/direct": 1}
    assert not log.exists()  # parsed once, then removed
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1")
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert b._visible_gpus() == 2
