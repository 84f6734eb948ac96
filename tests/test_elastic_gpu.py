"""Elastic local-SGD on the GPU: bench_drop.py with 3 peer processes sharing one MI355X (gloo
carries the averaging rounds between GPU buffers, since RCCL does not run two ranks on one
device). One peer crashes mid-window; the survivors detect it by lease expiry, regroup and keep
training through the HIP kernels + hipGraph step."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_drop_three_gpu_peers_one_crash(gpu, tmp_path):
    out = tmp_path / "drop.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench_drop.py"), "--peers", "3", "--model", "gpt2-tiny", "--batch", "4",
           "--seq", "64", "--steps", "14", "--warmup", "4", "--lease", "0.5", "--json-out", str(out), "--timeout", "150"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(out.read_text())
    assert rec["n_gpus"] >= 1 and rec["dtype"] == "bf16"
    assert rec["regroup_step"] is not None and rec["regroup_step"] >= rec["config"]["drop_at"]
    assert rec["ms_per_step_after"] > 0 and rec["samples_per_s_after"] > 0


def test_bench_drop_gpu_peers_killed_then_rejoin(gpu, tmp_path):
    """Config 4 on one GPU: 2 of 4 GPU peers SIGKILLed inside the averaging all-to-all, replacement
    processes join the running job (the admission streams the anchor GPU->host->GPU over gloo
    point-to-point) and the full group trains on."""
    out = tmp_path / "drop.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench_drop.py"), "--peers", "4", "--model", "gpt2-tiny", "--batch", "4",
           "--seq", "64", "--steps", "10", "--warmup", "4", "--lease", "0.5", "--json-out", str(out), "--timeout", "150",
           "--fault", "collective", "--drop-peers", "2,3", "--rejoin", "--after-rejoin", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(out.read_text())
    assert rec["rounds_aborted_and_redone"] >= 1
    assert rec["rejoin_step"] is not None and len(rec["joiner_admission_ms"]) == 2
    assert rec["samples_per_s_after_rejoin"] > 0
