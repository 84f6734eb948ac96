"""Command-line entry points with the reference's REPLs.

  python server.py [server_ip] [--port 9999] ...          REPL: `quit`
  python worker.py [server_ip own_ip] [--port 9999] ...   REPL: `request live|<path>`, `end`, anything else quits
  python -m distributedvolunteercomputing_amd.cli.main train ...   local-SGD training peer
  python -m distributedvolunteercomputing_amd.cli.main video ...   one-node video job (torchrun, one volunteer per GPU)
  python -m distributedvolunteercomputing_amd.cli.main status [server_ip]   a coordinator's status JSON
(``vcx <command>`` once installed: pyproject.toml)

Positional arguments keep the reference's form (server.py:166-169, worker.py:341-344);
everything else is an optional flag with the reference default.
"""
from __future__ import annotations

import argparse
import sys

from .. import config


def server_main(argv=None):
    ap = argparse.ArgumentParser(prog="server.py", description="volunteer-computing coordinator")
    ap.add_argument("ip", nargs="?", default="localhost")
    ap.add_argument("--port", type=int, default=9999, help="UDP control port")
    ap.add_argument("--policy", default="round_robin", choices=["round_robin", "least_loaded"])
    ap.add_argument("--credits", type=int, default=2, help="max chunks in flight per volunteer")
    ap.add_argument("--lease", type=float, default=10.0, help="heartbeat lease (s)")
    ap.add_argument("--ephemeral-ports", action="store_true", help="data ports from the OS instead of 5555..5599")
    ap.add_argument("--train-store-port", type=int, default=None,
                    help="also host the rendezvous store for training peers on this TCP port")
    ap.add_argument("--train-token", default=None,
                    help="admission token training peers must present (tjoin) to get the rendezvous store")
    ap.add_argument("--data-plane", default="relay", choices=["relay", "p2p"],
                    help="relay: chunk bytes through this process (reference); p2p: metadata only, chunks "
                         "travel between the volunteers over pair groups (RCCL between GPU volunteers)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    from ..control.coordinator import coordinator

    c = coordinator(a.ip, a.port, ephemeral_ports=a.ephemeral_ports, policy=a.policy, credits=a.credits,
                    lease_s=a.lease, verbose=a.verbose, train_store_port=a.train_store_port,
                    data_plane=a.data_plane, train_token=a.train_token)
    print(f"\nlistening on {a.ip} port {c.control_port}", flush=True)
    while True:
        try:
            line = input("\nEnter quit to exit\n")
        except EOFError:
            line = "quit"
        if line.strip() == "quit":
            c.exit_threads()
            print("done.")
            return 0
        if line.strip() == "status":
            print(c.status())


def worker_main(argv=None):
    ap = argparse.ArgumentParser(prog="worker.py", description="volunteer client (worker / requester)")
    ap.add_argument("server_ip", nargs="?", default="localhost")
    ap.add_argument("own_ip", nargs="?", default="localhost")
    ap.add_argument("--port", type=int, default=9999, help="coordinator UDP control port")
    ap.add_argument("--data-port", type=int, default=5554, help="own data port (0 = ephemeral)")
    ap.add_argument("--prototxt", default=None, help="Caffe prototxt (default: built-in MobileNet-SSD)")
    ap.add_argument("--caffemodel", default="MobileNetSSD_deploy.caffemodel",
                    help="weights (random init when absent, as in this environment)")
    ap.add_argument("--device", default=None,
                    help="cuda:N or cpu (default: LOCAL_RANK's GPU under a launcher, else the first GPU no other "
                         "volunteer on this host holds, so hand-launched volunteers spread over a node's GPUs)")
    ap.add_argument("--confidence", type=float, default=0.2)
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--out-ext", default=".y4m", choices=[".y4m", ".npy", ""])
    ap.add_argument("--p2p-backend", default=None, choices=[None, "nccl", "gloo"],
                    help="pair-group backend on a p2p coordinator (default: RCCL with several GPUs)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    from ..control.peer import client
    from ..jobs.video import DetectorEngine

    from ..utils.devices import claim_device

    dev = a.device or claim_device()
    eng = DetectorEngine(device=dev, prototxt=a.prototxt, caffemodel=a.caffemodel, conf_thresh=a.confidence)
    w = client(a.server_ip, a.own_ip, control_port=a.port, my_port=a.data_port, engine=eng, out_dir=a.out_dir,
               out_ext=a.out_ext, verbose=a.verbose, chunk=a.chunk, p2p_backend=a.p2p_backend)
    while True:
        try:
            line = input("\nEnter request to become requester or end to stop requesting or quit to exit\n")
        except EOFError:
            line = "quit"
        if "request" in line:
            parts = line.split(" ")
            if len(parts) < 2:
                print("usage: request live|<path>")
                continue
            w.become_requester(parts[1])
        elif line == "end":
            w.stop_requesting_thread()
        else:
            w.exit_threads()
            print("done.")
            return 0


def train_main(argv=None):
    from ..jobs.train import main as tmain

    return tmain(argv)


def video_main(argv=None):
    """One-node video job, one process per GPU (torchrun): rank 0 hosts the coordinator on the
    p2p data plane and requests; every other rank is a worker volunteer (control/node_job.py)."""
    import os

    import torch

    ap = argparse.ArgumentParser(prog="video", description=video_main.__doc__)
    ap.add_argument("--source", default="synthetic:1000:1280x720")
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--out-ext", default=".y4m", choices=[".y4m", ".npy", ""])
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--port", type=int, default=9999, help="coordinator UDP control port")
    ap.add_argument("--store-port", type=int, default=config.get().store_port_video)
    a = ap.parse_args(argv)
    from ..control.node_job import run_node_job
    from ..jobs.video import DetectorEngine

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count()) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    res = run_node_job(a.source, a.out_dir, engine_factory=lambda: DetectorEngine(device=dev), chunk=a.chunk,
                       control_port=a.port, store_port=a.store_port, out_ext=a.out_ext)
    if int(os.environ.get("RANK", "0")) == 0:
        print(res, flush=True)
    return 0


def status_main(argv=None):
    """Print a running coordinator's status (pool, queue, data plane, per-volunteer metrics)."""
    import json

    ap = argparse.ArgumentParser(prog="status", description=status_main.__doc__)
    ap.add_argument("server_ip", nargs="?", default="localhost")
    ap.add_argument("--port", type=int, default=9999, help="coordinator UDP control port")
    ap.add_argument("--config", action="store_true", help="print this process's runtime config instead")
    a = ap.parse_args(argv)
    if a.config:
        print(config.describe())
        return 0
    from ..control import protocol

    cc = protocol.ControlClient(a.server_ip, a.port, retries=3)
    try:
        print(json.dumps(json.loads(cc.call("status", "status:0")), indent=2))
    except TimeoutError as e:
        print(f"no reply: {e}", file=sys.stderr)
        return 1
    return 0


COMMANDS = {"server": server_main, "worker": worker_main, "train": train_main, "video": video_main,
            "status": status_main}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print(f"usage: vcx {{{'|'.join(COMMANDS)}}} ...  (or python -m distributedvolunteercomputing_amd.cli.main)")
        return 2
    return COMMANDS[argv[0]](argv[1:])


if __name__ == "__main__":
    sys.exit(main())
