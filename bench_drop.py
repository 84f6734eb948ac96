#!/usr/bin/env python3
"""Step time under a 1-peer drop: the second half of the BASELINE.json metric
("samples/sec GPT-2-small local-SGD at 1/2/4/8 peers; step-time under 1-peer drop").

    python bench_drop.py --peers P [--model gpt2] [--batch 64] [--steps 24] [--warmup 8] [--lease 1.0]
                         [--fault step|collective|stop] [--drop-peers 3,4]

Faults: ``step`` — the victim exits between two steps (heartbeat stops); ``collective`` — the
victim SIGKILLs itself from INSIDE the averaging all-reduce of the first round at or after
``--drop-at`` (the other peers are blocked in that collective: their watchdog or the failed
transport aborts it, they recover to a new generation and redo the round); ``stop`` — the
victim SIGSTOPs itself inside the collective (no socket error anywhere: only the lease-based
watchdog can tell), and stays frozen until the launcher kills it at the end.

This process plays the coordinator: it hosts the rendezvous store (so no peer is special and
any peer may die) and starts P peer processes, one per visible GPU (round-robin when P exceeds
the GPUs; RCCL does not run two ranks on one device, so peers sharing a GPU use gloo). Every
peer runs the elastic local-SGD trainer (parallel/elastic.py + parallel/local_sgd.py). At step
``--drop-at`` (default: mid-window, between two averaging rounds) peer ``--drop-peer`` crashes
without a goodbye (the process exits). The survivors notice at once through their liveness links
to it (a closed TCP connection; a SIGSTOPped victim closes nothing and is found by the lease),
agree on the next generation, build a fresh process group and go on. The JSON line breaks the
stall into ``detect_ms`` (fault -> first sign), ``comm_build_ms`` (the new communicator) and
``redo_ms`` (new communicator -> end of the redone round). Every peer times each step (device-synchronised); the launcher prints ONE JSON line
with the step time before the drop, across the window that contains it, after it, and the
stall of the round that absorbed the detection and regroup.

Reference analog: the reference has no failure handling (a dead volunteer hangs the job,
SURVEY.md §5.3); this measures the replacement.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=2)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--steps", type=int, default=24, help="timed window (contains the drop)")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--drop-at", type=int, default=None, help="step at which the peer dies (default: mid-window)")
    ap.add_argument("--drop-peer", type=int, default=None, help="default: the last peer")
    ap.add_argument("--drop-peers", default=None, help="comma-separated victims (overrides --drop-peer)")
    ap.add_argument("--fault", default="step", choices=["step", "collective", "stop"])
    ap.add_argument("--lease", type=float, default=1.0, help="heartbeat lease (s) after which a silent peer is dead")
    ap.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--timeout", type=float, default=900.0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--rejoin", action="store_true",
                    help="respawn each killed victim; it joins the running job (BASELINE config 4: kill then rejoin)")
    ap.add_argument("--after-rejoin", type=int, default=8,
                    help="with --rejoin: survivors keep stepping until the full group ran this many steps")
    # internal (peer processes)
    ap.add_argument("--peer", type=int, default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--join", action="store_true", help="(internal) a replacement peer joining the running job")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- peer
def peer_main(a):
    import faulthandler

    from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms

    # a peer still running shortly before the launcher's kill prints every thread's Python stack
    # (where a hung peer sits) to its log
    faulthandler.dump_traceback_later(max(5.0, a.timeout - 15.0), exit=False)

    ngpu = int(os.environ.get("VCX_DROP_NGPU", "0"))
    local = a.peer % ngpu if ngpu else 0
    enable_tuned_gemms(local)
    import torch
    import torch.distributed as dist

    import signal

    from distributedvolunteercomputing_amd.models.gpt2 import GPT2, GPT2Config
    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    cuda = ngpu > 0
    device = torch.device("cuda", local) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    backend = a.backend or ("nccl" if cuda and ngpu >= a.peers else "gloo")
    store = dist.TCPStore("127.0.0.1", a.port, None, False, timeout=datetime.timedelta(seconds=300),
                          wait_for_workers=False)
    mem = ElasticMembership(store, a.peer, backend=backend, device=device, lease_s=a.lease,
                            heartbeat_s=max(a.lease / 10, 0.02))
    victims = [int(v) for v in a.drop_peers.split(",")]
    armed = {"on": False}
    if a.peer in victims and a.fault != "step":
        sig = signal.SIGKILL if a.fault == "collective" else signal.SIGSTOP

        def hook(grp, op):  # fires after the op was issued: the other peers are inside it
            if armed["on"] and op in ("allreduce", "alltoall", "all_gather"):
                print(f"[peer {a.peer}] fault injection: {signal.Signals(sig).name} inside {op}", flush=True)
                store.set(f"vcx/drop/t_fault/{a.peer}", repr(time.time()))
                os.kill(os.getpid(), sig)
        mem.fault_hook = hook
    if a.join:
        mem.join()
    else:
        mem.bootstrap(list(range(a.peers)))
    cfg = GPT2Config.preset(a.model)
    cfg.n_ctx = max(cfg.n_ctx, a.seq)
    torch.manual_seed(0)
    dtype = torch.bfloat16 if cuda else torch.float32
    model = GPT2(cfg).to(device=device, dtype=dtype)
    tcfg = LocalSGDConfig(H=a.H, comm_dtype=dtype)
    tr = LocalSGDTrainer(model, tcfg, membership=mem, device=device)
    if a.join:
        return joiner_loop(a, tr, mem, store, cfg, device, cuda)
    g = torch.Generator(device=device).manual_seed(1000 + a.peer)
    pool = [torch.randint(0, cfg.vocab_size, (a.batch, a.seq + 1), device=device, generator=g) for _ in range(4)]

    def batch(i):
        b = pool[i % len(pool)]
        return b[:, :-1], b[:, 1:]

    def sync():
        if cuda:
            torch.cuda.synchronize()

    w0 = 0
    if a.graph and cuda:
        w0 = min(3, a.warmup)
        tr.capture(*batch(0), warmup=w0)
    for i in range(w0, a.warmup):
        tr.step(*batch(i))
    sync()
    mem.group.barrier()
    timeline = []
    i = a.warmup
    t_cap = time.time() + a.timeout * 0.8
    full_since = None
    gen_at_drop = 1 << 30
    while True:
        if i == a.drop_at:
            gen_at_drop = mem.gen
        if i >= a.warmup + a.steps:
            if not a.rejoin or a.peer in victims:
                break
            # config 4: keep going until the victims are back and the full group ran a while
            # (the drop and the rejoin can land in ONE new generation when the replacements
            # register before the survivors agree on the recovery round)
            if timeline and timeline[-1]["members"] == a.peers and timeline[-1]["gen"] > gen_at_drop:
                full_since = i if full_since is None else full_since
                if i - full_since >= a.after_rejoin:
                    break
            if time.time() > t_cap:
                break
        if a.peer in victims and i == a.drop_at:
            if a.fault == "step":
                print(f"[peer {a.peer}] fault injection: crashing at step {i}", flush=True)
                store.set(f"vcx/drop/t_fault/{a.peer}", repr(time.time()))
                os._exit(0)  # no leave(), no goodbye: the survivors must notice on their own
            armed["on"] = True  # die inside the next averaging collective
        t0 = time.perf_counter()
        st = tr.step(*batch(i))
        sync()
        timeline.append({"step": i, "ms": (time.perf_counter() - t0) * 1e3, "synced": bool(st.synced),
                         "members": st.members, "gen": mem.gen, "sync_ms": st.sync_ms if st.synced else 0.0,
                         "t_end": time.time(), "t_sync_end": tr.t_sync_end if st.synced else None,
                         "admit_stages": tr.last_round_stages if st.synced else None})
        i += 1
    store.set("vcx/drop/done", "1")
    with open(os.path.join(a.out, f"peer{a.peer}.json"), "w") as f:
        t_fault = {v: float(store.get(f"vcx/drop/t_fault/{v}")) for v in victims
                   if store.check([f"vcx/drop/t_fault/{v}"])}
        json.dump({"peer": a.peer, "backend": backend, "timeline": timeline, "events": mem.events,
                   "failed_rounds": tr.failed_rounds, "eof": mem.eof_events, "t_fault": t_fault}, f)
    mem.leave()  # graceful: a joiner still stepping regroups without this peer at its next round
    return 0


def joiner_loop(a, tr, mem, store, cfg, device, cuda):
    """A replacement peer: admitted into the running job (params, anchor and buffers streamed from
    a member), then steps with the group until the survivors are done."""
    import torch

    t0 = time.perf_counter()
    tr.join_running_job()
    admit_ms = (time.perf_counter() - t0) * 1e3
    g = torch.Generator(device=device).manual_seed(2000 + a.peer)
    pool = [torch.randint(0, cfg.vocab_size, (a.batch, a.seq + 1), device=device, generator=g) for _ in range(2)]
    n = 0
    if a.graph and cuda:  # replay the local step as one hipGraph like the other peers
        tr.capture(pool[0][:, :-1], pool[0][:, 1:], warmup=1)
        n = 1
    while not store.check(["vcx/drop/done"]):
        b = pool[n % len(pool)]
        tr.step(b[:, :-1], b[:, 1:])
        n += 1
    if cuda:
        torch.cuda.synchronize()
    with open(os.path.join(a.out, f"joiner{a.peer}.json"), "w") as f:
        json.dump({"peer": a.peer, "admit_ms": admit_ms, "admit_stages": getattr(tr, "admit_stages", None), "steps": n,
                   "gen": mem.gen, "events": mem.events}, f)
    mem.leave()
    return 0


# ----------------------------------------------------------------------------- launcher
def launcher(a):
    import torch
    import torch.distributed as dist

    ngpu = torch.cuda.device_count()  # does not initialise the GPU in this process
    if a.drop_peer is None:
        a.drop_peer = a.peers - 1
    if a.drop_peers is None:
        a.drop_peers = str(a.drop_peer)
    victims = [int(v) for v in a.drop_peers.split(",")]
    if a.drop_at is None:
        a.drop_at = a.warmup + a.steps // 2 + (1 if a.H > 1 else 0)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    store = dist.TCPStore("127.0.0.1", port, None, True, timeout=datetime.timedelta(seconds=300),
                          wait_for_workers=False)
    out = tempfile.mkdtemp(prefix="vcx_drop_")
    env = dict(os.environ, VCX_DROP_NGPU=str(ngpu), PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    common = [sys.executable, os.path.abspath(__file__), "--peers", str(a.peers), "--model", a.model,
              "--batch", str(a.batch), "--seq", str(a.seq), "--H", str(a.H), "--steps", str(a.steps),
              "--warmup", str(a.warmup), "--drop-at", str(a.drop_at), "--drop-peers", a.drop_peers,
              "--fault", a.fault,
              "--lease", str(a.lease), "--graph", str(a.graph), "--port", str(port), "--out", out]
    if a.backend:
        common += ["--backend", a.backend]
    if a.rejoin:
        common += ["--rejoin", "--after-rejoin", str(a.after_rejoin), "--timeout", str(a.timeout)]
    def peer_env(r):
        if a.backend == "nccl" and a.peers > max(ngpu, 1):
            # RCCL rehearsal with several peers per GPU: a distinct host identity per peer gets past
            # RCCL's duplicate-GPU check, and the communicators run over loopback sockets
            # (scripts/rccl_rehearsal_launch.py); the RCCL code paths are the real ones
            return dict(env, NCCL_HOSTID=f"vcx-peer-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        return env

    procs = [subprocess.Popen(common + ["--peer", str(r)], env=peer_env(r)) for r in range(a.peers)]
    t_end = time.time() + a.timeout
    rc = {}
    survivors = [r for r in range(a.peers) if r not in victims]
    joiners = {}
    t_dead = {}
    t_beat = time.time()
    while not all(r in rc for r in survivors) and time.time() < t_end:
        if time.time() - t_beat > 30:  # progress for a supervisor that kills silent runs
            t_beat = time.time()
            print(f"[bench_drop] waiting: exited {rc}, joiners {sorted(joiners)}", file=sys.stderr, flush=True)
        for r, p in enumerate(procs):
            if r not in rc and p.poll() is not None:
                rc[r] = p.returncode
                t_dead[r] = time.time()
        if a.rejoin:
            for v in victims:
                if v in rc and v not in joiners:  # the victim is gone: start its replacement
                    joiners[v] = subprocess.Popen(common + ["--peer", str(v), "--join"], env=peer_env(v))
        time.sleep(0.2)
    for v, p in joiners.items():
        deadline = max(t_end, time.time() + 5.0)
        while p.poll() is None and time.time() < deadline:
            try:
                p.wait(timeout=min(30.0, max(1.0, deadline - time.time())))
            except subprocess.TimeoutExpired:
                print(f"[bench_drop] waiting for joiner {v}", file=sys.stderr, flush=True)
        if p.poll() is None:
            p.kill()
            p.wait()
        if p.returncode != 0:
            print(f"[bench_drop] joiner {v} exited with {p.returncode}", file=sys.stderr)
    for r, p in enumerate(procs):
        if r not in rc:
            p.kill()  # timeout, or a SIGSTOPped victim still frozen
            p.wait()
            rc[r] = "timeout" if r in survivors else "killed"
    bad = {r: c for r, c in rc.items() if r in survivors and c != 0}
    if bad:
        print(f"[bench_drop] peers failed: {bad}", file=sys.stderr)
        return 1
    tl = {}
    backend = None
    failed_rounds = 0
    detect, build, redo = [], [], []
    stages = {}  # regroup-round anatomy, max over survivors (where a slow one goes)
    staged = []  # staged admission on the survivors: (bg build ms, connect wait ms, go wait ms)
    for r in survivors:
        with open(os.path.join(out, f"peer{r}.json")) as f:
            d = json.load(f)
        backend = d["backend"]
        for e in d["events"]:
            if e["event"] == "staged":
                cn = [c for c in d["events"] if c["event"] == "connect" and c["gen"] == e["gen"]]
                go = [c for c in d["events"] if c["event"] == "go" and c["gen"] == e["gen"]]
                staged.append({"gen": e["gen"], "bg_build_ms": cn[0].get("bg_build_ms") if cn else None,
                               "connect_wait_ms": cn[0]["ms"] if cn else 0.0, "go_wait_ms": go[0]["ms"] if go else None})
        failed_rounds = max(failed_rounds, d.get("failed_rounds", 0))
        tf = min(d.get("t_fault", {}).values(), default=None)
        if tf is not None:
            # detection: the first sign of the failure on this survivor (a liveness EOF from a
            # victim, an aborted collective, or — without either — the regroup itself)
            sig = [t for m, t in d.get("eof", []) if m in victims and t >= tf]
            sig += [e["t"] for e in d["events"] if e["event"] == "abort" and e["t"] >= tf]
            rg = [e for e in d["events"] if e["event"] == "regroup" and e.get("t", 0) >= tf]
            if rg and not sig:
                sig = [rg[0]["t"]]
            if sig:
                detect.append((min(sig) - tf) * 1e3)
            if rg:
                cn = [e for e in d["events"] if e["event"] == "connect" and e["gen"] == rg[0]["gen"]]
                if cn:
                    build.append(cn[0]["ms"])
                    # redo: from the new generation's communicator to the end of the step that
                    # carried the redone (or delayed) averaging round
                    ends = [e["t_end"] for e in d["timeline"] if e["gen"] >= rg[0]["gen"] and e["synced"]]
                    if ends:
                        redo.append((min(ends) - cn[0]["t"]) * 1e3)
                # the averaging call that absorbed the failure, stage by stage
                st_ = next((e for e in d["timeline"] if e["gen"] >= rg[0]["gen"] and e["synced"]), None) if rg else None
                if st_ is not None and st_.get("t_sync_end") and rg[0].get("t_in"):
                    t1 = st_["t_sync_end"]
                    t0 = t1 - st_["sync_ms"] / 1e3
                    ab = [e["t"] for e in d["events"] if e["event"] == "abort" and t0 <= e["t"] <= t1]
                    cn = [e for e in d["events"] if e["event"] == "connect" and e["gen"] == rg[0]["gen"]]
                    parts = {
                        # sync start -> first sign of trouble inside it (aborted collective), if any
                        "before_abort_ms": (min(ab) - t0) * 1e3 if ab else 0.0,
                        # (abort ->) entry into the round that formed the new generation
                        "to_round_ms": (rg[0]["t_in"] - (min(ab) if ab else t0)) * 1e3,
                        "bell_wait_ms": rg[0].get("bell_wait_ms") or 0.0,
                        "scan_ms": rg[0].get("scan_ms") or 0.0,
                        "decide_ms": rg[0].get("decide_ms") or 0.0,
                        "group_object_ms": rg[0].get("adopt_ms") or 0.0,
                        "comm_build_ms": cn[0]["ms"] if cn else 0.0,
                        "collective_after_build_ms": (t1 - cn[0]["t"]) * 1e3 if cn else 0.0,
                    }
                    acc = parts["before_abort_ms"] + parts["to_round_ms"] + parts["decide_ms"] + \
                        parts["group_object_ms"] + parts["comm_build_ms"] + parts["collective_after_build_ms"]
                    parts["unaccounted_ms"] = st_["sync_ms"] - acc
                    parts["sync_ms"] = st_["sync_ms"]
                    for k_, v_ in parts.items():
                        stages[k_] = max(stages.get(k_, v_), v_)
        for e in d["timeline"]:
            cur = tl.setdefault(e["step"], dict(e))
            cur["ms"] = max(cur["ms"], e["ms"])  # a step ends when its slowest survivor is done
            if e.get("admit_stages"):  # members' admission-round anatomy, max over survivors
                ms = cur.setdefault("member_stages", {})
                for k_, v_ in e["admit_stages"].items():
                    ms[k_] = max(ms.get(k_, v_), v_)
    steps = sorted(tl)
    before = [tl[s]["ms"] for s in steps if s < a.drop_at]
    gen_before = max((tl[s]["gen"] for s in steps if s < a.drop_at), default=0)
    regroup = next((s for s in steps if s >= a.drop_at and tl[s]["gen"] > gen_before and tl[s]["synced"]), None)
    # after the drop: the survivors-only steps (without --rejoin: every step after the regroup)
    after = [tl[s]["ms"] for s in steps if regroup is not None and s > regroup
             and (not a.rejoin or tl[s]["members"] < a.peers)]
    window = [tl[s]["ms"] for s in steps]
    mean = lambda xs: sum(xs) / len(xs) if xs else float("nan")  # noqa: E731
    # the stall: the averaging call that detected the silent peer (lease wait + agreement + new
    # process group + first collective on it) against a steady averaging call before the drop
    steady_sync = mean([tl[s]["sync_ms"] for s in steps if s < a.drop_at and tl[s]["synced"]])
    regroup_sync = tl[regroup]["sync_ms"] if regroup is not None else float("nan")
    rec = {
        "metric": "step-time under 1-peer drop, GPT-2-small local-SGD",
        "value": round(mean(window), 3),
        "unit": "ms/step",
        "n_gpus": min(ngpu, a.peers) if ngpu else 0,
        "peers": a.peers,
        "steps": a.steps,
        "warmup": a.warmup,
        "higher_is_better": False,
        "dtype": "bf16" if ngpu else "fp32",
        "data": "synthetic (random tokens, random-init weights)",
        "config": {"model": a.model, "per_peer_batch": a.batch, "seq_len": a.seq, "H": a.H,
                   "backend": backend, "lease_s": a.lease, "drop_at": a.drop_at, "drop_peers": victims,
                   "fault": a.fault},
        "rounds_aborted_and_redone": failed_rounds,
        "ms_per_step_before": round(mean(before), 3),
        "ms_per_step_after": round(mean(after), 3),
        "regroup_step": regroup,
        "steady_sync_ms": round(steady_sync, 3),
        "regroup_sync_ms": round(regroup_sync, 3),
        "drop_stall_ms": round(regroup_sync - steady_sync, 3),
        # stall anatomy (max over survivors): fault -> first sign of it, the new generation's
        # communicator build, and communicator -> end of the redone round
        "detect_ms": round(max(detect), 3) if detect else None,
        "comm_build_ms": round(max(build), 3) if build else None,
        "redo_ms": round(max(redo), 3) if redo else None,
        "regroup_stages_ms": {k: round(v, 3) for k, v in stages.items()} or None,
        "liveness": os.environ.get("VCX_ELASTIC_LIVENESS", "1") not in ("0", "false", "no", "off"),
        "samples_per_s_before": round(a.peers * a.batch / mean(before) * 1e3, 2),
        "samples_per_s_after": round(len(survivors) * a.batch / mean(after) * 1e3, 2) if after else None,
    }
    if a.rejoin:
        rj = next((s for s in steps if regroup is not None and s >= regroup and tl[s]["members"] == a.peers), None)
        back = [tl[s]["ms"] for s in steps if rj is not None and s > rj]
        adm, adm_st = [], []
        for v in victims:
            fn = os.path.join(out, f"joiner{v}.json")
            if os.path.exists(fn):
                with open(fn) as f:
                    jd = json.load(f)
                adm.append(jd["admit_ms"])
                adm_st.append(jd.get("admit_stages"))
        rec["metric"] = "step-time under peer drop and rejoin, local-SGD"
        rec["rejoin_step"] = rj
        rec["rejoin_sync_ms"] = round(tl[rj]["sync_ms"], 3) if rj is not None else None
        # joiner_admission_ms: the joiner's whole join_running_job (communicator connect, the wait for
        # the members to finish their local steps, the admission round); joiner_admission_round_ms:
        # the admission round alone (model broadcast + reduction + verdict/apply); rejoin_stall_ms:
        # what the admission round cost the running members over a steady averaging round
        rec["joiner_admission_ms"] = [round(x, 1) for x in adm]
        rec["joiner_admission_round_ms"] = [round(s_["admission_round_ms"], 1) for s_ in adm_st
                                            if s_ and "admission_round_ms" in s_]
        rec["joiner_admission_stages"] = adm_st
        sj = os.environ.get("VCX_ELASTIC_STAGE_JOINS", "gloo")
        rec["staged_admission"] = sj == "gloo" and backend == "gloo"
        # per survivor: how long its background communicator build ran, what was left of it to wait
        # for at the switch, and the line-up wait before the admission round
        rec["staged_survivors"] = staged
        rec["rejoin_stall_ms"] = round(tl[rj]["sync_ms"] - steady_sync, 3) if rj is not None else None
        # the running members' side of that stall (max over survivors): membership agreement, the new
        # group's communicator init (its first, one-element collective), the model broadcast, the
        # reduction, guard / verdict / apply -- their sum is the members' admission averaging call
        rec["rejoin_member_stages_ms"] = tl[rj].get("member_stages") if rj is not None else None
        rec["ms_per_step_after_rejoin"] = round(mean(back), 3) if back else None
        rec["samples_per_s_after_rejoin"] = round(a.peers * a.batch / mean(back) * 1e3, 2) if back else None
    line = json.dumps(rec)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    del store
    return 0


def main(argv=None):
    a = parse(argv)
    if a.peer is not None:
        return peer_main(a)
    return launcher(a)


if __name__ == "__main__":
    sys.exit(main())
