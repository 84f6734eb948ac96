"""The volunteer client: worker role (batched inference on chunks) and requester role
(capture -> chunk -> submit -> reassemble in order -> write video).

Public API kept from the reference (/root/reference/worker.py):
``client(server_ip='localhost', own_ip='localhost')``, ``.become_requester(path)``,
``.stop_requesting_thread()``, ``.exit_threads()``, ``.log(msg)``, tunables ``verbose``,
``req_rep``, ``number_of_frames_in_chunk=100``, ``max_buffer=4000``, ``my_port='5554'``; the job
prints ``final frame time taken for the job = <sec>`` like the reference.

Behavioural fixes, each deliberate:
* the first frame is processed (the reference reads it only to size the writer and drops it);
* the tail chunk (< 100 frames) is sent (the reference drops it: worker.py:126);
* chunks are contiguous [n, H, W, 3] arrays (no strip-packing index misalignment);
* a chunk is inferred as ONE batch on the GPU;
* frames are pre-resized to the 400-px annotation width on the requester (the worker would
  resize them anyway, worker.py:243), cutting the uplink ~10x for 720p input;
* heartbeats keep the lease alive; a dead worker's chunks are re-dispatched by the coordinator.
"""
from __future__ import annotations

import os
import queue
import threading
import time

import numpy as np
import torch

from ..io.video import open_sink, open_source
from ..jobs.video import DetectorEngine, Engine, OrderedSink
from ..ops import vision as V
from ..utils.metrics import Metrics
from . import protocol
from .transport import FrameHub, FrameSender


class client:  # noqa: N801 (reference class name)
    verbose = False
    req_rep = True
    number_of_frames_in_chunk = 100
    max_buffer = 4000
    my_port = "5554"
    heartbeat_s = 1.0
    preresize = True

    def log(self, message):
        if self.verbose:
            print(message, flush=True)

    def __init__(self, server_ip: str = "localhost", own_ip: str = "localhost", *,
                 control_port: int = protocol.DEFAULT_CONTROL_PORT, my_port: int | str | None = None,
                 engine: Engine | None = None, out_dir: str = ".", out_ext: str = ".y4m",
                 verbose: bool | None = None, chunk: int | None = None):
        if verbose is not None:
            self.verbose = verbose
        if chunk is not None:
            self.number_of_frames_in_chunk = chunk
        self.server_ip = server_ip
        self.out_dir = out_dir
        # requester-side batched pre-resize runs on the GPU when there is one (CPU volunteers
        # send raw frames; the worker resizes them as the reference does, worker.py:243)
        self.resize_device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        self.out_ext = out_ext
        self.metrics = Metrics("client")
        self.engine = engine
        self._engine_lock = threading.Lock()
        # data port first: the coordinator connects to it while handling our join
        port = int(self.my_port if my_port is None else my_port)
        self.hub = FrameHub(port, REQ_REP=self.req_rep, capacity=8)
        self.my_ip = f"{own_ip}:{self.hub.port}"
        self.ctrl = protocol.ControlClient(server_ip, control_port, verbose=self.verbose)
        self.hb_ctrl = protocol.ControlClient(server_ip, control_port, timeout_s=0.5)  # own socket: no reply theft
        self.connect_to_port = self.ctrl.call("join", self.my_ip)
        self.sender = FrameSender(f"tcp://{server_ip}:{self.connect_to_port}", REQ_REP=self.req_rep)
        self.log(f"joined {server_ip}:{control_port}; uplink port {self.connect_to_port}, data port {self.hub.port}")

        # job state (requester role)
        self.path_out_num = 0
        self.path_out = None
        self.start_time = 0.0
        self.final_sent_frame = 0
        self.sink: OrderedSink | None = None
        self.job_times: list[float] = []

        self.send_q: queue.Queue = queue.Queue(maxsize=self.max_buffer)
        self.work_q: queue.Queue = queue.Queue(maxsize=4)
        self.continue_requesting = False
        self.continue_procesing = True
        self.continue_sending = True
        self.continue_receiving = True
        self._threads = []
        for fn, nm in ((self.worker, "worker"), (self.send_image_thread, "send"),
                       (self.recv_image_thread, "recv"), (self._heartbeat, "hb")):
            t = threading.Thread(target=fn, name=f"vcx-client-{nm}", daemon=True)
            t.start()
            self._threads.append(t)
        self._req_thread = None

    # ------------------------------------------------------------------ engine
    def _get_engine(self) -> Engine:
        with self._engine_lock:
            if self.engine is None:
                self.engine = DetectorEngine()
            return self.engine

    # ------------------------------------------------------------------ requester role
    def requester(self, path):
        self.path_out = os.path.join(self.out_dir, f"video{self.path_out_num}{self.out_ext}")
        self.path_out_num += 1
        if self.sink is not None:
            self.sink.close()
        self.final_sent_frame = 0
        src = open_source(path)
        time.sleep(0.0 if path != "live" else 0.5)  # camera warm-up in the reference: 2 s
        out_path = self.path_out

        def done(sink):
            dt = sink.t_done - self.start_time
            self.job_times.append(dt)
            self.metrics.observe("job_s", dt)
            print(f"final frame time taken for the job = {dt}", flush=True)

        self.sink = OrderedSink(lambda w, h: open_sink(out_path, w, h, 30), on_done=done)
        self.start_time = time.time()
        n = 0
        while self.continue_requesting:
            ok, frame = src.read()
            if not ok:
                break
            n += 1
            self.send_q.put((n, frame))
        src.release()
        self.final_sent_frame = n
        self.send_q.put(("flush", None))
        self.sink.set_final(n)
        print(f"final frame sent : {n}\n", flush=True)
        if self.continue_requesting:  # EOF (not a user `end`)
            self.stop_requesting_thread()
        self.log("requester terminated.")

    def become_requester(self, path):
        self.ctrl.call("request", self.my_ip)
        self.continue_requesting = True
        self._req_thread = threading.Thread(target=self.requester, args=(path,), name="vcx-requester", daemon=True)
        self._req_thread.start()

    def stop_requesting_thread(self):
        self.ctrl.call("stop", self.my_ip)
        self.continue_requesting = False

    def wait_job(self, timeout: float | None = None) -> float | None:
        """Block until the current job's last frame is written; returns its wall time."""
        if self._req_thread is not None:
            self._req_thread.join(timeout)
        if self.sink is None:
            return None
        if not self.sink.done.wait(timeout):
            return None
        return self.job_times[-1] if self.job_times else None

    # ------------------------------------------------------------------ send (chunk packing)
    def send_image_thread(self):
        frames, nums = [], []
        C = self.number_of_frames_in_chunk

        def flush():
            if not frames:
                return
            chunk = np.stack(frames)
            if self.preresize and self.resize_device is not None and chunk.shape[2] != 400:
                # one batched resize kernel per chunk on this volunteer's GPU: ~10x less uplink
                t = torch.from_numpy(chunk).to(self.resize_device, non_blocking=True)
                chunk = V.resize_width(t, 400).cpu().numpy()
            info = f"{self.my_ip}||request||{'-'.join(map(str, nums))}||{chunk.shape[1]}||{chunk.shape[2]}"
            if not self.sender.send_image(info, chunk):
                self.log("uplink send failed")
            self.metrics.incr("chunks_sent")
            frames.clear()
            nums.clear()

        while self.continue_sending:
            try:
                item = self.send_q.get(timeout=0.2)
            except queue.Empty:
                continue
            n, f = item
            if n == "flush":
                flush()
                continue
            if frames and f.shape != frames[0].shape:
                flush()  # a chunk holds frames of one size only
            frames.append(f)
            nums.append(n)
            if len(frames) >= C:
                flush()

    # ------------------------------------------------------------------ receive
    def recv_image_thread(self):
        while self.continue_receiving:
            r = self.hub.recv_frame(timeout=0.2)
            if r is None:
                continue
            hdr, arr, _ = r
            parts = hdr["msg"].split("||")
            requester, command = parts[0], parts[1]
            nums = [int(x) for x in parts[2].split("-")] if parts[2] else []
            if command == "request":
                self.work_q.put((hdr, arr, requester, nums))
            elif command == "processed":
                if requester != self.my_ip or self.sink is None:
                    print("frame not mine.", flush=True)
                    continue
                for i, n in enumerate(nums):
                    self.sink.push(n, arr[i])

    # ------------------------------------------------------------------ worker role
    def worker(self):
        """Worker role, two chunks deep: chunk k+1 is submitted to the engine (its host copy and
        H2D start at once) before chunk k's result is collected and sent, so the upload of one
        chunk overlaps the network of the previous one (DetectorEngine.submit)."""
        pending = None
        while self.continue_procesing:
            try:
                item = self.work_q.get(timeout=0.002 if pending is not None else 0.2)
            except queue.Empty:
                item = None
            if item is not None:
                hdr, arr, requester, nums = item
                job = self._get_engine().submit(arr, requester)
                nxt = (job, hdr, requester, nums, time.perf_counter())
            else:
                nxt = None
            if pending is not None and (nxt is not None or self.work_q.empty()):
                self._finish(*pending)
                pending = None
            pending = nxt if nxt is not None else pending
        if pending is not None:
            self._finish(*pending)

    def _finish(self, job, hdr, requester, nums, t0):
        out, counts = job.result()
        self.metrics.observe("chunk_infer_ms", (time.perf_counter() - t0) * 1e3)
        self.metrics.incr("frames_processed", len(nums))
        info = f"{requester}||processed||{'-'.join(map(str, nums))}||{out.shape[1]}||{out.shape[2]}"
        self.sender.send_image(info, out, chunk=hdr.get("chunk", -1))

    # ------------------------------------------------------------------ heartbeat / leave
    def _heartbeat(self):
        while self.continue_receiving:
            time.sleep(self.heartbeat_s)
            try:
                self.hb_ctrl.call("hb", self.my_ip, retries=1)
            except Exception:
                pass

    def exit_threads(self):
        try:
            self.ctrl.call("end", self.my_ip, retries=5)
        except TimeoutError:
            pass
        self.continue_requesting = False
        self.continue_procesing = False
        self.continue_sending = False
        self.continue_receiving = False
        for t in self._threads:
            t.join(timeout=2)
        self.hub.close()
        self.sender.close()
        if self.sink is not None:
            self.sink.close()


Client = client
