"""The reference command lines and REPLs, end to end (VERDICT r2 missing #8).

`python server.py 127.0.0.1 --port P` and two `python worker.py 127.0.0.1 127.0.0.1 --port P
--data-port 0` processes driven through their stdin exactly like a user at the reference's
prompts: the requester types `request synthetic:250:320x180`, waits for the job-time line, types
`end` (stop requesting), then `quit` (any other line quits, /root/reference/worker.py:353-356);
the server gets `quit` (/root/reference/server.py:171-175). The requester's output video must hold
all 250 frames (the reference drops the first frame and the tail chunk) and every process must
exit 0. The detector runs with random weights on the CPU here (no caffemodel in the image).
"""
import os
import queue
import subprocess
import sys
import threading
import time

import numpy as np

from tests import _mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Proc:
    def __init__(self, args, cwd, env):
        self.p = subprocess.Popen([sys.executable, "-u", *args], cwd=cwd, env=env, stdin=subprocess.PIPE,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1)
        self.lines: queue.Queue = queue.Queue()
        self.out: list[str] = []
        threading.Thread(target=self._pump, daemon=True).start()

    def _pump(self):
        for line in self.p.stdout:
            self.out.append(line)
            self.lines.put(line)

    def send(self, line):
        self.p.stdin.write(line + "\n")
        self.p.stdin.flush()

    def wait_for(self, text, timeout):
        t_end = time.time() + timeout
        while time.time() < t_end:
            if any(text in ln for ln in self.out):
                return True
            try:
                self.lines.get(timeout=0.2)
            except queue.Empty:
                pass
        return False


def test_reference_repls_end_to_end(tmp_path):
    port = _mp.free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    srv = _Proc(["server.py", "127.0.0.1", "--port", str(port), "--ephemeral-ports", "--lease", "30"], ROOT, env)
    procs = [srv]
    try:
        assert srv.wait_for("listening on", 60), "".join(srv.out)
        out_req, out_w = tmp_path / "req", tmp_path / "w"
        common = ["worker.py", "127.0.0.1", "127.0.0.1", "--port", str(port), "--data-port", "0", "--out-ext", ".npy"]
        req = _Proc(common + ["--out-dir", str(out_req)], ROOT, env)
        wrk = _Proc(common + ["--out-dir", str(out_w)], ROOT, env)
        procs += [req, wrk]
        for w in (req, wrk):
            assert w.wait_for("Enter request", 120), "".join(w.out)
        req.send("request synthetic:250:320x180")
        assert req.wait_for("final frame time taken for the job", 300), "".join(req.out)[-3000:]
        req.send("end")  # stop requesting: back to the worker pool
        time.sleep(0.5)
        req.send("quit")  # anything else quits (and says `end` to the coordinator)
        wrk.send("quit")
        for w in (req, wrk):
            assert w.p.wait(timeout=60) == 0, "".join(w.out)[-3000:]
        srv.send("quit")
        assert srv.p.wait(timeout=60) == 0, "".join(srv.out)[-3000:]
        video = np.load(out_req / "video0.npy")
        assert video.shape == (250, 225, 400, 3), video.shape  # every frame, annotated at 400 px wide
        assert any("final frame sent : 250" in ln for ln in req.out)
        assert "done." in "".join(req.out) and "done." in "".join(srv.out)
    finally:
        for p in procs:
            if p.p.poll() is None:
                p.p.kill()
                p.p.wait()
