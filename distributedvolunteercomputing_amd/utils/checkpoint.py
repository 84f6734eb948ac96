"""Training checkpoint format ("vcx-ckpt-v1") with restore onto a different peer count.

The reference persists nothing but ``video<N>.mp4``, so this format is
defined here. One directory per step:

    <root>/step_<step:08d>/
        manifest.json            format, step, generation, members, model config, flat layout
                                 (segment name/offset/numel/shape/decay), optimizer config,
                                 and the list of shard files with the flat [lo, hi) range each covers
        params.safetensors       the bf16 flat parameter buffer, the optimizer scalars ("ostate") and
                                 global extras: "buffers" (BN running stats, fp32), "psgd_Q"
                                 (PowerSGD warm start) — written by one peer
        state_<peer>.safetensors fp32 optimizer-state slices ("master", "m", "v", ["outer_mom"],
                                 ["ef": mean error feedback]) of the flat range [lo, hi) this peer
                                 owned; per-peer quantities (local-SGD moments, error feedback)
                                 are stored as their mean over the peers

Tensors are stored with safetensors (no pickle: loading executes nothing from the file).
A checkpoint written by P peers can be restored by P' peers: every peer reads just the flat
ranges it needs from whichever shard files cover them (``ShardReader.read_range``).
A ``LATEST`` file in the root names the newest complete step (written last, atomically).
"""
from __future__ import annotations

import json
import os
import time

import torch
from safetensors.torch import load_file, safe_open, save_file

FORMAT = "vcx-ckpt-v1"


def _step_dir(root, step):
    return os.path.join(root, f"step_{int(step):08d}")


def layout_dict(flat) -> dict:
    return {"numel": flat.numel, "n_decay": flat.n_decay,
            "segments": [{"name": s.name, "offset": s.offset, "numel": s.numel, "shape": list(s.shape),
                          "decay": s.decay, "channels_last": s.channels_last} for s in flat.segments]}


def save_checkpoint(trainer, root: str, step: int, *, peer_id: int, is_writer: bool, members=None,
                    generation: int = 0, model_config: dict | None = None, extra: dict | None = None,
                    barrier=None) -> str:
    """Every peer calls this; each writes its own state slice, the writer peer also writes the
    parameters and (after `barrier`, if given) the manifest and LATEST."""
    d = _step_dir(root, step)
    os.makedirs(d, exist_ok=True)
    lo, hi, tensors = trainer.checkpoint_slice()
    fname = f"state_{peer_id}.safetensors"
    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, os.path.join(d, fname),
              metadata={"lo": str(lo), "hi": str(hi), "peer": str(peer_id)})
    with open(os.path.join(d, f"state_{peer_id}.json"), "w") as f:
        json.dump({"file": fname, "lo": lo, "hi": hi, "peer": peer_id, "keys": sorted(tensors)}, f)
    if is_writer:
        glob = {"param": trainer.flat.param.detach().cpu(), "ostate": trainer.ostate.detach().cpu()}
        if hasattr(trainer, "checkpoint_global"):  # BN buffers, PowerSGD Q, ...
            glob.update({k: v.detach().contiguous().cpu() for k, v in trainer.checkpoint_global().items()})
        save_file(glob, os.path.join(d, "params.safetensors"))
    if barrier is not None:
        barrier()
    if is_writer:
        shards = []
        for fn in sorted(os.listdir(d)):
            if fn.startswith("state_") and fn.endswith(".json"):
                with open(os.path.join(d, fn)) as f:
                    shards.append(json.load(f))
        man = {"format": FORMAT, "step": int(step), "time": time.time(), "generation": generation,
               "members": list(members or []), "model": model_config or {}, "flat": layout_dict(trainer.flat),
               "trainer": type(trainer).__name__, "shards": shards, "extra": extra or {}}
        tmp = os.path.join(d, "manifest.json.tmp")
        with open(tmp, "w") as f:
            json.dump(man, f, indent=1)
        os.replace(tmp, os.path.join(d, "manifest.json"))
        tmp = os.path.join(root, "LATEST.tmp")
        with open(tmp, "w") as f:
            f.write(os.path.basename(d))
        os.replace(tmp, os.path.join(root, "LATEST"))
    return d


def latest(root: str) -> str | None:
    p = os.path.join(root, "LATEST")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = os.path.join(root, f.read().strip())
    return d if os.path.exists(os.path.join(d, "manifest.json")) else None


class ShardReader:
    def __init__(self, ckpt_dir: str):
        self.dir = ckpt_dir
        with open(os.path.join(ckpt_dir, "manifest.json")) as f:
            self.manifest = json.load(f)
        if self.manifest.get("format") != FORMAT:
            raise ValueError(f"{ckpt_dir}: unknown checkpoint format {self.manifest.get('format')!r}")
        self.shards = sorted(self.manifest["shards"], key=lambda s: (s["lo"], s["peer"]))

    @property
    def step(self) -> int:
        return int(self.manifest["step"])

    def params(self):
        t = load_file(os.path.join(self.dir, "params.safetensors"))
        return t["param"], t["ostate"]

    def global_tensor(self, key: str):
        """A tensor of params.safetensors other than param/ostate, or None."""
        with safe_open(os.path.join(self.dir, "params.safetensors"), framework="pt") as f:
            return f.get_tensor(key) if key in f.keys() else None

    def has_key(self, key: str) -> bool:
        return any(key in s["keys"] for s in self.shards)

    def read_range(self, key: str, lo: int, hi: int) -> torch.Tensor:
        """Assemble flat[lo:hi] of tensor `key` from the shard files that cover it."""
        out = torch.zeros(hi - lo, dtype=torch.float32)
        covered = torch.zeros(hi - lo, dtype=torch.bool)
        for s in self.shards:
            a, b = max(lo, s["lo"]), min(hi, s["hi"])
            if a >= b or key not in s["keys"]:
                continue
            with safe_open(os.path.join(self.dir, s["file"]), framework="pt") as f:
                sl = f.get_slice(key)
                out[a - lo : b - lo] = sl[a - s["lo"] : b - s["lo"]]
            covered[a - lo : b - lo] = True
        if not bool(covered.all()):
            raise ValueError(f"checkpoint {self.dir}: {key}[{lo}:{hi}] not fully covered by any shard")
        return out

    def check_layout(self, flat):
        want = layout_dict(flat)
        have = self.manifest["flat"]
        if have["numel"] != want["numel"] or [s["name"] for s in have["segments"]] != [s["name"] for s in
                                                                                    want["segments"]]:
            raise ValueError("checkpoint flat layout does not match this model")
        # a segment's element order follows its parameter's memory format (flat_params.segment_view)
        fmt = [(s["name"], bool(s.get("channels_last", False))) for s in have["segments"]]
        if fmt != [(s["name"], s["channels_last"]) for s in want["segments"]]:
            raise ValueError("checkpoint parameter memory formats (channels-last) do not match this model")
