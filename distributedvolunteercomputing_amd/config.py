"""One place for every runtime tunable of the framework.

Each field has a default, an environment variable that overrides it at import time, and can be
changed in code with :func:`update` (or temporarily with :func:`override`). Modules read the
live object (``config.get().field``) at the point of use, never a module-level copy, so an
update takes effect for the next call.

    from distributedvolunteercomputing_amd import config
    config.update(gemm="vcx")            # hand-written MFMA GEMM for the Linear layers
    with config.override(force_reference_ops=True):
        ...                              # plain torch ops (numerics oracle)
    print(config.describe())             # every field, its env var and current value

The reference configures itself with module constants and argv only (/root/reference/worker.py:
16-18, server.py:9-12); those job-level knobs remain command-line flags of the CLIs.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
import threading


def _bool(s: str) -> bool:
    return s.strip().lower() in ("1", "true", "yes", "on")


@dataclasses.dataclass
class RuntimeConfig:
    # ---- compute path
    gemm: str = "lib"  # VCX_GEMM: "lib" (hipBLASLt/rocBLAS) or "vcx" (csrc/kernels/gemm.hip, opt-in: 0.74-0.84x lib)
    mlp: str = "fused"  # VCX_MLP: GPT-2 MLP fc (+bias+GELU) and fc2-dgrad (*gelu' + bias grad) on the persistent
    # hand-written GEMM's fused epilogues (csrc/kernels/gemm_ps.hip), other GEMMs on `gemm`; "lib": library + passes
    # VCX_NARROW_GEMM: GEMMs with <= 128 output columns and >= 32k rows (ResNet 1x1 convolutions) on
    # the vision GEMM ("vision") or the library ("lib")
    narrow_gemm: str = "lib"
    # VCX_MLP_GRAD_FWD: the fused fc forward stores gelu'(pre) instead of pre, so the fc2 input gradient's
    # epilogue is one multiply (gemm_ps epilogues 5 / 6) instead of gelu'(pre) per element (4)
    mlp_grad_fwd: bool = True
    # VCX_GEMM_FWD: forward GEMMs x W^T (+ b) and input gradients dY W of the linear layers on "lib" or "vcx"
    # (csrc/kernels/gemm_f.hip, opt-in: 0.85-0.93x the library at the GPT-2 shapes, profiles/r6_gemm_f.txt)
    gemm_fwd: str = "lib"
    dgrad_ps: bool = True  # VCX_DGRAD_PS: input gradients dX = dY W with K <= 2304 on gemm_ps (measured faster)
    gemm_wgrad: str = "vcx"  # VCX_GEMM_WGRAD: weight gradients on "vcx" (gemm_wg, hand-written) or "lib" (split-M batched GEMM)
    # VCX_WGRAD_WIDE: also outputs of more than 128 256x256 tiles with <= 1024 input columns on gemm_wg (the
    # GPT-2 LM heads, [50304, 768 | 1024]: 1..4 token splits, ragged last row panel)
    wgrad_wide: bool = True
    # VCX_WGRAD_RAGGED: outputs whose row count is a multiple of 128 but not 256 (half-empty last row panel;
    # ResNet-50 stage 2's [128, 256 | 512]) on gemm_wg too -- config 3 8849-8871 vs 8918-8960 img/s without
    # (gpurun_out/c26), so off; the LM heads take the ragged panel regardless
    wgrad_ragged: bool = False
    gemm_select: bool = False  # VCX_GEMM_SELECT: per-shape layout probe of the forward GEMMs (no in-step gain)
    wgrad_big_split_min_m: int = 16384  # VCX_WGRAD_BIG_SPLIT_MIN_M: rows above which weight grads split over K
    async_wgrad: bool = False  # VCX_ASYNC_WGRAD: weight-grad GEMMs on a side stream (measured slower)
    lmhead_chunk: int = 0  # VCX_LMHEAD_CHUNK: token rows per LM-head GEMM + xent pass (0 = one pass)
    force_reference_ops: bool = False  # VCX_FORCE_REFERENCE_OPS: torch ops instead of the HIP kernels
    tunableop: str = "on"  # VCX_TUNABLEOP: "on" loads the shipped hipBLASLt selections, "off" skips them
    tunableop_file: str = ""  # VCX_TUNABLEOP_FILE: alternative TunableOp results file
    offload_arch: str = "gfx950"  # VCX_OFFLOAD_ARCH: target of the in-tree HIP build
    colour_native: bool = True  # VCX_COLOUR_NATIVE: video BGR<->YUV in the C++ runtime (False: numpy)
    # VCX_REGISTER_SOURCE: a requester page-locks a memory-mapped source (hipHostRegister) and uploads
    # chunks straight from it (False: each chunk is copied into pinned memory first)
    register_source: bool = True
    sink_gpu: bool = True  # VCX_SINK_GPU: a GPU requester converts its Y4M output on the GPU (False: on the host)
    resnet_conv1x1: str = "gemm"  # VCX_RESNET_CONV1X1: ResNet 1x1 convolutions as GEMMs on the NHWC view ("gemm")
    # or through the convolution library ("conv")
    # VCX_CONV_FIND: library (MIOpen) convolutions of the ResNets pick the fastest solver per shape by
    # timing them on first use (torch.backends.cudnn.benchmark) instead of the immediate-mode heuristic:
    # ResNet-50 config 3 6886-7011 vs 6593 img/s (profiles/r4_resnet50_ab.txt); costs seconds once per shape
    conv_find: bool = True
    resnet_bn: str = "fused"  # VCX_RESNET_BN: ResNet train-mode BatchNorm (+ add) + ReLU as fused HIP passes ("fused")
    # or the torch composition ("torch")
    # VCX_BN_LAYER_WS: each BatchNorm module keeps its own [4C] workspace so the finalize of its
    # statistics runs inside the apply / dx passes (2 launches per layer and direction instead of 3)
    bn_layer_ws: bool = True
    # VCX_CONV3X3_WGRAD: weight gradients of the ResNet 3x3 convolutions with Cin, Cout % 128 == 0 on gemm_wg with
    # the patch matrix gathered while staging ("vcx"), or MIOpen's ("lib")
    conv3x3_wgrad: str = "vcx"
    # VCX_CONV3X3_FWD: forwards (and stride-1 input gradients) of the ResNet 3x3 convolutions on gemm_f's implicit
    # GEMM ("vcx": 1.09-1.38x MIOpen at every stage, profiles/r6_conv3x3_fwd.txt), or MIOpen's ("lib")
    conv3x3_fwd: str = "vcx"
    # VCX_ENGINE_BATCH: chunks a volunteer that already holds several runs through the detector as ONE batch
    # (1 = one chunk per network launch)
    engine_batch: int = 2
    resnet_join: bool = True  # VCX_RESNET_JOIN: identity-shortcut gradient added in conv1's dgrad GEMM (GradJoin)
    # VCX_RESNET_PROJ_JOIN: projection shortcuts add their input gradient into the one conv1 left (GradJoin)
    resnet_proj_join: bool = True
    # ---- distributed / control plane
    gloo_host: str = "127.0.0.1"  # VCX_GLOO_HOST: interface gloo peer groups bind to
    p2p_backend: str = ""  # VCX_P2P_BACKEND: pair-group backend of the p2p chunk plane ("" = auto)
    elastic_debug: bool = False  # VCX_ELASTIC_DEBUG: trace membership decisions to stderr
    elastic_liveness: bool = True  # VCX_ELASTIC_LIVENESS: TCP liveness links (process death seen at once)
    # VCX_ELASTIC_STAGE_JOINS: a joiner's generation is agreed one round early and its communicator
    # built during the local steps (the admission round pays no communicator init): "gloo" (default:
    # gloo groups only; the RCCL form broke the members at 8 ranks on one card, profiles/
    # r4_rccl8_rehearsal_1gpu.txt, and was removed in round 5), or "off"
    elastic_stage_joins: str = "gloo"
    # VCX_UPLINK_PIPELINE: the requester packs / resizes chunk k+1 while a wire thread ships chunk k:
    # "relay" (default: the relay plane only -- same-box A/B with the npy sink, relay 6463 vs 5506,
    # p2p 4650 vs 6101 frames/s: on the p2p plane the wire stage ships only metadata and the extra
    # thread's host copies just contend; profiles/r4_video_job_spans.txt), "all", or "off"
    uplink_pipeline: str = "relay"
    # VCX_SHARED_SOURCE_ROOT: on the p2p chunk plane, a requester whose source is a memory-mapped .npy file
    # under this directory sends each chunk as an index window (file, first frame, count) and every worker
    # reads its window from the file and uploads it over its OWN host link (8 GPUs: 8 links instead of the
    # requester's one); a worker reads only windows of .npy files under its own value. "" = off (the
    # requester uploads, resizes and sends the frames). node_job sets it to the source's directory.
    shared_source_root: str = ""
    store_port_train: int = 29611  # VCX_STORE_PORT (train CLI): rendezvous store port
    store_port_video: int = 29612  # VCX_STORE_PORT (video CLI): job-control store port
    # ---- observability
    trace_dir: str = ""  # VCX_TRACE_DIR: per-span device-time traces (utils/trace.py)
    metrics_dir: str = ""  # VCX_METRICS_DIR: JSON-lines metrics snapshots (utils/metrics.py)


# field -> (environment variable, parser)
_ENV = {
    "gemm": ("VCX_GEMM", str),
    "mlp": ("VCX_MLP", str),
    "dgrad_ps": ("VCX_DGRAD_PS", _bool),
    "mlp_grad_fwd": ("VCX_MLP_GRAD_FWD", _bool),
    "narrow_gemm": ("VCX_NARROW_GEMM", str),
    "resnet_conv1x1": ("VCX_RESNET_CONV1X1", str),
    "resnet_bn": ("VCX_RESNET_BN", str),
    "resnet_join": ("VCX_RESNET_JOIN", _bool),
    "engine_batch": ("VCX_ENGINE_BATCH", int),
    "conv3x3_wgrad": ("VCX_CONV3X3_WGRAD", str),
    "conv3x3_fwd": ("VCX_CONV3X3_FWD", str),
    "resnet_proj_join": ("VCX_RESNET_PROJ_JOIN", _bool),
    "bn_layer_ws": ("VCX_BN_LAYER_WS", _bool),
    "conv_find": ("VCX_CONV_FIND", _bool),
    "gemm_wgrad": ("VCX_GEMM_WGRAD", str),
    "gemm_fwd": ("VCX_GEMM_FWD", str),
    "wgrad_wide": ("VCX_WGRAD_WIDE", _bool),
    "wgrad_ragged": ("VCX_WGRAD_RAGGED", _bool),
    "gemm_select": ("VCX_GEMM_SELECT", _bool),
    "wgrad_big_split_min_m": ("VCX_WGRAD_BIG_SPLIT_MIN_M", int),
    "async_wgrad": ("VCX_ASYNC_WGRAD", _bool),
    "lmhead_chunk": ("VCX_LMHEAD_CHUNK", int),
    "force_reference_ops": ("VCX_FORCE_REFERENCE_OPS", _bool),
    "tunableop": ("VCX_TUNABLEOP", str),
    "tunableop_file": ("VCX_TUNABLEOP_FILE", str),
    "offload_arch": ("VCX_OFFLOAD_ARCH", str),
    "colour_native": ("VCX_COLOUR_NATIVE", _bool),
    "register_source": ("VCX_REGISTER_SOURCE", _bool),
    "sink_gpu": ("VCX_SINK_GPU", _bool),
    "gloo_host": ("VCX_GLOO_HOST", str),
    "p2p_backend": ("VCX_P2P_BACKEND", str),
    "elastic_debug": ("VCX_ELASTIC_DEBUG", _bool),
    "elastic_liveness": ("VCX_ELASTIC_LIVENESS", _bool),
    "elastic_stage_joins": ("VCX_ELASTIC_STAGE_JOINS", str),
    "uplink_pipeline": ("VCX_UPLINK_PIPELINE", str),
    "shared_source_root": ("VCX_SHARED_SOURCE_ROOT", str),
    "store_port_train": ("VCX_STORE_PORT", int),
    "store_port_video": ("VCX_STORE_PORT", int),
    "trace_dir": ("VCX_TRACE_DIR", str),
    "metrics_dir": ("VCX_METRICS_DIR", str),
}
_CHOICES = {"narrow_gemm": ("lib", "vision"), "conv3x3_wgrad": ("lib", "vcx"), "conv3x3_fwd": ("lib", "vcx"), "gemm": ("lib", "vcx"), "mlp": ("fused", "lib"), "gemm_wgrad": ("lib", "vcx"), "gemm_fwd": ("lib", "vcx"), "tunableop": ("on", "off"), "p2p_backend": ("", "gloo", "nccl"), "elastic_stage_joins": ("gloo", "off"),
            "uplink_pipeline": ("relay", "all", "off")}

_lock = threading.Lock()


def _validate(cfg: RuntimeConfig):
    for k, allowed in _CHOICES.items():
        if getattr(cfg, k) not in allowed:
            raise ValueError(f"config.{k} must be one of {allowed}, not {getattr(cfg, k)!r}")


def from_env(env=None) -> RuntimeConfig:
    """A config with the defaults overridden by the VCX_* variables present in `env`."""
    env = os.environ if env is None else env
    cfg = RuntimeConfig()
    for field, (var, parse) in _ENV.items():
        if var in env and env[var] != "":
            try:
                setattr(cfg, field, parse(env[var]))
            except ValueError as e:
                raise ValueError(f"{var}={env[var]!r}: {e}") from None
    _validate(cfg)
    return cfg


_CONFIG = from_env()


def get() -> RuntimeConfig:
    return _CONFIG


def update(**kw) -> RuntimeConfig:
    """Change fields of the live config (validated); returns it."""
    with _lock:
        unknown = set(kw) - {f.name for f in dataclasses.fields(RuntimeConfig)}
        if unknown:
            raise AttributeError(f"unknown config fields: {sorted(unknown)}")
        new = dataclasses.replace(_CONFIG, **kw)
        _validate(new)
        for k, v in kw.items():
            setattr(_CONFIG, k, v)
    return _CONFIG


@contextlib.contextmanager
def override(**kw):
    """Temporarily change fields; restored on exit (not thread-scoped: the config is global)."""
    old = {k: getattr(_CONFIG, k) for k in kw}
    update(**kw)
    try:
        yield _CONFIG
    finally:
        update(**old)


def describe() -> str:
    rows = []
    for f in dataclasses.fields(RuntimeConfig):
        var = _ENV.get(f.name, ("", None))[0]
        rows.append(f"{f.name:24s} {var:28s} {getattr(_CONFIG, f.name)!r}")
    return "\n".join(rows)
