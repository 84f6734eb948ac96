"""In-tree native build: HIP kernels for gfx950 + torch bindings + the C++ runtime.

Two shared objects are produced inside the package directory (so they travel with the repo
snapshot to a GPU box and are what the python process actually loads):

* ``_C.<abi>.so``      — every ``csrc/kernels/*.hip`` compiled by ``hipcc --offload-arch=gfx950``
                          plus the torch/pybind bindings (``csrc/bindings*.cpp``).
* ``_native.<abi>.so`` — the host runtime in ``csrc/runtime/*.cpp`` (framed TCP transport,
                          reorder buffer, chunk scheduler, video container writer). It links only
                          pybind11 + libstdc++ so it is usable on CPU-only volunteers.

Objects are cached under ``build/`` keyed by a content hash of the source and the headers it
may include, so a rebuild after editing one kernel recompiles one file.

Usage: ``python -m distributedvolunteercomputing_amd._build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

from . import _digest as _srcdigest
from . import config

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = config.get().offload_arch
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the gfx950 kernels)")


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths("cuda")]
    libdir = Path(torch.__file__).resolve().parent / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdir, abi


def _py_includes():
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _digest(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        h.update(str(p.name).encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _run(cmd, label):
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"[vcx build] {label} failed:\n{' '.join(cmd)}\n{proc.stdout}")
    return proc.stdout


def _compile_all(jobs, nproc):
    """jobs: list of (label, cmd, obj_path, stamp). Skips objects whose stamp matches."""
    todo = []
    for label, cmd, obj, stamp in jobs:
        st = obj.with_suffix(obj.suffix + ".stamp")
        if obj.exists() and st.exists() and st.read_text() == stamp:
            continue
        todo.append((label, cmd, obj, st, stamp))
    if not todo:
        return 0
    with cf.ThreadPoolExecutor(max_workers=max(1, nproc)) as ex:
        futs = {ex.submit(_run, cmd, label): (obj, st, stamp, label) for label, cmd, obj, st, stamp in todo}
        for f in cf.as_completed(futs):
            obj, st, stamp, label = futs[f]
            f.result()
            st.write_text(stamp)
            print(f"[vcx build] compiled {label}", flush=True)
    return len(todo)


def _digest_object(kind: str, symbol: str, compiler: list[str]) -> tuple[Path, str]:
    """Compile a one-function object returning the sources' digest (linked into the extension, read
    back by the loader, _digest.check)."""
    d = _srcdigest.source_digest(kind)
    src = BUILD / f"{kind}_digest.cpp"
    obj = BUILD / f"{kind}_digest.o"
    text = f'extern "C" const char* {symbol}() {{ return "{d}"; }}\n'
    if not (src.exists() and src.read_text() == text and obj.exists()):
        src.write_text(text)
        _run([*compiler, "-O2", "-fPIC", "-c", str(src), "-o", str(obj)], f"{kind} digest")
    return obj, d


def _needs_link(out: Path, n: int, d: str) -> bool:
    st = BUILD / (out.name + ".digest")
    return bool(n) or not out.exists() or not st.exists() or st.read_text() != d


def _linked(out: Path, d: str):
    (BUILD / (out.name + ".digest")).write_text(d)


# Per-file compiler flags. attention.hip: no SLP vectorisation. The SLP vectorizer packs adjacent scalar f32
# adds / multiplies of the softmax and dS = P (dP - delta) into v_pk_add_f32 / v_pk_mul_f32, which cost ~22-26
# cycles more than the scalar pair when issued between MFMAs (MI355X_MICROARCH.md, "price of one filler beside
# MFMAs"); without it the dK/dV tile body issues scalar ops only and the 3-wave forward stops spilling: forward
# 0.184-0.188 vs 0.192 ms, backward 0.557-0.559 vs 0.573-0.577, bench 1071-1073 vs 1060-1062 samples/s, outputs
# identical (profiles/r6_attention_noslp.txt). Measured and not applied: attention_hm.hip (Llama GQA backward
# 0.555 vs 0.541 ms), gemm_ps.hip + gemm.hip (bench 1086-1089 vs 1090-1091), vision.hip (detector chunk 1.179 vs
# 1.185 ms eager: even).
FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"]}


def build_C(nproc: int = 8, force: bool = False) -> Path:
    hipcc = _hipcc()
    inc, libdir, abi = _torch_flags()
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = list((CSRC / "kernels").glob("*.h"))
    kern_flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast-honor-pragmas",
                  "-munsafe-fp-atomics", f"-I{CSRC}", f"-I{CSRC / 'kernels'}"]
    bind_flags = ["-O2", "-fPIC", "-std=c++17", f"-I{CSRC}", "-D__HIP_PLATFORM_AMD__=1",
                  "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                  f"-D_GLIBCXX_USE_CXX11_ABI={abi}"] + inc + _py_includes()
    jobs, objs = [], []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        obj = BUILD / (src.stem + ".hip.o")
        flags = kern_flags + FILE_FLAGS.get(src.name, [])
        stamp = _digest([src] + headers, " ".join(flags))
        jobs.append((src.name, [hipcc, *flags, "-c", str(src), "-o", str(obj)], obj, stamp))
        objs.append(obj)
    for src in sorted(CSRC.glob("bindings*.cpp")):
        obj = BUILD / (src.stem + ".cpp.o")
        stamp = _digest([src] + headers, " ".join(bind_flags))
        jobs.append((src.name, [hipcc, *bind_flags, "-c", str(src), "-o", str(obj)], obj, stamp))
        objs.append(obj)
    if force:
        for _, _, obj, _ in jobs:
            obj.with_suffix(obj.suffix + ".stamp").unlink(missing_ok=True)
    n = _compile_all(jobs, nproc)
    dobj, dig = _digest_object("C", "vcx_source_digest", [hipcc])
    objs.append(dobj)
    out = PKG / f"_C{EXT}"
    if _needs_link(out, n, dig):
        # hipBLASLt: torch's own bundled copy (same library instance torch's GEMMs use)
        libs = ["-ltorch", "-ltorch_cpu", "-lc10", "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64",
                "-lhipblaslt"]
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out),
              f"-L{libdir}", *libs, f"-Wl,-rpath,{libdir}"], "link _C")
        _linked(out, dig)
        print(f"[vcx build] linked {out.name}", flush=True)
    return out


def build_native(nproc: int = 8, force: bool = False) -> Path:
    cxx = shutil.which("g++") or "g++"
    BUILD.mkdir(parents=True, exist_ok=True)
    rt = CSRC / "runtime"
    headers = list(rt.glob("*.h"))
    flags = ["-O3", "-fPIC", "-std=c++17", "-pthread", f"-I{rt}", *_py_includes()]
    jobs, objs = [], []
    for src in sorted(rt.glob("*.cpp")):
        obj = BUILD / ("rt_" + src.stem + ".o")
        stamp = _digest([src] + headers, " ".join(flags))
        jobs.append((src.name, [cxx, *flags, "-c", str(src), "-o", str(obj)], obj, stamp))
        objs.append(obj)
    if not objs:
        raise RuntimeError("no runtime sources found")
    if force:
        for _, _, obj, _ in jobs:
            obj.with_suffix(obj.suffix + ".stamp").unlink(missing_ok=True)
    n = _compile_all(jobs, nproc)
    dobj, dig = _digest_object("native", "vcx_native_source_digest", [cxx])
    objs.append(dobj)
    out = PKG / f"_native{EXT}"
    if _needs_link(out, n, dig):
        _run([cxx, "-shared", "-fPIC", "-pthread", *map(str, objs), "-o", str(out)], "link _native")
        _linked(out, dig)
        print(f"[vcx build] linked {out.name}", flush=True)
    return out


def build_all(nproc: int | None = None, force: bool = False):
    nproc = nproc or min(8, os.cpu_count() or 4)
    a = build_native(nproc, force)
    b = build_C(nproc, force)
    return a, b


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["C", "native"], default=None)
    a = ap.parse_args(argv)
    nproc = a.j or min(8, os.cpu_count() or 4)
    if a.only == "C":
        build_C(nproc, a.force)
    elif a.only == "native":
        build_native(nproc, a.force)
    else:
        build_all(nproc, a.force)


if __name__ == "__main__":
    sys.exit(main())
