"""Race detection for the host runtime.

The C++ scheduler, reorder index and framed TCP transport are compiled together with a stress
driver (tests/csrc/runtime_stress.cpp) under ThreadSanitizer and under AddressSanitizer +
UndefinedBehaviorSanitizer, and run: data races, use-after-free, leaks, overflows and UB all
fail the test. (GPU sanitizers are not available on this pool; the HIP kernels are covered by
host-side shape checks in the bindings and the numerics tests.)
"""
import os
import platform
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "distributedvolunteercomputing_amd", "csrc", "runtime")


def _compiler():
    # LLVM's sanitizer runtimes (ROCm's clang): GCC 11's libtsan does not intercept
    # pthread_cond_clockwait (std::condition_variable::wait_for) and reports false "double lock"s
    for c in ("/opt/rocm/lib/llvm/bin/clang++", shutil.which("clang++"), shutil.which("g++")):
        if c and os.path.exists(c):
            return c
    return None


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_runtime_under_sanitizer(tmp_path, san):
    gxx = _compiler()
    if gxx is None:
        pytest.skip("no C++ compiler")
    exe = str(tmp_path / "stress")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", f"-I{RT}", os.path.join(ROOT, "tests", "csrc", "runtime_stress.cpp"),
           os.path.join(RT, "scheduler.cpp"), os.path.join(RT, "transport.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ,
               TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1 verify_asan_link_order=0 exitcode=67",
               UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must be the first DSO of the child
    run = [exe]
    p = subprocess.run(run, capture_output=True, text=True, timeout=300, env=env)
    if p.returncode != 0 and "unexpected memory mapping" in p.stderr:
        # TSan cannot start under high-entropy ASLR: rerun with address randomisation off
        p = subprocess.run(["setarch", platform.machine(), "-R", exe], capture_output=True, text=True,
                           timeout=300, env=env)
    if p.returncode != 0 and ("unexpected memory mapping" in p.stderr or "ptrace" in p.stderr):
        pytest.skip(f"{san} sanitizer cannot run in this container: {p.stderr[-300:]}")
    assert p.returncode == 0, p.stderr[-6000:]
    assert "OK" in p.stdout
