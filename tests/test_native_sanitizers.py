"""Native I/O engine under AddressSanitizer/UBSan and ThreadSanitizer (host code only).

SURVEY 5.2: the reference has no race detection; here the C++ engine's
worker pool, completion queue and eventfd protocol are exercised by a
multi-threaded stress driver built with -fsanitize=address,undefined and,
separately, -fsanitize=thread.
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "hipsnapshot", "csrc", "hsio.cpp"),
       os.path.join(ROOT, "hipsnapshot", "csrc", "hsz_cpu.cpp"),
       os.path.join(ROOT, "tests", "native", "hsio_stress.cpp")]


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_hsio_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    exe = str(tmp_path / "stress")
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           "-pthread", "-o", exe] + SRC
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        pytest.skip(f"sanitizer toolchain unavailable: {proc.stderr[-300:]}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    run = subprocess.run([exe, str(tmp_path / "data")], capture_output=True, text=True, env=env,
                         timeout=300)
    assert run.returncode == 0, run.stderr[-3000:]
    assert "ok" in run.stdout


def test_hsz_decoder_fuzz_under_asan(tmp_path):
    """The CPU HSZ1 decoder reads 8 bytes at a time and past lane boundaries;
    corrupted frames must never make it read outside the frame."""
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    exe = str(tmp_path / "fuzz")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-pthread", "-o", exe,
           os.path.join(ROOT, "tests", "native", "hsz_fuzz.cpp")]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        pytest.skip(f"sanitizer toolchain unavailable: {proc.stderr[-300:]}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert run.returncode == 0, run.stdout[-500:] + run.stderr[-3000:]
    assert "ok" in run.stdout
