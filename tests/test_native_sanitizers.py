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

pytestmark = pytest.mark.slow

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


# --- native restore / drain engines on CPU device stubs --------------------------

ENGINE_SRC = [os.path.join(ROOT, "tests", "native", "engine_stress.cpp"),
              os.path.join(ROOT, "tests", "native", "engine_stubs.cpp"),
              os.path.join(ROOT, "hipsnapshot", "csrc", "hsrestore.cpp"),
              os.path.join(ROOT, "hipsnapshot", "csrc", "hsdrain.cpp")]
SAN_ENV = dict(ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _build_engine_stress(tmp_path, san, sources=None):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    exe = str(tmp_path / f"engine_{san.replace(',', '_') or 'plain'}")
    flags = [f"-fsanitize={san}", "-fno-omit-frame-pointer"] if san else []
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-pthread", "-I",
           os.path.join(ROOT, "tests", "native")] + flags + ["-o", exe] + (sources or ENGINE_SRC)
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        if san:
            pytest.skip(f"sanitizer toolchain unavailable: {proc.stderr[-300:]}")
        raise AssertionError(proc.stderr[-3000:])
    return exe


@pytest.mark.parametrize("mode,rounds", [("restore", 24), ("drain", 24), ("ringwrap", 1),
                                         ("restore-trim", 16)])
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_native_engines_under_sanitizer(tmp_path, san, mode, rounds):
    """csrc/hsrestore.cpp and csrc/hsdrain.cpp (host code: readers,
    completion / retire threads, rings, slot fills, budget waits, drain
    writers and parked writers) driven by tests/native/engine_stress.cpp over
    CPU stand-ins of every device hook (random completion delays, injected
    upload / copy / file / memory failures, budgets below one blob, the
    c026ee7 ring wrap), concurrent restores on the shared pools while
    another thread frees every idle block (restore-trim)."""
    exe = _build_engine_stress(tmp_path, san)
    if san == "thread":
        rounds = max(1, rounds // 2)  # ~5x slower under TSan
    run = subprocess.run([exe, mode, str(tmp_path / "data"), str(rounds)], capture_output=True,
                         text=True, env=dict(os.environ, **SAN_ENV), timeout=600)
    assert run.returncode == 0, run.stdout[-500:] + run.stderr[-4000:]
    assert "ok" in run.stdout
    assert "runtime error" not in run.stderr, run.stderr[-3000:]


def test_ring_wrap_regression_hangs_without_the_fix(tmp_path):
    """The stress case for c026ee7 must catch the bug: with the fix taken out
    of the engine (an emptied ring restarting at offset 0), the blob longer
    than both free ends waits forever."""
    src = open(ENGINE_SRC[2]).read()
    fix = "    if (live.empty()) head = tail = (head + cap - 1) / cap * cap;\n"
    assert src.count(fix) == 1
    reverted = tmp_path / "hsrestore_reverted.cpp"
    reverted.write_text(src.replace(fix, ""))
    exe = _build_engine_stress(tmp_path, "", ENGINE_SRC[:2] + [str(reverted)] + ENGINE_SRC[3:])
    proc = subprocess.Popen([exe, "ringwrap", str(tmp_path / "rw")], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)
    try:
        out, err = proc.communicate(timeout=20)
    except subprocess.TimeoutExpired:
        proc.kill()
        proc.communicate()
        return  # hung, as the unfixed engine does
    raise AssertionError(f"the engine without the fix finished the ring-wrap case: "
                         f"rc {proc.returncode} {out[-200:]!r} {err[-500:]!r}")
