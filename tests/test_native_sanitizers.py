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


def test_drain_helper_protocol_under_asan(tmp_path, monkeypatch):
    """The drain helper (csrc/hsdrain_helper.cpp) built with ASan/UBSan,
    driven through its real Python client against a host-only stand-in for
    _hsgpu.so (tests/native/hsdrain_stub.cpp): drains, the mapping cache,
    unmaps, an out-of-range blob, a wrong magic and an oversized field."""
    import struct

    from hipsnapshot import _build
    from hipsnapshot.engine import drain_process
    from hipsnapshot.ops import native

    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    flags = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
             "-fno-omit-frame-pointer"]
    stub = str(tmp_path / "libstub.so")
    exe = str(tmp_path / "helper")
    for cmd in ([cxx] + flags + ["-shared", "-fPIC", "-o", stub,
                                 os.path.join(ROOT, "tests", "native", "hsdrain_stub.cpp")],
                [cxx] + flags + ["-o", exe, os.path.join(ROOT, "hipsnapshot", "csrc",
                                                         "hsdrain_helper.cpp"), "-ldl"]):
        proc = subprocess.run(cmd, capture_output=True, text=True)
        if proc.returncode != 0:
            pytest.skip(f"sanitizer toolchain unavailable: {proc.stderr[-300:]}")
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    monkeypatch.setenv("UBSAN_OPTIONS", "halt_on_error=1:print_stacktrace=1")
    monkeypatch.setattr(_build, "DRAIN_HELPER", exe)
    monkeypatch.setattr(_build, "HSGPU_SO", stub)
    monkeypatch.setattr(native, "hip_runtime_path", lambda: stub)

    pattern = bytes((i * 7 + 3) & 0xFF for i in range(1 << 20))
    handle = b"\xab" + bytes(63)
    h = drain_process.DrainHelper()
    try:
        blobs = [(0, 4096, str(tmp_path / "a")), (12345, 777, str(tmp_path / "b"))]
        for close_after in (False, True):  # second job hits the mapping cache, then unmaps
            rc, written, sums, stats, map_s, msg = h.drain(0, handle, blobs, 1 << 20, 2, 1, 0,
                                                           8, close_after)
            assert rc == 0 and written == 4096 + 777, msg
            assert sums == [sum(pattern[o:o + n]) for o, n, _ in blobs]
            assert len(stats) == len(native.NativeDrain.STATS)
            for o, n, p in blobs:
                assert open(p, "rb").read() == pattern[o:o + n]
        h.close_handle(handle)  # not mapped any more: a no-op
        rc, _w, _s, _st, _m, msg = h.drain(0, handle, [((1 << 20) - 10, 100, str(tmp_path / "c"))],
                                           1 << 20, 2, 1, 0, 8, True)
        assert rc == -14 and "failed" in msg
        h._send(struct.pack("=II", 0xDEADBEEF, 1))  # wrong magic: the helper exits
        assert h.proc.wait(timeout=30) == 3
    finally:
        h.shutdown()
    h = drain_process.DrainHelper()
    try:  # a 2 MiB handle field is refused: the helper stops reading and exits
        h._send(struct.pack("=IIiI", 0x48534448, 1, 0, 2 << 20))
        assert h.proc.wait(timeout=30) == 0
    finally:
        h.shutdown()
