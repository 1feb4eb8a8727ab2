"""In-tree build of hipsnapshot's native libraries.

* ``_hsio.so``  -- C++17 file-I/O engine (g++/clang++, no HIP), used on every box.
* ``_hsgpu.so`` -- HIP data plane for gfx950 (hipcc --offload-arch=gfx950).

Both are plain C ABIs loaded with ctypes, so they build in seconds without
torch headers and travel with the repository snapshot to the GPU box.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
HSIO_SO = os.path.join(PKG_DIR, "_hsio.so")
HSGPU_SO = os.path.join(PKG_DIR, "_hsgpu.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
# The kernels use gfx950-only builtins (MFMA 32x32x16 bf16, fp8 conversions):
# build for gfx950 whatever else PYTORCH_ROCM_ARCH lists (ROCm images often
# start that list with older targets).  ``python -m
# hipsnapshot._build --arch gfx950`` names the target explicitly.
SUPPORTED_ARCHS = ("gfx950",)


def gpu_archs(override: str = "") -> list:
    want = [a.strip() for a in (override or os.environ.get("PYTORCH_ROCM_ARCH", "")).replace(
        ",", ";").split(";") if a.strip()]
    # feature suffixes (gfx950:xnack-) keep their base name's support
    picked = [a for a in want if a.split(":")[0] in SUPPORTED_ARCHS]
    if override and not picked:
        raise ValueError(f"--arch {override!r}: the kernels build for {SUPPORTED_ARCHS} only")
    return picked or list(SUPPORTED_ARCHS)


GPU_ARCH = gpu_archs()[0]


def _stale(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    mtime = os.path.getmtime(out)
    return any(os.path.getmtime(s) > mtime for s in srcs)


def _run(cmd) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"native build failed: {' '.join(cmd)}\n{proc.stdout}")


def _atomic_build(out: str, cmd_for) -> None:
    tmp = f"{out}.{os.getpid()}.tmp"
    _run(cmd_for(tmp))
    os.replace(tmp, out)


def build_hsio(force: bool = False) -> str:
    srcs = [os.path.join(CSRC, "hsio.cpp"), os.path.join(CSRC, "hsz_cpu.cpp"),
            os.path.join(CSRC, "hschk.cpp")]
    if force or _stale(HSIO_SO, srcs):
        cxx = shutil.which("g++") or shutil.which("c++") or os.path.join(ROCM, "llvm/bin/clang++")
        _atomic_build(HSIO_SO, lambda out: [cxx, "-O3", "-std=c++17", "-fPIC", "-shared",
                                            "-pthread", "-Wall", "-o", out] + srcs)
    return HSIO_SO


def build_hsgpu(force: bool = False, arch: str = "") -> str:
    # hsdrain.cpp / hsrestore.cpp are host-only engines (their HIP calls sit
    # in hshost.hip); hipcc builds them as plain C++ into the same library
    srcs = [os.path.join(CSRC, "hsgpu.hip"), os.path.join(CSRC, "hsz.hip"),
            os.path.join(CSRC, "hsdma.hip"), os.path.join(CSRC, "hshost.hip"),
            os.path.join(CSRC, "hsdrain.cpp"), os.path.join(CSRC, "hsrestore.cpp")]
    if force or _stale(HSGPU_SO, srcs):
        hipcc = os.path.join(ROCM, "bin", "hipcc")
        if not os.path.exists(hipcc):
            hipcc = shutil.which("hipcc") or hipcc
        archs = [f"--offload-arch={a}" for a in gpu_archs(arch)]
        _atomic_build(HSGPU_SO, lambda out: [hipcc] + archs + ["-O3", "-std=c++17", "-fPIC",
                                                               "-shared", "-Wall", "-o", out]
                      + srcs + ["-ldl"])
    return HSGPU_SO


def build_all(force: bool = False, arch: str = "") -> None:
    build_hsio(force)
    build_hsgpu(force or bool(arch), arch)


if __name__ == "__main__":
    _arch = sys.argv[sys.argv.index("--arch") + 1] if "--arch" in sys.argv else ""
    build_all(force="--force" in sys.argv, arch=_arch)
    print(HSIO_SO)
    print(HSGPU_SO)
