"""Builds bookkeeper_amd/libbkdigest.so (gfx950) in-tree with hipcc.

The shared library is the product: HIP kernels + the C-ABI of include/bkdigest.h.
It is git-ignored but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import threading

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libbkdigest.so")
SOURCES = [os.path.join(CSRC, "bkdigest.hip")]
# CPU route and host worker pool (plain C++, built with the host compiler)
HOST_SOURCES = [os.path.join(CSRC, "host_crc.cpp"), os.path.join(CSRC, "host_batch.cpp")]
DEPS = SOURCES + HOST_SOURCES + [os.path.join(CSRC, f) for f in (
    "crc_kernels.hpp", "crc_tables.hpp", "plan_kernels.hpp", "host_crc.hpp", "host_batch.hpp")] + [os.path.join(ROOT, "include", "bkdigest.h")]
ARCH = os.environ.get("BKD_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build libbkdigest.so")


def cxx() -> str:
    for cand in (os.environ.get("CXX"), shutil.which("g++"), shutil.which("c++")):
        if cand and shutil.which(cand):
            return cand
    return hipcc()


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build_native(force: bool = False, extra_flags: list[str] | None = None, out: str | None = None) -> str:
    out = out or LIB
    if not force and out == LIB and not needs_build():
        return out
    objs = []
    for src in HOST_SOURCES:
        obj = os.path.join(CSRC, os.path.splitext(os.path.basename(src))[0] + f"_{os.getpid()}_{threading.get_ident()}.o")
        subprocess.run([cxx(), "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-pthread", "-c", src, "-o", obj],
                       check=True)
        objs.append(obj)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp"] + objs + SOURCES + ["-lpthread"] + list(
        extra_flags or [])
    try:
        subprocess.run(cmd, check=True)
    finally:
        for obj in objs:
            os.remove(obj)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_native(force=True))
