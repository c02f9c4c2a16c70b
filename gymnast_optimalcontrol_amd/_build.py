"""Build the in-tree HIP library ``libgymnast_acrobot.so`` for gfx950 (MI355X).

    python -m gymnast_optimalcontrol_amd._build          # or __graft_entry__.build()

hipcc cross-compiles without a GPU.  The .so is git-ignored but travels to the GPU box with
the working tree.  Nothing here ever falls back to a CPU implementation.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB_NAME = "libgymnast_acrobot.so"
LIB_PATH = os.path.join(PKG, LIB_NAME)
SOURCES = [os.path.join(CSRC, "acrobot_kernels.hip"), os.path.join(CSRC, "tracking_kernels.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "acrobot_device.hpp"), os.path.join(INCLUDE, "gymnast_acrobot.h")]
ARCH = os.environ.get("GYM_OFFLOAD_ARCH", "gfx950")
BUILD_ID_TAG = b"gym-build-id:"      # marker in front of the id string inside the library's .rodata


def source_hash(defines=(), arch: str | None = None) -> str:
    """Build id: sha256 over the kernel sources and the ABI header (names and contents), the offload architecture
    and the sorted extra preprocessor defines, 16 hex digits.  The library embeds the id it was compiled from
    (gym_build_id); _lib.load refuses anything but the canonical id (no defines, GYM_OFFLOAD_ARCH), so neither a
    stale libgymnast_acrobot.so that travelled with the tree nor an A/B variant compiled with extra defines can run
    silently as the product."""
    h = hashlib.sha256()
    h.update(f"arch={arch or ARCH}\0defines={' '.join(sorted(defines))}\0".encode())
    for p in sorted(DEPS):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def embedded_build_id(path: str = LIB_PATH) -> str | None:
    """The build id compiled into the library file at ``path`` (read from the file, nothing is loaded)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_TAG)
    if i < 0:
        return None
    raw = data[i + len(BUILD_ID_TAG): i + len(BUILD_ID_TAG) + 16]
    return raw.decode("ascii", "replace")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP library)")


def needs_build() -> bool:
    """Rebuild unless the library's embedded build id is the tree's source hash (contents, not mtimes)."""
    return embedded_build_id(LIB_PATH) != source_hash()


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """Compile the library (``out`` and ``defines`` build A/B variants for measurement)."""
    target = out or LIB_PATH
    if out is None and not force and not needs_build():
        return LIB_PATH
    tmp = target + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           f"-DGYM_BUILD_ID=\"{source_hash(defines)}\"", *[f"-D{d}" for d in defines], "-I", INCLUDE, "-I", CSRC, *SOURCES, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
