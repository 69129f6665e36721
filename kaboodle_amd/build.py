"""In-tree build of the HIP library (gfx950): kaboodle_amd/libkaboodle_sim.so.

    python -m kaboodle_amd.build        # or __graft_entry__.build()
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "kb_sim.hip")
OUT = os.path.join(HERE, "libkaboodle_sim.so")
ARCH = os.environ.get("KB_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result", "-Wno-unused-value", "-lrccl", "-pthread"]


def deps() -> list[str]:
    """Every input of the library build (the translation unit and what it includes from this repository)."""
    return [SRC] + [os.path.join(HERE, "csrc", f) for f in ("kb_device.h", "kb_common.h", "kb_round.h", "kb_tick.h", "kb_waves.h", "kb_xfer.h", "kb_wire.h", "kb_sparse.h", "kb_sparse_host.h")] + [
        os.path.join(os.path.dirname(HERE), "include", "kaboodle_sim.h")]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in deps())


def src_sha16() -> str:
    """Identity of the library's sources and build command (hipcc's output is not byte-reproducible: two builds of
    the same sources differ, so measurement records carry this beside the binary's SHA, and bench.py accepts either)."""
    import hashlib
    h = hashlib.sha256()
    h.update(" ".join([ARCH, *FLAGS]).encode())
    for p in deps():
        h.update(os.path.relpath(p, os.path.dirname(HERE)).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def build(force: bool = False) -> str:
    if force or needs_build():
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        extra = os.environ.get("KB_EXTRA_FLAGS", "").split()   # e.g. -DKB_RP_PROF (dev profiling builds)
        cmd = [hipcc, f"--offload-arch={ARCH}", *FLAGS, *extra, "-o", OUT + ".tmp", SRC]
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
