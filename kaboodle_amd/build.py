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


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [SRC] + [os.path.join(HERE, "csrc", f) for f in ("kb_device.h", "kb_common.h", "kb_round.h", "kb_tick.h", "kb_waves.h", "kb_xfer.h", "kb_wire.h", "kb_sparse.h", "kb_sparse_host.h")] + [
            os.path.join(os.path.dirname(HERE), "include", "kaboodle_sim.h")]
    return any(os.path.getmtime(p) > t for p in deps)


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
