"""kaboodle_amd — MI355X-native bulk-synchronous simulator of serval/kaboodle's SWIM round.

The product is the HIP library `libkaboodle_sim.so` (C ABI: include/kaboodle_sim.h).  This package is
its Python host mirror: `Mesh` owns one simulated mesh on one GPU, `Kaboodle` is a per-peer view with the
reference's method names (src/lib.rs:65-369).  There is no CPU fallback: without the built library or
a GPU every entry point raises.
"""
from __future__ import annotations

import os

from ._ffi import (KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_INIT_JOIN,  # noqa: F401
                   KbError, Sim, SimConfig, SimLib, STATE_NAMES)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkaboodle_sim.so")
_LIB = None


def lib() -> SimLib:
    """The loaded HIP library (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
        _LIB = SimLib(LIB_PATH, "kb_")
    return _LIB


def require_gpu() -> None:
    """Fail loudly when there is no GPU (the product has no CPU path)."""
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("kaboodle_amd needs an MI355X (HIP device); none is visible")
    lib()


def rccl_unique_id() -> bytes:
    """RCCL unique id for kb_sim_create_rank (made on rank 0, broadcast by the host)."""
    from ._ffi import rccl_unique_id as _uid
    return _uid(lib())


class Mesh(Sim):
    """One simulated mesh on the GPU, or one row shard of it.

    Mesh(cfg)                              the whole mesh on this process's GPU
    Mesh(cfg, shards=k)                    k row shards inside this process (one GPU; exchange by copies)
    Mesh(cfg, rank=r, world=w, uid=u)      this process's shard of a mesh over w GPUs (RCCL exchange)
    """

    def __init__(self, cfg: SimConfig | None = None, shards: int = 0, rank: int | None = None,
                 world: int | None = None, uid: bytes | None = None, **kw):
        super().__init__(lib(), cfg or SimConfig(**kw), shards=shards, rank=rank, world=world, uid=uid)

    def node(self, i: int) -> "Kaboodle":
        return Kaboodle(self, i)


class Kaboodle:
    """Per-peer view mirroring the reference `Kaboodle` struct (src/lib.rs:65-369)."""

    def __init__(self, mesh: Mesh, node: int):
        self.mesh, self.id = mesh, node

    def start(self) -> None:                      # src/lib.rs:136-156 (effective next round)
        self.mesh.start_node(self.id)

    def stop(self) -> None:                       # src/lib.rs:159-183
        self.mesh.stop_node(self.id)

    def is_running(self) -> bool:                 # src/lib.rs:307-309
        return self.mesh.is_running(self.id)

    def self_addr(self):                          # src/lib.rs:312-314
        return self.mesh.format_addr(self.id) if self.is_running() else None

    def ping_addrs(self, peers) -> None:          # src/lib.rs:268-297
        self.mesh.ping_addrs(self.id, list(peers))

    def set_identity(self, identity: bytes) -> None:   # src/lib.rs:323-336
        self.mesh.set_identity(self.id, identity)

    def fingerprint(self) -> int:                 # src/lib.rs:301-304
        return self.mesh.fingerprint(self.id)

    def peers(self) -> dict:                      # src/lib.rs:339-345: addr -> identity
        return {self.mesh.format_addr(p): p for p in self.mesh.peers(self.id)}

    def peer_states(self) -> dict:                # src/lib.rs:348-354
        return {self.mesh.format_addr(p): (STATE_NAMES[s], since) for p, s, since in self.mesh.peer_states(self.id)}
