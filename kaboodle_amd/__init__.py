"""kaboodle_amd — MI355X-native bulk-synchronous simulator of serval/kaboodle's SWIM round.

The product is the HIP library `libkaboodle_sim.so` (C ABI: include/kaboodle_sim.h).  This package is
its Python host mirror: `Mesh` owns one simulated mesh on one GPU, `Kaboodle` is a per-peer view with the
reference's method names (src/lib.rs:65-369).  There is no CPU fallback: without the built library or
a GPU every entry point raises.
"""
from __future__ import annotations

import collections
import os

from ._ffi import (KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_INIT_JOIN,  # noqa: F401
                   KbError, Sim, SimConfig, SimLib, STATE_NAMES)

LIB_PATH = os.environ.get("KB_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkaboodle_sim.so")
# (KB_LIB_PATH: an alternative build of the same library, for A/B timing experiments only)
_LIB = None


def lib() -> SimLib:
    """The loaded HIP library (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
        # torch's wheel carries its own HIP runtime.  Loaded first, it satisfies the library's libamdhip64
        # dependency; loaded after the library, it maps a second runtime next to /opt/rocm's, and the one that
        # initialises second finds no device (kb_sim_create: "no HIP device", tools/diag/hip_load_order.py).
        import torch  # noqa: F401
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
        self._subs: dict[int, dict[str, list[Channel]]] = {}

    def node(self, i: int) -> "Kaboodle":
        return Kaboodle(self, i)

    def subscribe(self, node: int, kind: str, ch: "Channel") -> "Channel":
        """Add a discover_* channel of `node` (kind: peers | departures | fingerprints).  The first one
        attaches the device observer and drains it, so channels see only later changes, as a channel
        created on a running Kaboodle does (src/lib.rs:186-263)."""
        if node not in self._subs:
            self.watch(node)
            self.events(node)
            self._subs[node] = {"peers": [], "departures": [], "fingerprints": []}
        self._subs[node][kind].append(ch)
        return ch

    def step(self, rounds: int = 1) -> None:
        """Advance `rounds` rounds, then fan one event batch per observed node out to its channels
        (handle_known_peers_events, src/events.rs:49-123)."""
        super().step(rounds)
        for node, subs in self._subs.items():
            if not any(subs.values()):
                continue
            disc, dep, fp, changed = self.events(node)
            for x in disc:
                for c in subs["peers"]:
                    c.send((self.format_addr(x), self.identity(x)))
            for x in dep:
                for c in subs["departures"]:
                    c.send(self.format_addr(x))
            if changed:
                for c in subs["fingerprints"]:
                    c.send(fp)
            for k in subs:                        # closed channels are dropped (events.rs:29-38)
                subs[k] = [c for c in subs[k] if not c.closed]


def discover_mesh_member(mesh: "Mesh", prober=("192.0.2.1", 40000), max_rounds: int = 64):
    """Kaboodle::discover_mesh_member (src/lib.rs, src/discovery.rs:30-89) against a simulated mesh: broadcast
    Probe(prober), wait for a ProbeResponse, re-broadcast with the reference's back-off (1 s, x1.25, at most
    10 s; one protocol period = one round = 1000 ms).  Steps the mesh.  Returns (responder address,
    identity) of the first response (canonical order), or None after max_rounds."""
    interval_ms, last_ms, now_ms, waited = 1000, None, 0, 0
    for _ in range(max_rounds):
        if last_ms is None or last_ms <= now_ms - interval_ms:
            mesh.probe(prober)
            last_ms, waited = now_ms, 0
        mesh.step(1)
        now_ms += 1000
        waited += 1000
        got = [r for r in mesh.probe_responses() if r[3] == tuple(prober)]
        if got:
            return mesh.format_addr(got[0][1]), got[0][4]
        if waited >= interval_ms:                  # timeout: longer wait, then probe again (discovery.rs:62-73)
            interval_ms = min(10000, int(interval_ms * 1.25))
            waited = 0
    return None


class Channel:
    """The receiving end of a discover_* channel (tokio UnboundedReceiver / oneshot Receiver in the
    reference, src/lib.rs:186-263), filled by Mesh.step."""

    def __init__(self, oneshot: bool = False):
        self._q: collections.deque = collections.deque()
        self.oneshot, self.closed = oneshot, False

    def send(self, item) -> None:
        if self.closed:
            return
        self._q.append(item)
        if self.oneshot:
            self.closed = True

    def try_recv(self):
        """The next item, or None when nothing is pending."""
        return self._q.popleft() if self._q else None

    def drain(self) -> list:
        out = list(self._q)
        self._q.clear()
        return out

    def close(self) -> None:
        self.closed = True


class Kaboodle:
    """Per-peer view mirroring the reference `Kaboodle` struct (src/lib.rs:65-369)."""

    def __init__(self, mesh: Mesh, node: int):
        self.mesh, self.id = mesh, node
        self._identity = None                     # set while stopped: announced from the next start

    def start(self) -> None:                      # src/lib.rs:136-156 (effective next round)
        """Start, or restart after stop: the reference binds a fresh ephemeral socket on every start
        (src/kaboodle.rs:138-152) and keeps its known_peers map, so a restarted peer has a new address
        (kb_sim_restart_node); its event channels follow it."""
        old = self.id
        self.id = self.mesh.restart_node(old)
        self._identity = None
        if self.id != old and old in self.mesh._subs:
            self.mesh._subs[self.id] = self.mesh._subs.pop(old)

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
        self._identity = bytes(identity)

    def fingerprint(self) -> int:                 # src/lib.rs:301-304
        return self.mesh.fingerprint(self.id)

    def peers(self) -> dict:                      # src/lib.rs:339-345: addr -> identity
        return {self.mesh.format_addr(p): self.mesh.identity(p) for p in self.mesh.peers(self.id)}

    def identity(self) -> bytes:                  # the identity this peer announces (Kaboodle.identity)
        return self._identity if self._identity is not None else self.mesh.identity(self.id)

    def discover_peers(self) -> Channel:          # src/lib.rs:221-236: (addr, identity) per new peer
        return self.mesh.subscribe(self.id, "peers", Channel())

    def discover_next_peer(self) -> Channel:      # src/lib.rs:238-263: the next one only
        return self.mesh.subscribe(self.id, "peers", Channel(oneshot=True))

    def discover_departures(self) -> Channel:     # src/lib.rs:185-199: addr per departed peer
        return self.mesh.subscribe(self.id, "departures", Channel())

    def discover_fingerprint_changes(self) -> Channel:   # src/lib.rs:201-219
        return self.mesh.subscribe(self.id, "fingerprints", Channel())

    def peer_states(self) -> dict:                # src/lib.rs:348-354: addr -> PeerInfo
        """PeerInfo per known peer (src/structs.rs:18-22): identity bytes, state name, round of its Instant
        (None = older than the stamp window), latency in simulated ms (None = never measured)."""
        out = {}
        for p, s, since, lat, ident in self.mesh.peer_states(self.id):
            out[self.mesh.format_addr(p)] = PeerInfo(ident, STATE_NAMES[s], None if since == -2**31 else since,
                                                     None if lat == 0xFFFFFFFF else lat)
        return out


class PeerInfo(collections.namedtuple("PeerInfo", "identity state since latency")):
    """PeerInfo {identity, state, latency} (src/structs.rs:18-22), the state's Instant as a round."""
