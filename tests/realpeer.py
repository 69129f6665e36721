"""A real Kaboodle instance on UDP sockets, for bridge tests: a compact Python restatement of one instance's
protocol loop (src/kaboodle.rs), speaking the reference's wire format through kaboodle_amd.wire.  Test
infrastructure only (the reference binary cannot be built here: no Rust toolchain).

The clock is explicit (`tick(now_ms)`, one call per protocol period, PROTOCOL_PERIOD = 1000 ms, :38) so a
test can interleave it with the bridge's rounds.  What it does per tick, in the reference's order
(KaboodleInner::tick, :746-786, and the receive handlers):
  * broadcasts (:256-331): Join{addr} -> insert Known(now), answer a new peer with KnownPeers of the whole map
    (maybe_send_known_peers_to_peer, :356-392, no truncation at these sizes); Failed(p) -> removed only if
    the datagram's source is a member (:268-283);
  * unicast (:394-548): the prologue inserts the sender as Known(now) with the envelope identity; Ack{p}
    forwards to the peers curious about p and syncs (maybe_sync_known_peers, :707-740); KnownPeers inserts the
    unknown ones as Known(now - MAX_PEER_SHARE_AGE); KnownPeersRequest answers with the Known peers heard
    within MAX_PEER_SHARE_AGE (not self, not the requester) and syncs; Ping -> Ack{self, fp, n};
    PingRequest(p) -> note the requester as curious, Ping p;
  * suspects (:557-640): WaitingForPing older than PING_TIMEOUT -> PingRequest(p) to up to NUM_INDIRECT other
    Known peers, WaitingForIndirectPing; WaitingForIndirectPing older than PING_TIMEOUT -> removed, Failed(p)
    broadcast;
  * ping (:655-703): Ping one of the five Known peers (not self) with the oldest instants, WaitingForPing;
  * Join re-broadcast while it knows only itself (maybe_broadcast_join, :228-251).
"""
from __future__ import annotations

import random
import socket
import zlib

from kaboodle_amd import wire

PING_TIMEOUT_MS = 2000               # src/kaboodle.rs:62
MAX_PEER_SHARE_AGE_MS = 10000        # :49
REBROADCAST_INTERVAL_MS = 10000      # :65
NUM_INDIRECT = 3                     # NUM_INDIRECT_PING_PEERS (:52)


class RealPeer:
    def __init__(self, identity: bytes, broadcast_to, ip: str = "127.0.0.1", seed: int = 1):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((ip, 0))
        self.sock.setblocking(False)
        self.bsock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)   # broadcast_out_sock: its own port
        self.bsock.bind((ip, 0))
        self.bin = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)     # what the mesh's broadcasts reach
        self.bin.bind((ip, 0))
        self.bin.setblocking(False)
        self.addr = self.sock.getsockname()
        self.identity, self.broadcast_to = identity, broadcast_to
        self.rng = random.Random(seed)
        self.now = 0
        # addr -> [identity, state, instant]; state: "known" | "wfp" (WaitingForPing) | "wfip"
        self.peers: dict[tuple, list] = {self.addr: [identity, "known", 0]}
        self.curious: dict[tuple, list] = {}
        self.last_join = None
        self.log: list[tuple] = []           # (now, direction, kind, peer address)

    # ---- helpers ----
    def fingerprint(self) -> int:
        """generate_fingerprint's shape (:71-83): a CRC-32 over the sorted address strings (the exact bytes do
        not matter here: the mesh's canonical addresses never match real ones, bridge.py)."""
        return zlib.crc32("".join(sorted(f"{a[0]}:{a[1]}" for a in self.peers)).encode())

    def send(self, to, kind: str, **kw) -> None:
        self.sock.sendto(wire.encode(kind, identity=self.identity, **kw), to)
        self.log.append((self.now, "out", kind, to))

    def broadcast(self, kind: str, **kw) -> None:
        self.bsock.sendto(wire.encode(kind, **kw), self.broadcast_to)

    def known_list(self, exclude=()):
        return [(a, v[0]) for a, v in self.peers.items() if a not in exclude]

    def insert(self, addr, identity: bytes, instant: int) -> bool:
        new = addr not in self.peers
        self.peers[addr] = [identity, "known", instant]
        return new

    def maybe_sync(self, peer, fp: int, n: int) -> None:
        if fp == self.fingerprint() or len(self.peers) > n:
            return
        self.send(peer, "KnownPeersRequest", fingerprint=self.fingerprint(), num_peers=len(self.peers))

    # ---- one protocol period ----
    def tick(self, now_ms: int) -> None:
        self.now = now_ms
        self._broadcasts()
        self._unicast()
        self._suspects()
        self._ping()
        if self.last_join is None or (len(self.peers) == 1 and now_ms - self.last_join >= REBROADCAST_INTERVAL_MS):
            self.last_join = now_ms
            self.broadcast("Join", identity=self.identity, peer=self.addr)

    def _broadcasts(self) -> None:
        while True:
            try:
                dg, src = self.bin.recvfrom(wire.INCOMING_BUFFER_SIZE)
            except BlockingIOError:
                return
            m = wire.receive(dg, "broadcast")
            if m["kind"] == "Join" and m["peer"] != self.addr:
                if self.insert(m["peer"], m["identity"], self.now):
                    self.send(m["peer"], "KnownPeers", peers=self.known_list())
            elif m["kind"] == "Failed" and m["peer"] != self.addr and src in self.peers:
                self.peers.pop(m["peer"], None)

    def _unicast(self) -> None:
        while True:
            try:
                dg, src = self.sock.recvfrom(wire.INCOMING_BUFFER_SIZE)
            except BlockingIOError:
                return
            env = wire.receive(dg, "unicast")
            self.log.append((self.now, "in", env["kind"], src))
            self.insert(src, env["identity"], self.now)                    # the prologue (:406-415)
            k = env["kind"]
            if k == "Ack":
                for obs in self.curious.pop(env["peer"], []):
                    self.send(obs, "Ack", peer=env["peer"], fingerprint=env["fingerprint"], num_peers=env["num_peers"])
                self.maybe_sync(env["peer"], env["fingerprint"], env["num_peers"])
            elif k == "KnownPeers":
                for a, ident in env["peers"]:
                    if a not in self.peers:
                        self.peers[a] = [ident, "known", self.now - MAX_PEER_SHARE_AGE_MS]
            elif k == "KnownPeersRequest":
                share = [(a, v[0]) for a, v in self.peers.items() if v[1] == "known" and a not in (self.addr, src)
                         and self.now - v[2] < MAX_PEER_SHARE_AGE_MS]
                self.send(src, "KnownPeers", peers=share)
                self.maybe_sync(src, env["fingerprint"], env["num_peers"])
            elif k == "Ping":
                self.send(src, "Ack", peer=self.addr, fingerprint=self.fingerprint(), num_peers=len(self.peers))
            elif k == "PingRequest":
                obs = self.curious.setdefault(env["peer"], [])
                if src not in obs:
                    obs.append(src)
                self.send(env["peer"], "Ping")

    def _suspects(self) -> None:
        for a, v in list(self.peers.items()):
            if v[1] == "wfp" and self.now - v[2] >= PING_TIMEOUT_MS:
                others = [b for b, w in self.peers.items() if w[1] == "known" and b not in (a, self.addr)]
                for b in self.rng.sample(others, min(NUM_INDIRECT, len(others))):
                    self.send(b, "PingRequest", peer=a)
                v[1], v[2] = "wfip", self.now
            elif v[1] == "wfip" and self.now - v[2] >= PING_TIMEOUT_MS:
                del self.peers[a]
                self.broadcast("Failed", peer=a)

    def _ping(self) -> None:
        cands = sorted((v[2], a) for a, v in self.peers.items() if v[1] == "known" and a != self.addr)[:5]
        if cands:
            _, a = self.rng.choice(cands)
            self.peers[a][1], self.peers[a][2] = "wfp", self.now
            self.send(a, "Ping")

    def close(self) -> None:
        for s in (self.sock, self.bsock, self.bin):
            s.close()
