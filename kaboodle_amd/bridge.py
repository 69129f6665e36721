"""A bridge between a simulated mesh and real Kaboodle instances on a network (SURVEY.md §8(f) items 3-4,
DESIGN.md §9).

Every simulated peer the real network talks to gets a real UDP socket of its own (`peer_socket`, bound on the
bridge's interface): its address on the wire, what real instances put in their maps, ping and send to.  A real
instance is an EXTERNAL peer of the mesh (kb_sim_set_external): an id no simulated instance binds, standing for
its real address.  `attach(addr, node)` pairs them; `auto_attach=[ids]` hands out ids from a pool to real
instances as they first show up (a Join broadcast or a datagram to a peer socket).

Each round (`Bridge.run_round`):
  1. broadcast socket, every waiting datagram read as the reference's broadcast receiver reads it (a zeroed
     10240-byte buffer, src/kaboodle.rs:256-262) and decoded as a SwimBroadcast:
       Probe(addr) -> queued into the mesh (kb_sim_probe): the running peers that should respond answer it
                      in the next round (maybe_respond_to_probe, :305-331);
       Join{addr}  -> from an attached (or newly auto-attached) real instance: injected as that external
                      peer's Join broadcast (kb_sim_inject, KB_WIRE_JOIN): every running simulated peer
                      inserts it and maybe answers with KnownPeers (:284-304), which leave in step 4;
                      from anyone else: counted, dropped;
       Failed(p)   -> counted, dropped: a receiver honours Failed only when the datagram's source address is
                      a member (:268-283), and a real instance broadcasts from its broadcast socket, never a
                      member address — the simulated receivers would ignore it too (KB_FAILED_SOCKET_FAITHFUL);
  2. peer sockets, every waiting datagram decoded as a SwimEnvelope (:394-403) and injected as a record from
     the sender's external id to that simulated peer, for wave 0 of the next round: Ping, PingRequest(p),
     Ack{p, fp, n}, KnownPeers{(addr, identity)}, KnownPeersRequest{fp, n}; addresses are mapped back to ids
     (a simulated peer's socket address, an attached real address); unknown addresses in a KnownPeers list
     are dropped (counted), as is a PingRequest / Ack about one; the envelope identity becomes the external
     peer's identity (the prologue's PeerInfo.identity, :406-415).  At most 33 records per external peer enter a
     round (kb_sim_inject's bound, the tick's emission capacity); the rest wait for the next round in arrival
     order, as late datagrams would (counted as "delayed");
  3. the mesh steps one round (one protocol period, 1000 ms; PING_TIMEOUT is 2000 ms, :62, so an Ack that
     comes back in the next round is in time);
  4. outbound: the records simulated peers addressed to external peers (kb_sim_exported) are encoded as
     SwimEnvelope{identity of the sender, msg} with every id mapped to its wire address and sent FROM the
     sender's peer socket (send_bytes on self.sock, :197-226), so the real instance sees the right source;
     the ProbeResponse{identity} of every responder goes to the prober from the responder's peer socket
     (:316-330); with forward_broadcasts, the mesh's Join{addr, identity} / Failed(addr) go to the broadcast
     address from the broadcast socket (broadcast_msg :188-195), addresses mapped the same way.

forward_broadcasts is off by default: without attached real instances, a real receiver of a simulated Join
would insert a peer socket it then pings through the bridge, which is sound but fills real views with the
whole simulated mesh.  Turn it on to let real instances hear the mesh's Joins.

Declared limits: fingerprints are computed over address strings (generate_fingerprint,
src/kaboodle.rs:71-83); the mesh uses its canonical 10.100.100.x addresses and real instances use the peer
sockets' addresses, so a mixed mesh never reports equal fingerprints across the boundary (membership still
flows, and the Ack/KnownPeersRequest exchanges a mismatch causes are carried like any other).  One socket per
simulated peer that reaches the network: the process file-descriptor limit bounds that number.  Addresses on
the wire are IPv4 (kb_wire_addr): an IPv6 interface is refused.
`mesh` is a kaboodle_amd.Mesh (or any object with step / probe / probe_responses / broadcasts / identity /
set_identity / set_external / inject / exported).
"""
from __future__ import annotations

import collections
import selectors
import socket

from . import wire
from .networking import Interface, best_available_interface, create_broadcast_sockets

DEFAULT_BROADCAST_PORT = 7475          # src/main.rs's default --broadcast-port
UNICAST_KINDS = ("Ping", "PingRequest", "Ack", "KnownPeers", "KnownPeersRequest")
MAX_RECORDS_PER_ROUND = 33             # kb_sim_inject: unicast records per external peer per round


class Bridge:
    def __init__(self, mesh, broadcast_port: int | None = None, interface: Interface | None = None,
                 sockets=None, forward_broadcasts: bool = False, auto_attach=(), max_peer_sockets: int = 16384):
        """sockets = (broadcast_in, broadcast_out, broadcast_addr, unicast) overrides the network setup
        (tests use loopback sockets; peer sockets then bind on the unicast socket's IP); otherwise the
        reference's sockets are created on `interface` (default: best_available_interface(), as Kaboodle::new
        does, src/lib.rs:98).  forward_broadcasts: also send the mesh's Join / Failed broadcasts.
        auto_attach: ids (never bound by a simulated instance) handed to real instances as they show up.
        max_peer_sockets: at most this many simulated peers get a socket (an address on the wire); beyond it, or
        when the OS refuses a socket, what needed one is dropped and counted instead of raising mid-round."""
        self.mesh = mesh
        self.max_peer_sockets = max_peer_sockets
        self.forward_broadcasts = forward_broadcasts
        if sockets is not None:
            self.bin, self.bout, self.baddr, self.usock = sockets
        else:
            if interface is None:
                interface = best_available_interface()
            if interface.is_ipv6:
                raise ValueError(f"interface {interface.name} is IPv6: the wire codec carries IPv4 socket addresses "
                                 f"only (kb_wire_addr); pass an IPv4 interface")
            if broadcast_port is None:
                broadcast_port = DEFAULT_BROADCAST_PORT
            self.bin, self.bout, self.baddr = create_broadcast_sockets(interface, broadcast_port)
            self.usock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)   # IPv4 only (refused above otherwise)
            self.usock.bind((interface.ip, 0))
        self.ip = self.usock.getsockname()[0]
        self.pool = list(auto_attach)
        self.ext_addr: dict[int, tuple] = {}       # external id -> real address
        self.ext_of: dict[tuple, int] = {}         # real address -> external id
        self.ext_ident: dict[int, bytes] = {}
        self.psock: dict[int, socket.socket] = {}  # simulated id -> its peer socket
        self.sim_of: dict[tuple, int] = {}         # peer socket address -> simulated id
        self.sel = selectors.DefaultSelector()
        self.pending: dict[int, collections.deque] = {}   # external id -> records waiting for injection
        self.stats = {"probes_in": 0, "external_join": 0, "external_failed": 0, "undecodable": 0,
                      "probe_responses_out": 0, "broadcasts_out": 0, "joins_in": 0, "unicast_in": 0,
                      "unicast_out": 0, "unknown_sender": 0, "unmapped_addr": 0, "inject_refused": 0,
                      "send_failed": 0, "delayed": 0, "no_socket": 0}

    # ---- addresses ----
    def attach(self, addr, node: int, identity: bytes | None = None) -> int:
        """Pair the real instance at `addr` with external id `node` (kb_sim_set_external)."""
        addr = (addr[0], int(addr[1]))
        if addr in self.ext_of:
            return self.ext_of[addr]
        self.mesh.set_external(node)
        self.ext_addr[node], self.ext_of[addr] = addr, node
        if identity is not None:
            self._set_identity(node, identity)
        return node

    def _set_identity(self, node: int, identity: bytes) -> None:
        if self.ext_ident.get(node) != identity:
            self.mesh.set_identity(node, identity)
            self.ext_ident[node] = identity

    def _external(self, addr, identity: bytes | None = None) -> int | None:
        """The external id of a real address: attached, or attached now from the pool."""
        addr = (addr[0], int(addr[1]))
        x = self.ext_of.get(addr)
        if x is None and self.pool:
            x = self.attach(addr, self.pool.pop(0))
        if x is not None and identity is not None:
            self._set_identity(x, identity)
        return x

    def peer_socket(self, node: int) -> socket.socket | None:
        """The real socket of simulated peer `node` (bound on first use; it is that peer's address for good, so
        sockets are never recycled).  None when no socket can be had: max_peer_sockets reached, or the OS refused
        one (EMFILE, ...) — the caller drops what needed it and counts it (stats["no_socket"])."""
        s = self.psock.get(node)
        if s is None:
            if len(self.psock) >= self.max_peer_sockets:
                self.stats["no_socket"] += 1
                return None
            try:
                s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            except OSError:
                self.stats["no_socket"] += 1
                return None
            try:
                s.bind((self.ip, 0))
                s.setblocking(False)
            except OSError:
                s.close()
                self.stats["no_socket"] += 1
                return None
            self.psock[node] = s
            self.sim_of[s.getsockname()] = node
            self.sel.register(s, selectors.EVENT_READ, node)
        return s

    def addr_for(self, node: int):
        """The wire address of id `node`: an external peer's real address, a simulated peer's socket (None: no
        socket could be bound for it)."""
        if node in self.ext_addr:
            return self.ext_addr[node]
        s = self.peer_socket(node)
        return s.getsockname() if s is not None else None

    def node_for(self, addr) -> int | None:
        """The id behind a wire address (None: an address the mesh has no id for)."""
        addr = (addr[0], int(addr[1]))
        if addr in self.ext_of:
            return self.ext_of[addr]
        return self.sim_of.get(addr)

    # ---- inbound ----
    def ingest(self, datagram: bytes, sender) -> str | None:
        """One datagram from the broadcast socket; returns the SwimBroadcast kind (None if undecodable)."""
        try:
            msg = wire.receive(datagram, "broadcast")
        except ValueError:
            self.stats["undecodable"] += 1
            return None
        if msg["kind"] == "Probe":
            self.mesh.probe(msg["peer"])
            self.stats["probes_in"] += 1
        elif msg["kind"] == "Join":
            x = None if msg["peer"] in self.sim_of else self._external(msg["peer"], msg["identity"])
            if x is None:
                self.stats["external_join"] += 1
            else:
                try:
                    self.mesh.inject(x, 0, wire.KINDS["Join"])
                    self.stats["joins_in"] += 1
                except Exception:                  # noqa: BLE001 — one Join per round: a repeat is dropped
                    self.stats["inject_refused"] += 1
        else:
            self.stats["external_failed"] += 1
        return msg["kind"]

    def ingest_unicast(self, datagram: bytes, src, node: int) -> str | None:
        """One datagram to simulated peer `node`'s socket from `src`; returns the SwimMessage kind queued for
        injection (pump injects the queue)."""
        try:
            env = wire.receive(datagram, "unicast")
        except ValueError:
            self.stats["undecodable"] += 1
            return None
        x = self._external(src, env["identity"])
        if x is None:
            self.stats["unknown_sender"] += 1
            return None
        kind = env["kind"]
        a, ids = 0, []
        if kind in ("PingRequest", "Ack"):
            a = self.node_for(env["peer"])
            if a is None:
                self.stats["unmapped_addr"] += 1
                return None
        elif kind == "KnownPeers":
            for addr, _ident in env["peers"]:
                j = self.node_for(addr)
                if j is None:
                    self.stats["unmapped_addr"] += 1
                else:
                    ids.append(j)
        q = self.pending.setdefault(x, collections.deque())
        q.append((node, wire.KINDS[kind], a, env.get("fingerprint", 0), env.get("num_peers", 0), ids))
        return kind

    def _flush(self) -> None:
        """Inject the queued records, at most MAX_RECORDS_PER_ROUND per external peer (the tick's emission
        bound, TICK_MAX); the rest wait for the next round, as a datagram that arrives late would."""
        for x, q in self.pending.items():
            k = 0
            while q and k < MAX_RECORDS_PER_ROUND:
                node, kind, a, fp, n, ids = q.popleft()
                k += 1
                try:
                    self.mesh.inject(x, node, kind, a=a, fp=fp, n=n, ids=ids)
                except Exception:                  # noqa: BLE001 — refused (a bad id): dropped
                    self.stats["inject_refused"] += 1
                    continue
                self.stats["unicast_in"] += 1
            self.stats["delayed"] += len(q)

    def pump(self) -> int:
        """Read every datagram waiting on the broadcast socket and on the peer sockets."""
        n = 0
        while True:
            try:
                data, sender = self.bin.recvfrom(wire.INCOMING_BUFFER_SIZE)
            except (BlockingIOError, InterruptedError):
                break
            self.ingest(data, sender)
            n += 1
        if self.psock:
            for key, _ in self.sel.select(timeout=0):
                while True:
                    try:
                        data, src = key.fileobj.recvfrom(wire.INCOMING_BUFFER_SIZE)
                    except (BlockingIOError, InterruptedError):
                        break
                    self.ingest_unicast(data, src, key.data)
                    n += 1
        self._flush()
        return n

    # ---- outbound ----
    def egress(self):
        """The round's datagrams: [(destination, datagram, sending socket, "probe_response" | "unicast" |
        "broadcast")]."""
        out = []
        for rnd, responder, probe, prober, ident in self.mesh.probe_responses():
            sock = self.peer_socket(responder)
            if sock is None:
                self.stats["send_failed"] += 1
                continue
            out.append((prober, wire.encode("ProbeResponse", identity=ident), sock, "probe_response"))
        if self.ext_addr:
            for (_r, _w, sender, dest, _seq, kind, a, fp, n, ids) in self.mesh.exported():
                name = UNICAST_KINDS[kind]
                sock = self.peer_socket(sender)
                kw = {}
                if name in ("PingRequest", "Ack"):
                    kw["peer"] = self.addr_for(a)
                if name in ("Ack", "KnownPeersRequest"):
                    kw["fingerprint"], kw["num_peers"] = fp, n
                if name == "KnownPeers":
                    peers = [(self.addr_for(j), j) for j in ids]
                    self.stats["unmapped_addr"] += sum(1 for ad, _ in peers if ad is None)
                    kw["peers"] = [(ad, self.mesh.identity(j)) for ad, j in peers if ad is not None]
                if sock is None or kw.get("peer", ()) is None:   # no socket to send from, or none for the named peer
                    self.stats["send_failed"] += 1
                    continue
                out.append((self.ext_addr[dest], wire.encode(name, identity=self.mesh.identity(sender), **kw), sock,
                            "unicast"))
        for kind, sender, peer in (self.mesh.broadcasts() if self.forward_broadcasts else ()):
            if kind == "Join":
                ad = self.addr_for(sender)
                if ad is None:
                    self.stats["send_failed"] += 1
                    continue
                out.append((self.baddr, wire.encode("Join", identity=self.mesh.identity(sender), peer=ad), self.bout,
                            "broadcast"))
            else:
                ad = self.addr_for(peer)
                if ad is None:
                    self.stats["send_failed"] += 1
                    continue
                out.append((self.baddr, wire.encode("Failed", peer=ad), self.bout, "broadcast"))
        return out

    def run_round(self) -> dict:
        """pump the inbound datagrams, step the mesh one round, send its outbound datagrams"""
        self.pump()
        self.mesh.step(1)
        for dest, dg, sock, what in self.egress():
            try:
                sock.sendto(dg, dest)
            except OSError:
                self.stats["send_failed"] += 1
                continue                       # the reference logs send failures and carries on (:324-329)
            self.stats[{"probe_response": "probe_responses_out", "unicast": "unicast_out",
                        "broadcast": "broadcasts_out"}[what]] += 1
        return dict(self.stats)

    def close(self) -> None:
        self.sel.close()
        for s in {self.bin, self.bout, self.usock, *self.psock.values()}:
            try:
                s.close()
            except OSError:
                pass
