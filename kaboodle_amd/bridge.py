"""A bridge between a simulated mesh and real Kaboodle instances on a network.

Each round (`Bridge.run_round`):
  1. every datagram waiting on the broadcast socket is read as the reference's broadcast receiver reads it
     (a zeroed 10240-byte buffer, src/kaboodle.rs:256-262) and decoded as a SwimBroadcast:
       Probe(addr)  -> queued into the mesh (kb_sim_probe): the running peers that should respond answer
                       it in the next round (maybe_respond_to_probe, src/kaboodle.rs:305-331);
       Join/Failed  -> counted and dropped: a real instance's unicast address is not a peer of the
                       simulated mesh (its ids are the canonical 10.100.100.x addresses), so it cannot be
                       inserted into simulated views or answered over the mesh;
  2. the mesh steps one round (one protocol period);
  3. the round's outbound traffic is encoded with the wire codec and sent: the ProbeResponse{identity} of
     every responder, to the prober, from the unicast socket (src/kaboodle.rs:316-330: send_bytes on
     self.sock).
A real `Kaboodle::discover_mesh_member` on the same network therefore discovers a simulated peer.

Not carried (declared): unicast envelopes between real and simulated peers.  For that reason
the mesh's own Join / Failed broadcasts are NOT sent by default (`forward_broadcasts=False`):
  - a real instance that receives a simulated Join inserts the canonical 10.100.100.x address as a peer
    and may answer it with KnownPeers (src/kaboodle.rs:284-304), later pings it (:655-703), gets no Ack
    (the bridge carries no unicast), suspects it and broadcasts Failed: a large simulated mesh would fill
    every real view with unreachable members;
  - a simulated Failed has no effect on a real receiver at all: Failed is honoured only if the datagram's
    source address is a member (:268-283), and the source here is the bridge's broadcast socket.
`forward_broadcasts=True` sends them anyway (SwimBroadcast::Join / Failed of the round's lists, to the
broadcast address from the broadcast socket, broadcast_msg :188-195), e.g. for a capture or a test.

Addresses on the wire are IPv4 (kb_wire_addr): an IPv6 interface is refused.
`mesh` is a kaboodle_amd.Mesh (or any object with step / probe / probe_responses / broadcasts / identity).
"""
from __future__ import annotations

import socket

from . import wire
from .networking import Interface, best_available_interface, create_broadcast_sockets

DEFAULT_BROADCAST_PORT = 7475          # src/main.rs's default --broadcast-port


class Bridge:
    def __init__(self, mesh, broadcast_port: int | None = None, interface: Interface | None = None,
                 sockets=None, forward_broadcasts: bool = False):
        """sockets = (broadcast_in, broadcast_out, broadcast_addr, unicast) overrides the network setup
        (tests use loopback sockets); otherwise the reference's sockets are created on `interface`
        (default: best_available_interface(), as Kaboodle::new does, src/lib.rs:98).  forward_broadcasts:
        also send the mesh's Join / Failed broadcasts (off by default: see the module docstring)."""
        self.mesh = mesh
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
        self.stats = {"probes_in": 0, "external_join": 0, "external_failed": 0, "undecodable": 0,
                      "probe_responses_out": 0, "broadcasts_out": 0}

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
            self.stats["external_join"] += 1
        else:
            self.stats["external_failed"] += 1
        return msg["kind"]

    def pump(self) -> int:
        """Read every datagram waiting on the broadcast socket."""
        n = 0
        while True:
            try:
                data, sender = self.bin.recvfrom(wire.INCOMING_BUFFER_SIZE)
            except (BlockingIOError, InterruptedError):
                return n
            self.ingest(data, sender)
            n += 1

    # ---- outbound ----
    def egress(self):
        """The round's datagrams: [(destination, datagram, "unicast" | "broadcast")]."""
        out = []
        for rnd, responder, probe, prober, ident in self.mesh.probe_responses():
            out.append((prober, wire.encode("ProbeResponse", identity=ident), "unicast"))
        for kind, sender, peer in (self.mesh.broadcasts() if self.forward_broadcasts else ()):
            if kind == "Join":
                out.append((self.baddr, wire.encode("Join", identity=self.mesh.identity(sender),
                                                    peer=wire.addr_of(sender)), "broadcast"))
            else:
                out.append((self.baddr, wire.encode("Failed", peer=wire.addr_of(peer)), "broadcast"))
        return out

    def run_round(self) -> dict:
        """pump the inbound broadcasts, step the mesh one round, send its outbound datagrams"""
        self.pump()
        self.mesh.step(1)
        for dest, dg, ch in self.egress():
            try:
                (self.usock if ch == "unicast" else self.bout).sendto(dg, dest)
            except OSError:
                continue                       # the reference logs send failures and carries on (:324-329)
            self.stats["probe_responses_out" if ch == "unicast" else "broadcasts_out"] += 1
        return dict(self.stats)

    def close(self) -> None:
        for s in {self.bin, self.bout, self.usock}:
            try:
                s.close()
            except OSError:
                pass
