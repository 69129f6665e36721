"""The bridge between a simulated mesh and real instances (kaboodle_amd.bridge) and the networking.rs
plumbing (kaboodle_amd.networking), on loopback sockets: a real discover_mesh_member's Probe datagram
reaches the mesh, the ProbeResponse comes back to the prober's socket from the responder's own socket and
decodes as discovery.rs decodes it; the mesh's Join broadcasts go out only when forwarding is asked for, as
SwimBroadcast datagrams a real instance decodes, carrying the simulated peer's socket address; and a real
instance (tests/realpeer.py) joins the simulated mesh through the bridge and stays a member over 40 rounds of
unicast traffic both ways.  The CPU oracle stands in for the mesh here; the gpu-marked tests run the same
exchanges against the HIP library on an MI355X."""
import os
import socket
import time

import pytest

import parity
from kaboodle_amd._ffi import KB_INIT_CONVERGED, Sim, SimConfig

pytestmark = pytest.mark.skipif(not os.path.exists(parity.GPU_SO), reason="wire codec lives in the HIP library")


def _udp():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    s.settimeout(2.0)
    return s


def _exchange(mesh):
    """one Probe in, the ProbeResponses out; Joins forwarded only by the opted-in bridge"""
    from kaboodle_amd import wire
    from kaboodle_amd.bridge import Bridge
    bin_ = _udp()
    bin_.setblocking(False)
    listener = _udp()                      # stands in for the broadcast address: what real instances receive
    listener.settimeout(0.3)
    uni = _udp()
    prober = _udp()                        # a real discover_mesh_member's socket
    for i in range(2):
        mesh.start_node(i)
    br = Bridge(mesh, sockets=(bin_, bin_, listener.getsockname(), uni))
    br.run_round()                         # round 0: the two Joins stay inside the mesh
    with pytest.raises(socket.timeout):
        listener.recvfrom(wire.INCOMING_BUFFER_SIZE)
    assert br.stats["broadcasts_out"] == 0
    # discover_mesh_member: Probe(self_addr) to the broadcast port
    paddr = prober.getsockname()
    prober.sendto(wire.encode("Probe", peer=paddr), bin_.getsockname())
    time.sleep(0.05)
    br.run_round()                         # ingested, delivered with round 1's broadcasts
    assert br.stats["probes_in"] == 1
    dg, src = prober.recvfrom(1024)
    env = wire.receive(dg, "discovery")    # discovery.rs:81 reads it as a SwimEnvelope
    assert src in (br.addr_for(0), br.addr_for(1))   # from the responder's own socket (src/kaboodle.rs:316-330)
    assert env["identity"] == mesh.identity(br.node_for(src))
    assert br.stats["probe_responses_out"] == 2  # n = 2: both answer (o = 0)
    # a real instance's Join with no external id to give it (no attach, no auto_attach pool): counted, dropped
    prober.sendto(wire.encode("Join", identity=b"real", peer=paddr), bin_.getsockname())
    time.sleep(0.05)
    br.run_round()
    assert br.stats["external_join"] == 1
    # forwarding on: the next Join broadcasts go out as SwimBroadcast::Join datagrams
    mesh.start_node(2)
    br.forward_broadcasts = True
    br.run_round()                         # round 3: node 2's Join
    dg, _src = listener.recvfrom(wire.INCOMING_BUFFER_SIZE)
    g = wire.receive(dg, "broadcast")
    assert (g["kind"], br.node_for(g["peer"]), g["identity"]) == ("Join", 2, mesh.identity(2))
    br.close()
    for s in (listener, prober):
        s.close()


def test_probe_over_udp_and_join_broadcasts():
    with Sim(parity.oracle_lib(), SimConfig(capacity=8, initial_nodes=0, id_len=5, seed=3)) as o:
        _exchange(o)


@pytest.mark.gpu
def test_bridge_hip_mesh():
    """The same exchange against the HIP library's mesh (kaboodle_amd.Mesh) on an MI355X."""
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    with kaboodle_amd.Mesh(SimConfig(capacity=8, initial_nodes=0, id_len=5, seed=3)) as m:
        _exchange(m)


def _real_instance_joins(mesh, rounds: int = 40):
    """A real instance (tests/realpeer.py, the reference's protocol loop on UDP sockets) joins a simulated mesh through
    the bridge and stays a member: its Join broadcast reaches every simulated peer (kb_sim_inject KB_WIRE_JOIN), the
    Join responses come back as KnownPeers from the responders' own sockets, its pings are acked by simulated peers
    and the simulated peers' pings to it are exported, sent, acked and injected back, for `rounds` rounds."""
    from kaboodle_amd import wire
    from kaboodle_amd.bridge import Bridge
    from realpeer import RealPeer
    n_sim = 24
    bin_ = _udp()
    bin_.setblocking(False)
    uni = _udp()
    real = RealPeer(b"real-0", bin_.getsockname(), seed=7)
    br = Bridge(mesh, sockets=(bin_, bin_, real.bin.getsockname(), uni), auto_attach=[30, 31], forward_broadcasts=True)
    mesh.step(1)                                   # the converged mesh's first round, before the instance starts
    t = 1000
    real.tick(t)                                   # Kaboodle::start: the Join broadcast (:228-251)
    st = br.run_round()
    assert st["joins_in"] == 1 and br.ext_of == {real.addr: 30} and mesh.identity(30) == b"real-0"
    assert all(30 in mesh.peers(i) for i in range(n_sim)), "the Join reached every simulated peer"
    for _ in range(rounds):
        t += 1000
        real.tick(t)
        time.sleep(0.002)
        br.run_round()
    sims = {br.addr_for(i) for i in range(n_sim)}
    known = set(real.peers) - {real.addr}
    assert len(known & sims) >= n_sim // 2, f"the real instance learnt {len(known & sims)} simulated peers"
    assert not known - sims, "every address it knows is a simulated peer's socket"
    assert all(30 in mesh.peers(i) for i in range(n_sim)), "the real instance stayed a member of every view"
    acked = {src for (_t, d, k, src) in real.log if d == "in" and k == "Ack"}
    pinged = {dst for (_t, d, k, dst) in real.log if d == "out" and k == "Ping"}
    assert pinged and pinged <= acked | {dst for (tt, d, k, dst) in real.log if d == "out" and tt >= t - 2000}
    assert any(k == "Ping" for (_t, d, k, _s) in real.log if d == "in"), "simulated peers pinged it"
    assert br.stats["unicast_in"] > rounds and br.stats["unicast_out"] > rounds and br.stats["unknown_sender"] == 0
    assert br.stats["unmapped_addr"] == 0 and br.stats["inject_refused"] == 0 and br.stats["undecodable"] == 0
    assert mesh.stats()["exported"] == br.stats["unicast_out"]
    real.close()
    br.close()
    return wire


def test_real_instance_joins_through_bridge():
    cfg = SimConfig(capacity=32, initial_nodes=24, init_mode=KB_INIT_CONVERGED, id_len=5, seed=11)
    with Sim(parity.oracle_lib(), cfg) as o:
        _real_instance_joins(o)


@pytest.mark.gpu
def test_real_instance_joins_hip_mesh():
    """The same join through the bridge against the HIP library's mesh on an MI355X."""
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    cfg = SimConfig(capacity=32, initial_nodes=24, init_mode=KB_INIT_CONVERGED, id_len=5, seed=11)
    with kaboodle_amd.Mesh(cfg) as m:
        _real_instance_joins(m)


def test_bridge_default_interface_and_ipv6(monkeypatch):
    """Bridge(mesh) with no interface takes best_available_interface() (Kaboodle::new, src/lib.rs:98);
    an IPv6 interface is refused with a clear error (the codec carries IPv4 addresses)."""
    from kaboodle_amd import bridge, networking
    monkeypatch.setattr(bridge, "best_available_interface", lambda: networking.Interface("lo", "127.0.0.1", None))
    br = bridge.Bridge(object(), broadcast_port=0)
    assert br.usock.getsockname()[0] == "127.0.0.1" and not br.forward_broadcasts
    br.close()
    monkeypatch.setattr(bridge, "best_available_interface", lambda: networking.Interface("v6", "fe80::1", 2))
    with pytest.raises(ValueError, match="IPv6"):
        bridge.Bridge(object(), broadcast_port=0)


def test_networking_plumbing():
    from kaboodle_amd import networking
    lo = networking.Interface("lo", "127.0.0.1", None)
    sin, sout, baddr = networking.create_broadcast_sockets(lo, 0)
    try:
        assert baddr[0] == "255.255.255.255"
        assert sin.getsockopt(socket.SOL_SOCKET, socket.SO_BROADCAST) == 1
        assert sin.getsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR) == 1
        assert sin.getsockname()[0] == "0.0.0.0"
    finally:
        sin.close()
        sout.close()
    with pytest.raises(networking.UnableToFindInterfaceNumber):
        networking.create_broadcast_sockets(networking.Interface("x", "fe80::1", None), 0)
    ifs = networking.non_loopback_interfaces()
    assert all(not i.is_loopback() for i in ifs)
    if ifs:
        best = networking.best_available_interface()
        assert best in ifs and (best.is_ipv6 or not any(i.is_ipv6 for i in ifs))


def test_bridge_survives_socket_exhaustion():
    """a simulated peer that cannot get a socket (max_peer_sockets, or EMFILE from the OS) costs the
    datagrams that needed it (counted), never an exception after the round's exports were drained."""
    from kaboodle_amd.bridge import Bridge
    with Sim(parity.oracle_lib(), SimConfig(capacity=8, initial_nodes=0, id_len=5, seed=3)) as mesh:
        bin_ = _udp()
        bin_.setblocking(False)
        uni = _udp()
        for i in range(2):
            mesh.start_node(i)
        br = Bridge(mesh, sockets=(bin_, bin_, bin_.getsockname(), uni), max_peer_sockets=0)
        assert br.peer_socket(3) is None and br.addr_for(3) is None and br.stats["no_socket"] == 2
        br.run_round()
        mesh.probe(("127.0.0.1", 9))
        br.run_round()                     # both peers answer the Probe: no socket to answer from
        assert br.stats["send_failed"] == 2 and br.stats["probe_responses_out"] == 0
        br.close()
