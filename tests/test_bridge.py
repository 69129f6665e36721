"""The bridge between a simulated mesh and real instances (kaboodle_amd.bridge) and the networking.rs
plumbing (kaboodle_amd.networking), on loopback sockets: a real discover_mesh_member's Probe datagram
reaches the mesh, the ProbeResponse comes back to the prober's socket and decodes as discovery.rs decodes
it; the mesh's Join broadcasts go out only when forwarding is asked for (by default they would fill real
views with unreachable members, kaboodle_amd/bridge.py), as SwimBroadcast datagrams a real instance
decodes.  The CPU oracle stands in for the mesh here; test_bridge_hip_mesh runs the same exchange against
the HIP library on an MI355X."""
import os
import socket
import time

import pytest

import parity
from kaboodle_amd._ffi import Sim, SimConfig

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
    assert src == uni.getsockname() and env["identity"] in (mesh.identity(0), mesh.identity(1))
    assert br.stats["probe_responses_out"] == 2  # n = 2: both answer (o = 0)
    # a real instance's Join is not a simulated peer: counted, dropped
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
    assert (g["kind"], wire.id_of(g["peer"]), g["identity"]) == ("Join", 2, mesh.identity(2))
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
