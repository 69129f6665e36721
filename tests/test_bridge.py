"""The bridge between a simulated mesh and real instances (kaboodle_amd.bridge) and the networking.rs
plumbing (kaboodle_amd.networking), on loopback sockets with the CPU oracle standing in for the mesh: a
real discover_mesh_member's Probe datagram reaches the mesh, the ProbeResponse comes back to the prober's
socket and decodes as discovery.rs decodes it, and the mesh's Join broadcasts go out as SwimBroadcast
datagrams a real instance decodes."""
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


def test_probe_over_udp_and_join_broadcasts():
    from kaboodle_amd import wire
    from kaboodle_amd.bridge import Bridge
    bin_ = _udp()
    bin_.setblocking(False)
    listener = _udp()                      # stands in for the broadcast address: what real instances receive
    uni = _udp()
    prober = _udp()                        # a real discover_mesh_member's socket
    with Sim(parity.oracle_lib(), SimConfig(capacity=8, initial_nodes=0, id_len=5, seed=3)) as o:
        for i in range(2):
            o.start_node(i)
        br = Bridge(o, sockets=(bin_, bin_, listener.getsockname(), uni))
        br.run_round()                     # round 0: the two Joins go out
        got = []
        for _ in range(2):
            dg, _src = listener.recvfrom(wire.INCOMING_BUFFER_SIZE)
            got.append(wire.receive(dg, "broadcast"))
        assert [(g["kind"], wire.id_of(g["peer"]), g["identity"]) for g in got] == \
            [("Join", 0, o.identity(0)), ("Join", 1, o.identity(1))]
        # discover_mesh_member: Probe(self_addr) to the broadcast port
        paddr = prober.getsockname()
        prober.sendto(wire.encode("Probe", peer=paddr), bin_.getsockname())
        time.sleep(0.05)
        br.run_round()                     # ingested, delivered with round 1's broadcasts
        assert br.stats["probes_in"] == 1
        dg, src = prober.recvfrom(1024)
        env = wire.receive(dg, "discovery")          # discovery.rs:81 reads it as a SwimEnvelope
        assert src == uni.getsockname() and env["identity"] in (o.identity(0), o.identity(1))
        assert br.stats["probe_responses_out"] == 2  # n = 2: both answer (o = 0)
        # a real instance's Join is not a simulated peer: counted, dropped
        prober.sendto(wire.encode("Join", identity=b"real", peer=paddr), bin_.getsockname())
        time.sleep(0.05)
        br.run_round()
        assert br.stats["external_join"] == 1
        br.close()
    for s in (listener, prober):
        s.close()


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
