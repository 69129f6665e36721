"""Discovery (src/discovery.rs:30-89) and maybe_respond_to_probe (src/kaboodle.rs:305-331) on the CPU oracle:
who answers a Probe, what the ProbeResponse datagram carries and how the prober decodes it, the
re-broadcast back-off of discover_mesh_member, and the broadcast lists a bridge would send."""
import os

import pytest

import parity
from kaboodle_amd._ffi import KB_INIT_CONVERGED, Sim, SimConfig

HIP = os.path.exists(parity.GPU_SO)


def test_small_mesh_always_answers():
    """should_respond_to_broadcast: o = n - 2 <= 0 answers always (a 1- or 2-peer mesh)."""
    with Sim(parity.oracle_lib(), SimConfig(capacity=4, initial_nodes=2, seed=2)) as o:
        o.step(2)
        o.probe(("192.0.2.1", 9000))
        o.step(1)
        resp = o.probe_responses()
        assert sorted(r[1] for r in resp) == [0, 1]
        assert all(r[0] == 2 and r[3] == ("192.0.2.1", 9000) for r in resp)
        assert o.probe_responses() == []                  # drained
        assert o.stats()["probe_responses"] == 2


def test_large_mesh_answers_about_one_percent():
    """o = n - 2 large: respond with probability max(1, 100 - o^2) % = 1 %."""
    n = 1000
    with Sim(parity.oracle_lib(), SimConfig(capacity=n, initial_nodes=n, init_mode=KB_INIT_CONVERGED, seed=4)) as o:
        o.step(1)
        for k in range(20):
            o.probe(("192.0.2.9", 7000 + k))
        o.step(1)
        resp = o.probe_responses()
        assert 100 <= len(resp) <= 320, len(resp)           # 20 probes x 1000 peers x 1 %
        assert {r[2] for r in resp} == set(range(20))


def test_probe_lost_with_total_loss():
    with Sim(parity.oracle_lib(), SimConfig(capacity=4, initial_nodes=2, loss=1.0, seed=2)) as o:
        o.step(1)
        o.probe(("192.0.2.1", 9000))
        o.step(1)
        assert o.probe_responses() == []
        assert o.stats()["drop_bcast"] >= 2


@pytest.mark.skipif(not HIP, reason="wire codec lives in the HIP library (loads without a GPU)")
def test_probe_response_datagram_as_discovery_reads_it():
    """ProbeResponse{identity} read by discover_mesh_member from a 1024-byte buffer as a SwimEnvelope
    (src/discovery.rs:16,81): identity intact, the zero tail reads as Ping."""
    from kaboodle_amd import wire
    with Sim(parity.oracle_lib(), SimConfig(capacity=4, initial_nodes=2, id_len=6, seed=2)) as o:
        o.step(1)
        o.probe(("192.0.2.1", 9000))
        o.step(1)
        (rnd, responder, _, prober, ident), *_ = o.probe_responses()
        dg = wire.encode("ProbeResponse", identity=ident)
        env = wire.receive(dg, "discovery")
        assert env["kind"] == "Ping" and env["identity"] == ident == o.identity(responder)
        with pytest.raises(ValueError):
            wire.decode(dg, "unicast")                     # the datagram alone is a truncated envelope


@pytest.mark.skipif(not HIP, reason="the Mesh mirror binds the HIP library's ABI")
def test_discover_mesh_member_backoff():
    """The prober's schedule (discovery.rs:46-73): probe, wait 1 s, then 1.25 s, 1.56 s, ... up to 10 s
    between re-broadcasts, one simulated round per second; nothing answers under total loss."""
    import kaboodle_amd

    class Probed:                        # the oracle standing in for the Mesh (a Sim with the same methods)
        def __init__(self, sim):
            self.sim, self.rounds, self.probes = sim, 0, []

        def probe(self, a):
            self.probes.append(self.rounds)
            self.sim.probe(a)

        def step(self, k):
            self.sim.step(k)
            self.rounds += k

        def probe_responses(self):
            return self.sim.probe_responses()

        def format_addr(self, i):
            return self.sim.format_addr(i)

    with Sim(parity.oracle_lib(), SimConfig(capacity=4, initial_nodes=2, loss=1.0, seed=2)) as o:
        p = Probed(o)
        assert kaboodle_amd.discover_mesh_member(p, ("192.0.2.1", 9000), max_rounds=40) is None
        gaps = [b - a for a, b in zip(p.probes, p.probes[1:])]
        assert gaps[:3] == [2, 2, 2] and max(gaps) <= 10 and gaps == sorted(gaps), gaps
    with Sim(parity.oracle_lib(), SimConfig(capacity=4, initial_nodes=2, id_len=3, seed=2)) as o:
        o.step(1)
        addr, ident = kaboodle_amd.discover_mesh_member(Probed(o), ("192.0.2.1", 9000))
        assert addr == "10.100.100.100:10000" and ident == o.identity(0)


def test_broadcast_lists():
    """The Join / Failed lists of the last round (what a bridge sends on the multicast socket)."""
    with Sim(parity.oracle_lib(), SimConfig(capacity=8, initial_nodes=0, seed=1)) as o:
        for i in range(3):
            o.start_node(i)
        o.step(1)
        assert o.broadcasts() == [("Join", 0, 0), ("Join", 1, 1), ("Join", 2, 2)]
        o.step(1)
        assert o.broadcasts() == []
