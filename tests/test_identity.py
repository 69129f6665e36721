"""Identity and restarts on the boundary (src/lib.rs:136-183, :323-345, src/structs.rs:18-22), on the CPU
oracle.  set_identity is refused while the node runs as the API sees it (queued start/stop calls count).
Views hold the identity an address announced (PeerInfo.identity).  A stopped instance restarts at a fresh
address (src/kaboodle.rs:138-152) with its map (src/lib.rs:104), carrying the identity set while stopped;
the old address keeps its identity in the views that still hold it."""
import zlib

import pytest

import parity
from kaboodle_amd._ffi import KB_CAPACITY, KB_INIT_CONVERGED, KB_INVALID_OPERATION, KbError, Sim, SimConfig


def _fp(sim, node):
    h = 0
    for p in sim.peers(node):
        h = zlib.crc32(sim.format_addr(p).encode(), h)
        h = zlib.crc32(sim.identity(p), h)
    return h


def test_set_identity_and_restart_oracle():
    cfg = SimConfig(capacity=64, initial_nodes=60, init_mode=KB_INIT_CONVERGED, id_len=3, seed=4)
    with Sim(parity.oracle_lib(), cfg) as o:
        o.step(1)
        with pytest.raises(KbError) as e:
            o.set_identity(3, b"xyz")
        assert e.value.code == KB_INVALID_OPERATION
        old3 = o.identity(3)
        o.stop_node(3)
        o.set_identity(3, b"xyz")                  # kept for the instance's next address
        assert o.identity(3) == old3               # the views of address 3 hold what it announced
        with pytest.raises(KbError) as e:
            o.start_node(3)                        # a stopped instance that ran: restart instead
        assert e.value.code == KB_INVALID_OPERATION
        new = o.restart_node(3)
        assert new == 60 and o.identity(60) == b"xyz"
        assert o.restart_node(new) == new          # queued start: running as the API sees it (no-op)
        with pytest.raises(KbError):
            o.set_identity(new, b"abc")
        o.set_identity(62, b"new")                 # never bound: takes effect at once
        assert o.identity(62) == b"new" and o.restart_node(62) == 62
        o.step(1)
        before = set(o.peers(3))
        assert o.is_running(60) and not o.is_running(3)
        assert set(o.peers(60)) == (before | {60}) - {3} or 3 not in o.peers(60)
        assert o.stats()["next_free_id"] == 61
        o.step(2)
        ps = {e[0]: e[4] for e in o.peer_states(10)}
        assert ps.get(3, old3) == old3 and ps.get(60, b"xyz") == b"xyz"
        assert _fp(o, 10) == o.fingerprint(10) and _fp(o, 60) == o.fingerprint(60)


def test_restart_keeps_the_map_oracle():
    """The restarted instance's map is the old one minus the old self plus the new self; states, instants
    and latencies carry over (peer_states), curious peers and the ping queue do not."""
    cfg = SimConfig(capacity=40, initial_nodes=36, init_mode=KB_INIT_CONVERGED, loss=0.05, seed=8, track_latency=1)
    with Sim(parity.oracle_lib(), cfg) as o:
        o.step(6)
        o.stop_node(9)
        o.step(1)
        kept = [e for e in o.peer_states(9)]
        new = o.restart_node(9)
        o.step(0)                                  # nothing applied until the next round starts
        o.step(1)
        got = {e[0]: e for e in o.peer_states(new)}
        assert new in got and 9 not in got
        changed = [e for e in kept if e[0] in got and got[e[0]][1:4] != e[1:4]]
        assert len(changed) < len(kept)            # most entries untouched by one round
        assert o.curious(new) == [] or all(c[0] != 9 for c in o.curious(new))


def test_restart_capacity_oracle():
    cfg = SimConfig(capacity=8, initial_nodes=8, init_mode=KB_INIT_CONVERGED, seed=1)
    with Sim(parity.oracle_lib(), cfg) as o:
        o.step(1)
        o.stop_node(2)
        o.step(1)
        with pytest.raises(KbError) as e:
            o.restart_node(2)
        assert e.value.code == KB_CAPACITY
