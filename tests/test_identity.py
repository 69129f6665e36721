"""Identity on the boundary (src/lib.rs:323-345, src/structs.rs:18-22), on the CPU oracle: set_identity is
refused while the node runs as the API sees it (queued start/stop calls count), peers and peer_states
carry the identity bytes, and a changed identity is what fingerprints use from then on."""
import pytest

import parity
from kaboodle_amd._ffi import KB_INIT_CONVERGED, KB_INVALID_OPERATION, KbError, Sim, SimConfig


def test_set_identity_lifecycle_oracle():
    cfg = SimConfig(capacity=64, initial_nodes=60, init_mode=KB_INIT_CONVERGED, id_len=3, seed=4)
    with Sim(parity.oracle_lib(), cfg) as o:
        o.step(1)
        with pytest.raises(KbError) as e:
            o.set_identity(3, b"xyz")
        assert e.value.code == KB_INVALID_OPERATION
        o.stop_node(3)
        o.set_identity(3, b"xyz")
        assert o.identity(3) == b"xyz"
        o.start_node(3)
        with pytest.raises(KbError):
            o.set_identity(3, b"abc")
        o.set_identity(62, b"new")                 # never started: allowed
        o.step(2)
        ps = {e[0]: e[4] for e in o.peer_states(10)}
        assert ps[3] == b"xyz" and all(len(v) == 3 for v in ps.values())
        # the fingerprint is generate_fingerprint over (addr || identity) in address order
        import zlib
        h = 0
        for p in o.peers(10):
            h = zlib.crc32(o.format_addr(p).encode(), h)
            h = zlib.crc32(o.identity(p), h)
        assert h == o.fingerprint(10)
