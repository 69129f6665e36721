"""Wire codec: the C ABI's kb_wire_* against byte vectors derived by hand from
the bincode 1.3.3 legacy encoding rules (little-endian fixed-width integers, u64 lengths, u32 enum
variant tags, serde's non-human-readable SocketAddr = newtype variant V4(tag 0) + 4 octets + u16 port,
bytes::Bytes = u64 length + bytes) applied to src/structs.rs:65-116.  The reference cannot be built here,
so these vectors are spec-derived: parity with crates.io bincode itself is unpinned.  They are also
checked against the simulator's own size rule 20 + L + Σ(18 + L_j) and its
10240-byte receive buffer (src/kaboodle.rs:43).  Host code only: runs without a GPU."""
import os
import random

import pytest

from parity import GPU_SO

pytestmark = pytest.mark.skipif(not os.path.exists(GPU_SO), reason="HIP library not built (run __graft_entry__.build())")


def W():
    from kaboodle_amd import wire
    return wire


def h(s: str) -> bytes:
    return bytes.fromhex(s.replace(" ", ""))


Z8 = "00" * 8


def test_addresses():
    w = W()
    assert w.addr_of(0) == ("10.100.100.100", 10000)
    assert w.addr_of(50000) == ("10.100.100.101", 10000)
    assert w.addr_of(1234567) == ("10.100.100.124", 44567)
    assert w.id_of(w.addr_of(7799999)) == 7799999
    assert w.id_of(("192.168.1.7", 4000)) is None


@pytest.mark.parametrize("kind,kw,hexbytes", [
    ("Ping", dict(identity=b"top-left"), "0800000000000000 746f702d6c656674 00000000"),
    ("PingRequest", dict(peer=("10.100.100.100", 10005)), Z8 + "01000000 00000000 0a646464 1527"),
    ("Ack", dict(identity=b"ab", peer=("10.100.100.101", 10000), fingerprint=0x981285C8, num_peers=4),
     "0200000000000000 6162 02000000 00000000 0a646465 1027 c8851298 04000000"),
    ("KnownPeersRequest", dict(fingerprint=0x42561112, num_peers=7), Z8 + "04000000 12115642 07000000"),
    ("KnownPeers", dict(peers=[(("10.100.100.100", 10000), b"x"), (("10.100.100.100", 10001), b"")]),
     Z8 + "03000000 0200000000000000" + "00000000 0a646464 1027 0100000000000000 78"
     + "00000000 0a646464 1127" + Z8),
])
def test_envelope_vectors(kind, kw, hexbytes):
    w = W()
    want = h(hexbytes)
    got = w.encode(kind, **kw)
    assert got == want, got.hex()
    d = w.decode(got, "unicast")
    assert d["kind"] == kind and d["identity"] == kw.get("identity", b"")
    for k in ("peer", "fingerprint", "num_peers", "peers"):
        if k in kw:
            assert d[k] == kw[k]


@pytest.mark.parametrize("kind,kw,channel,hexbytes", [
    ("Join", dict(peer=("10.100.100.100", 10003), identity=b"z"), "broadcast",
     "00000000 00000000 0a646464 1327 0100000000000000 7a"),
    ("Failed", dict(peer=("10.100.100.100", 10002)), "broadcast", "01000000 00000000 0a646464 1227"),
    ("Probe", dict(peer=("192.168.1.7", 4000)), "broadcast", "02000000 00000000 c0a80107 a00f"),
    ("ProbeResponse", dict(identity=b"hi"), "probe_response", "0200000000000000 6869"),
])
def test_broadcast_and_probe_vectors(kind, kw, channel, hexbytes):
    w = W()
    got = w.encode(kind, **kw)
    assert got == h(hexbytes), got.hex()
    d = w.decode(got, channel)
    assert d["kind"] == kind
    if "peer" in kw:
        assert d["peer"] == kw["peer"]
    assert d["identity"] == kw.get("identity", b"")


@pytest.mark.parametrize("L", [0, 5, 32])
def test_known_peers_size_rule_and_receive_buffer(L):
    """The encoded size is exactly 20 + L + Σ(18 + L_j), the rule the simulator applies (Q3): capk
    entries fit the 10240-byte receive buffer, one more arrives truncated and is undecodable."""
    w = W()
    me = bytes(range(65, 65 + L))
    capk = (10240 - 20 - L) // (18 + L)
    ents = [(w.addr_of(j), bytes((j + k) % 256 for k in range(L))) for j in range(capk + 1)]
    ok = w.encode("KnownPeers", identity=me, peers=ents[:capk])
    assert len(ok) == 20 + L + capk * (18 + L) <= 10240
    assert [p for p, _ in w.decode(ok)["peers"]] == [a for a, _ in ents[:capk]]
    big = w.encode("KnownPeers", identity=me, peers=ents)
    assert len(big) == 20 + L + (capk + 1) * (18 + L) > 10240
    with pytest.raises(ValueError):
        w.decode(big)                                   # truncated at 10240 bytes by the receiver


def test_round_trips_and_malformed():
    w = W()
    rng = random.Random(7)
    for _ in range(200):
        kind = rng.choice(list(w.KINDS))
        ident = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 33)))
        peer = w.addr_of(rng.randrange(7_800_000))
        kw = {}
        if kind in ("Ping", "KnownPeersRequest", "Ack", "PingRequest", "KnownPeers", "Join", "ProbeResponse"):
            kw["identity"] = ident
        if kind in ("PingRequest", "Ack", "Join", "Failed", "Probe"):
            kw["peer"] = peer
        if kind in ("Ack", "KnownPeersRequest"):
            kw["fingerprint"], kw["num_peers"] = rng.randrange(2 ** 32), rng.randrange(2 ** 32)
        if kind == "KnownPeers":
            kw["peers"] = [(w.addr_of(rng.randrange(10 ** 6)), bytes(rng.randrange(256) for _ in range(rng.randrange(4))))
                           for _ in range(rng.randrange(20))]
        channel = "broadcast" if kind in ("Join", "Failed", "Probe") else (
            "probe_response" if kind == "ProbeResponse" else "unicast")
        data = w.encode(kind, **kw)
        d = w.decode(data + b"\x00trailing", channel)   # bincode::deserialize ignores trailing bytes
        assert d["kind"] == kind
        for k, v in kw.items():
            assert d[k] == v, (kind, k)
        for cut in (1, len(data) // 2):
            if cut < len(data):
                with pytest.raises(ValueError):
                    w.decode(data[:-cut], channel)
    with pytest.raises(ValueError):
        w.decode(h(Z8 + "05000000"))                        # no such SwimMessage variant
    with pytest.raises(ValueError):
        w.decode(h(Z8 + "01000000 01000000") + bytes(18))   # SocketAddr::V6
