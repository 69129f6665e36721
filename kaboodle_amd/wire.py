"""The datagrams a real Kaboodle instance exchanges, over the C ABI's codec
(include/kaboodle_sim.h `kb_wire_*`, kaboodle_amd/csrc/kb_wire.h): bincode 1.3.3 of the serde types of
src/structs.rs:65-116.

    encode("Ack", identity=b"node-a", peer=addr_of(5), fingerprint=fp, num_peers=n) -> bytes
    decode(datagram, "unicast") -> dict(kind=..., identity=..., peer=..., ...)

Addresses are ``(ip, port)`` tuples with a dotted IPv4 string; ``addr_of(id)`` / ``id_of(addr)`` map the
simulator's ids.  A KnownPeers message carries ``peers=[(addr, identity), ...]``.
"""
from __future__ import annotations

import ctypes as C

KINDS = {"Ping": 0, "PingRequest": 1, "Ack": 2, "KnownPeers": 3, "KnownPeersRequest": 4,   # SwimMessage
         "Join": 16, "Failed": 17, "Probe": 18,                                          # SwimBroadcast
         "ProbeResponse": 32}
NAMES = {v: k for k, v in KINDS.items()}
CHANNELS = {"unicast": 0, "broadcast": 1, "probe_response": 2}
INCOMING_BUFFER_SIZE = 10240       # src/kaboodle.rs:43: longer datagrams arrive truncated
DISCOVERY_BUFFER_SIZE = 1024       # src/discovery.rs:16: discover_mesh_member's receive buffer


class KbWireAddr(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 4), ("port", C.c_uint16), ("pad", C.c_uint16)]


class KbWireEntry(C.Structure):
    _fields_ = [("addr", KbWireAddr), ("id_off", C.c_uint32), ("id_len", C.c_uint32)]


class KbWireMsg(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("identity_off", C.c_uint32), ("identity_len", C.c_uint32),
                ("peer", KbWireAddr), ("fingerprint", C.c_uint32), ("num_peers", C.c_uint32),
                ("n_entries", C.c_uint32)]


def _lib():
    from . import lib
    cd = lib().lib
    if not getattr(cd, "_kb_wire_bound", False):
        cd.kb_wire_encode.restype = C.c_int
        cd.kb_wire_encode.argtypes = [C.POINTER(KbWireMsg), C.POINTER(KbWireEntry), C.c_char_p, C.c_void_p,
                                      C.c_size_t, C.POINTER(C.c_size_t)]
        cd.kb_wire_decode.restype = C.c_int
        cd.kb_wire_decode.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.POINTER(KbWireMsg), C.POINTER(KbWireEntry),
                                      C.c_size_t]
        cd.kb_wire_addr_of_id.restype = C.c_int
        cd.kb_wire_addr_of_id.argtypes = [C.c_uint32, C.POINTER(KbWireAddr)]
        cd.kb_wire_id_of_addr.restype = C.c_int
        cd.kb_wire_id_of_addr.argtypes = [C.POINTER(KbWireAddr), C.POINTER(C.c_uint32)]
        cd._kb_wire_bound = True
    return cd


def _to_c(addr) -> KbWireAddr:
    ip, port = addr
    a = KbWireAddr()
    for k, part in enumerate(ip.split(".")):
        a.ip[k] = int(part)
    a.port = port
    return a


def _from_c(a: KbWireAddr):
    return ".".join(str(a.ip[k]) for k in range(4)), int(a.port)


def addr_of(node_id: int):
    a = KbWireAddr()
    if _lib().kb_wire_addr_of_id(node_id, C.byref(a)) != 0:
        raise ValueError(f"no simulated address for id {node_id}")
    return _from_c(a)


def id_of(addr) -> int | None:
    out = C.c_uint32()
    return int(out.value) if _lib().kb_wire_id_of_addr(C.byref(_to_c(addr)), C.byref(out)) == 0 else None


def encode(kind: str, identity: bytes = b"", peer=None, fingerprint: int = 0, num_peers: int = 0,
           peers=()) -> bytes:
    """One datagram: SwimEnvelope{identity, msg} for the SwimMessage kinds, a SwimBroadcast for Join (its
    identity) / Failed / Probe, ProbeResponse{identity}."""
    blob = bytearray(identity)
    m = KbWireMsg(kind=KINDS[kind], identity_off=0, identity_len=len(identity), fingerprint=fingerprint,
                  num_peers=num_peers, n_entries=len(peers))
    if peer is not None:
        m.peer = _to_c(peer)
    entries = (KbWireEntry * max(1, len(peers)))()
    for k, (a, ident) in enumerate(peers):
        entries[k].addr = _to_c(a)
        entries[k].id_off, entries[k].id_len = len(blob), len(ident)
        blob += ident
    size = C.c_size_t()
    cd = _lib()
    rc = cd.kb_wire_encode(C.byref(m), entries, bytes(blob), None, 0, C.byref(size))
    if rc != 0:
        raise ValueError(f"kb_wire_encode: {rc}")
    out = C.create_string_buffer(size.value)
    rc = cd.kb_wire_encode(C.byref(m), entries, bytes(blob), C.cast(out, C.c_void_p), size.value, C.byref(size))
    if rc != 0:
        raise ValueError(f"kb_wire_encode: {rc}")
    return out.raw[: size.value]


def receive(datagram: bytes, channel: str = "unicast") -> dict:
    """The message as the reference's receivers decode it: they deserialize the whole reused receive
    buffer, not the datagram's length (`bincode::deserialize(&buf)`, src/kaboodle.rs:259,397): the bytes
    past the datagram are zeros (a fresh buffer), so a short datagram can still decode.  Channel
    "discovery" is discover_mesh_member's reply socket (src/discovery.rs:16,81): a 1024-byte buffer read
    as a SwimEnvelope, so a ProbeResponse{identity} decodes as SwimEnvelope{identity, Ping}."""
    size = DISCOVERY_BUFFER_SIZE if channel == "discovery" else INCOMING_BUFFER_SIZE
    buf = bytearray(size)
    k = min(len(datagram), size)
    buf[:k] = datagram[:k]
    return decode(bytes(buf), "unicast" if channel == "discovery" else channel)


def decode(datagram: bytes, channel: str = "unicast") -> dict:
    """The message in a datagram: at most INCOMING_BUFFER_SIZE bytes are read, so an oversize datagram
    fails (ValueError), as in the reference (Q3).  Decodes the datagram's own bytes only; `receive`
    reproduces the reference receivers' zero-padded buffer."""
    buf = bytes(datagram[:INCOMING_BUFFER_SIZE])
    m = KbWireMsg()
    cd = _lib()
    rc = cd.kb_wire_decode(buf, len(buf), CHANNELS[channel], C.byref(m), None, 0)
    if rc != 0:
        raise ValueError(f"undecodable datagram ({rc})")
    entries = (KbWireEntry * max(1, m.n_entries))()
    if m.n_entries:
        rc = cd.kb_wire_decode(buf, len(buf), CHANNELS[channel], C.byref(m), entries, m.n_entries)
        if rc != 0:
            raise ValueError(f"undecodable datagram ({rc})")
    out = {"kind": NAMES[m.kind], "identity": buf[m.identity_off:m.identity_off + m.identity_len]}
    if m.kind in (KINDS["PingRequest"], KINDS["Ack"], KINDS["Join"], KINDS["Failed"], KINDS["Probe"]):
        out["peer"] = _from_c(m.peer)
    if m.kind in (KINDS["Ack"], KINDS["KnownPeersRequest"]):
        out["fingerprint"], out["num_peers"] = int(m.fingerprint), int(m.num_peers)
    if m.kind == KINDS["KnownPeers"]:
        out["peers"] = [(_from_c(e.addr), buf[e.id_off:e.id_off + e.id_len]) for e in entries[: m.n_entries]]
    return out
