// kb_wire.h — the datagrams a real Kaboodle instance exchanges, host code:
// bincode 1.3.3 with its legacy defaults (`bincode::serialize`: little-endian fixed-width integers,
// u64 lengths, u32 enum variant tags, trailing bytes allowed on decode) of the serde types of
// src/structs.rs:65-116.
//   SwimEnvelope { identity: Bytes, msg: SwimMessage }        unicast socket     (kaboodle.rs:188-226, 394-403)
//   SwimBroadcast { Join{addr, identity} | Failed(Peer) | Probe(SocketAddr) }   multicast (kaboodle.rs:256-311)
//   ProbeResponse { identity: Bytes }                          reply to a Probe   (kaboodle.rs:312-331)
// SocketAddr is serde's non-human-readable form: newtype variant V4 = tag 0, then the four octets
// and the port (10 bytes); V6 (tag 1) is not produced by the simulator and is rejected on decode.
// Bytes = u64 length + bytes.  A KnownPeers map is u64 count + (addr, Bytes) pairs; the reference
// iterates a HashMap (any order), the encoder keeps the caller's order (the simulator's is id order).
// A datagram is read into a 10240-byte buffer (INCOMING_BUFFER_SIZE, :43), so a longer one arrives
// truncated and fails to decode: that is the simulator's oversize rule (Q3), and
// kb_wire_encode's size is exactly the 20 + L + Σ(18 + L_j) it uses.
#pragma once
#include <stdint.h>
#include <string.h>
#include "../../include/kaboodle_sim.h"

namespace kbw {

struct Writer {
  uint8_t* buf; size_t cap, n;
  void bytes(const void* p, size_t k) { if (n + k <= cap && buf) memcpy(buf + n, p, k); n += k; }
  void u16(uint16_t v) { uint8_t b[2] = {(uint8_t)v, (uint8_t)(v >> 8)}; bytes(b, 2); }
  void u32(uint32_t v) { uint8_t b[4]; for (int k = 0; k < 4; ++k) b[k] = (uint8_t)(v >> (8 * k)); bytes(b, 4); }
  void u64(uint64_t v) { uint8_t b[8]; for (int k = 0; k < 8; ++k) b[k] = (uint8_t)(v >> (8 * k)); bytes(b, 8); }
  void addr(const kb_wire_addr& a) { u32(0); bytes(a.ip, 4); u16(a.port); }        // SocketAddr::V4
  void blob(const uint8_t* p, uint32_t len) { u64(len); bytes(p, len); }              // bytes::Bytes
};

struct Reader {
  const uint8_t* buf; size_t len, n; bool ok;
  bool need(size_t k) { if (!ok || len - n < k || n > len) { ok = false; return false; } return true; }
  uint16_t u16() { if (!need(2)) return 0; uint16_t v = (uint16_t)(buf[n] | buf[n + 1] << 8); n += 2; return v; }
  uint32_t u32() { if (!need(4)) return 0; uint32_t v = 0; for (int k = 0; k < 4; ++k) v |= (uint32_t)buf[n + k] << (8 * k); n += 4; return v; }
  uint64_t u64() { if (!need(8)) return 0; uint64_t v = 0; for (int k = 0; k < 8; ++k) v |= (uint64_t)buf[n + k] << (8 * k); n += 8; return v; }
  void addr(kb_wire_addr& a) {
    memset(&a, 0, sizeof a);
    if (u32() != 0) { ok = false; return; }                   // only SocketAddr::V4
    if (!need(4)) return;
    memcpy(a.ip, buf + n, 4); n += 4;
    a.port = u16();
  }
  void blob(uint32_t& off, uint32_t& blen) {
    const uint64_t l = u64();
    if (!ok || l > len - n) { ok = false; return; }
    off = (uint32_t)n; blen = (uint32_t)l; n += (size_t)l;
  }
};

}  // namespace kbw

extern "C" int kb_wire_encode(const kb_wire_msg* m, const kb_wire_entry* entries, const uint8_t* idents, uint8_t* buf,
                              size_t cap, size_t* size) {
  if (!m || !size || (m->identity_len && !idents)) return KB_INVALID_ARGUMENT;
  kbw::Writer w{buf, cap, 0};
  const uint8_t* idp = idents ? idents + m->identity_off : nullptr;
  switch (m->kind) {
    case KB_WIRE_PING: case KB_WIRE_PING_REQUEST: case KB_WIRE_ACK: case KB_WIRE_KNOWN_PEERS:
    case KB_WIRE_KNOWN_PEERS_REQUEST:
      w.blob(idp, m->identity_len);                             // SwimEnvelope.identity
      w.u32(m->kind);                                           // SwimMessage variant (declaration order)
      if (m->kind == KB_WIRE_PING_REQUEST) w.addr(m->peer);
      else if (m->kind == KB_WIRE_ACK) { w.addr(m->peer); w.u32(m->fingerprint); w.u32(m->num_peers); }
      else if (m->kind == KB_WIRE_KNOWN_PEERS_REQUEST) { w.u32(m->fingerprint); w.u32(m->num_peers); }
      else if (m->kind == KB_WIRE_KNOWN_PEERS) {
        if (m->n_entries && (!entries || !idents)) return KB_INVALID_ARGUMENT;
        w.u64(m->n_entries);
        for (uint32_t k = 0; k < m->n_entries; ++k) { w.addr(entries[k].addr); w.blob(idents + entries[k].id_off, entries[k].id_len); }
      }
      break;
    case KB_WIRE_JOIN: w.u32(0); w.addr(m->peer); w.blob(idp, m->identity_len); break;
    case KB_WIRE_FAILED: w.u32(1); w.addr(m->peer); break;
    case KB_WIRE_PROBE: w.u32(2); w.addr(m->peer); break;
    case KB_WIRE_PROBE_RESPONSE: w.blob(idp, m->identity_len); break;
    default: return KB_INVALID_ARGUMENT;
  }
  *size = w.n;
  return (buf && cap >= w.n) || !buf ? KB_OK : KB_CAPACITY;
}

extern "C" int kb_wire_decode(const uint8_t* buf, size_t len, int channel, kb_wire_msg* m, kb_wire_entry* entries,
                              size_t cap) {
  if (!buf || !m) return KB_INVALID_ARGUMENT;
  memset(m, 0, sizeof *m);
  kbw::Reader r{buf, len, 0, true};
  if (channel == KB_WIRE_CHANNEL_UNICAST) {
    r.blob(m->identity_off, m->identity_len);
    const uint32_t tag = r.u32();
    if (!r.ok || tag > KB_WIRE_KNOWN_PEERS_REQUEST) return KB_INVALID_ARGUMENT;
    m->kind = tag;
    if (tag == KB_WIRE_PING_REQUEST) r.addr(m->peer);
    else if (tag == KB_WIRE_ACK) { r.addr(m->peer); m->fingerprint = r.u32(); m->num_peers = r.u32(); }
    else if (tag == KB_WIRE_KNOWN_PEERS_REQUEST) { m->fingerprint = r.u32(); m->num_peers = r.u32(); }
    else if (tag == KB_WIRE_KNOWN_PEERS) {
      const uint64_t cnt = r.u64();
      if (!r.ok || cnt > (len - r.n) / 18) return KB_INVALID_ARGUMENT;   // each entry takes >= 18 bytes
      m->n_entries = (uint32_t)cnt;
      for (uint64_t k = 0; k < cnt && r.ok; ++k) {
        kb_wire_entry e;
        r.addr(e.addr);
        r.blob(e.id_off, e.id_len);
        if (entries && k < cap) entries[k] = e;
      }
    }
  } else if (channel == KB_WIRE_CHANNEL_BROADCAST) {
    const uint32_t tag = r.u32();
    if (!r.ok || tag > 2) return KB_INVALID_ARGUMENT;
    m->kind = KB_WIRE_JOIN + tag;
    r.addr(m->peer);
    if (tag == 0) r.blob(m->identity_off, m->identity_len);
  } else if (channel == KB_WIRE_CHANNEL_PROBE_RESPONSE) {
    m->kind = KB_WIRE_PROBE_RESPONSE;
    r.blob(m->identity_off, m->identity_len);
  } else {
    return KB_INVALID_ARGUMENT;
  }
  if (!r.ok) return KB_INVALID_ARGUMENT;                        // truncated or malformed (trailing bytes allowed)
  return (entries && cap < m->n_entries) ? KB_CAPACITY : KB_OK;
}

// the simulator's canonical address of an id and back
extern "C" int kb_wire_addr_of_id(uint32_t id, kb_wire_addr* out) {
  if (!out || id >= 7800000u) return KB_INVALID_ARGUMENT;
  memset(out, 0, sizeof *out);
  out->ip[0] = 10; out->ip[1] = 100; out->ip[2] = 100; out->ip[3] = (uint8_t)(100 + id / 50000u);
  out->port = (uint16_t)(10000 + id % 50000u);
  return KB_OK;
}
extern "C" int kb_wire_id_of_addr(const kb_wire_addr* a, uint32_t* id) {
  if (!a || !id) return KB_INVALID_ARGUMENT;
  if (a->ip[0] != 10 || a->ip[1] != 100 || a->ip[2] != 100 || a->ip[3] < 100 || a->port < 10000 || a->port >= 60000)
    return KB_INVALID_ARGUMENT;                                 // not a simulated peer
  *id = (uint32_t)(a->ip[3] - 100) * 50000u + (uint32_t)(a->port - 10000);
  return *id < 7800000u ? KB_OK : KB_INVALID_ARGUMENT;
}
