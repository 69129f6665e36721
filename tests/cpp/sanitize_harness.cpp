// sanitize_harness.cpp — host harness run under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only,
// tests/test_sanitize.py builds it with g++ -fsanitize=address,undefined):
//   scenarios   the CPU oracle (oracle/kb_oracle.c: manual realloc'd outboxes, event lists, probe queues,
//               watch snapshots) through the whole kbo_ ABI on small meshes: joins, loss, churn, partition
//               and heal, stop / restart / set_identity, probes, event drains, latency, both failed
//               modes, the exact-LRU variant, and every inspection call;
//   decode      the network-facing wire decoder (kaboodle_amd/csrc/kb_wire.h, fed by bridge.py from real
//               sockets): datagrams from stdin (u32 length + bytes, repeated) decoded on every channel with
//               and without an entries buffer; valid encodings must round-trip.
//   fuzz N      N random and mutated datagrams (seeded xorshift) through the same decoder.
// Exit status 0 = every check passed (the sanitizers abort on the first error they find).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../kaboodle_amd/csrc/kb_wire.h"

extern "C" {
typedef struct kbo_sim kbo_sim;
void kbo_config_default(kb_config*);
int kbo_sim_create(const kb_config*, kbo_sim**);
int kbo_sim_destroy(kbo_sim*);
int kbo_sim_step(kbo_sim*, uint32_t);
int kbo_sim_start_node(kbo_sim*, uint32_t);
int kbo_sim_stop_node(kbo_sim*, uint32_t);
int kbo_sim_restart_node(kbo_sim*, uint32_t, uint32_t*);
int kbo_sim_ping_addrs(kbo_sim*, uint32_t, const uint32_t*, size_t);
int kbo_sim_set_identity(kbo_sim*, uint32_t, const uint8_t*, size_t);
int kbo_sim_identity(kbo_sim*, uint32_t, uint8_t*, size_t, size_t*);
int kbo_sim_fingerprint(kbo_sim*, uint32_t, uint32_t*);
int kbo_sim_fingerprints(kbo_sim*, uint32_t*, size_t);
int kbo_sim_true_fingerprint(kbo_sim*, uint32_t*);
int kbo_sim_peers(kbo_sim*, uint32_t, uint32_t*, size_t, size_t*);
int kbo_sim_peer_states(kbo_sim*, uint32_t, kb_peer_state*, size_t, size_t*);
int kbo_sim_stats(kbo_sim*, kb_stats*);
int kbo_sim_watch(kbo_sim*, uint32_t);
int kbo_sim_events(kbo_sim*, uint32_t, uint32_t*, size_t, size_t*, uint32_t*, size_t, size_t*, uint32_t*, int*);
int kbo_sim_probe(kbo_sim*, const kb_wire_addr*);
int kbo_sim_probe_responses(kbo_sim*, kb_probe_response*, size_t, size_t*);
int kbo_sim_broadcasts(kbo_sim*, kb_broadcast*, size_t, size_t*);
int kbo_sim_dump_row(kbo_sim*, uint32_t, uint8_t*, size_t);
int kbo_sim_dump_scalars(kbo_sim*, int32_t*, size_t);
int kbo_sim_dump_suspects(kbo_sim*, uint32_t, int32_t*, size_t, size_t*);
int kbo_sim_dump_curious(kbo_sim*, uint32_t, int32_t*, size_t, size_t*);
uint32_t kbo_fingerprint_of_set(const uint32_t*, size_t, const uint8_t*, size_t, const uint8_t*);
}

static int fails = 0;
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

// every inspection call of the ABI on every node (size queries first, then exact buffers)
static void inspect(kbo_sim* s, uint32_t C) {
  std::vector<uint32_t> fps(C);
  CHECK(kbo_sim_fingerprints(s, fps.data(), C) == KB_OK);
  uint32_t tf = 0;
  CHECK(kbo_sim_true_fingerprint(s, &tf) == KB_OK);
  std::vector<int32_t> sc(4 * C);
  CHECK(kbo_sim_dump_scalars(s, sc.data(), sc.size()) == KB_OK);
  std::vector<uint8_t> row(C);
  for (uint32_t i = 0; i < C; ++i) {
    size_t n = 0;
    CHECK(kbo_sim_peers(s, i, nullptr, 0, &n) == KB_OK);
    std::vector<uint32_t> p(n + 1);
    CHECK(kbo_sim_peers(s, i, p.data(), n, &n) == KB_OK);
    CHECK(kbo_sim_peer_states(s, i, nullptr, 0, &n) == KB_OK);
    std::vector<kb_peer_state> ps(n + 1);
    CHECK(kbo_sim_peer_states(s, i, ps.data(), n, &n) == KB_OK);
    if (n) CHECK(kbo_sim_peer_states(s, i, ps.data(), n - 1, &n) == KB_CAPACITY);
    CHECK(kbo_sim_dump_row(s, i, row.data(), C) == KB_OK);
    int32_t buf[64];
    CHECK(kbo_sim_dump_suspects(s, i, buf, 64, &n) == KB_OK);
    CHECK(kbo_sim_dump_curious(s, i, buf, 64, &n) == KB_OK);
    uint8_t id[32];
    CHECK(kbo_sim_identity(s, i, id, sizeof id, &n) == KB_OK);
    uint32_t f = 0;
    CHECK(kbo_sim_fingerprint(s, i, &f) == KB_OK);
  }
  size_t nb = 0;
  CHECK(kbo_sim_broadcasts(s, nullptr, 0, &nb) == KB_OK);
  std::vector<kb_broadcast> b(nb + 1);
  CHECK(kbo_sim_broadcasts(s, b.data(), nb, &nb) == KB_OK);
  size_t np = 0;
  CHECK(kbo_sim_probe_responses(s, nullptr, 0, &np) == KB_OK);
  std::vector<kb_probe_response> pr(np + 1);
  CHECK(kbo_sim_probe_responses(s, pr.data(), np, &np) == KB_OK);
  kb_stats st;
  CHECK(kbo_sim_stats(s, &st) == KB_OK);
}

static void drain(kbo_sim* s, uint32_t node) {
  size_t nd = 0, np = 0;
  uint32_t fp = 0;
  int ch = 0;
  if (kbo_sim_events(s, node, nullptr, 0, &nd, nullptr, 0, &np, &fp, &ch) != KB_OK) return;
  std::vector<uint32_t> d(nd + 1), p(np + 1);
  CHECK(kbo_sim_events(s, node, d.data(), nd, &nd, p.data(), np, &np, &fp, &ch) == KB_OK);
}

static int scenarios() {
  struct Sc { uint32_t cap, init, mode, loss_pm, churn_pm, faults, fmode, idlen, groups, lat, variant, rounds; };
  const Sc list[] = {
      {4, 0, KB_INIT_JOIN, 0, 0, 0, 0, 8, 0, 0, 0, 8},
      {300, 300, KB_INIT_JOIN, 20, 0, 0, 0, 5, 0, 1, 0, 20},
      {256, 240, KB_INIT_CONVERGED, 30, 10, 25, 0, 0, 0, 1, 0, 40},
      {200, 200, KB_INIT_CONVERGED, 50, 0, 0, 1, 0, 0, 0, 0, 20},
      {256, 256, KB_INIT_CONVERGED, 20, 0, 0, 0, 0, 2, 1, 0, 30},
      {160, 128, KB_INIT_CONVERGED, 20, 30, 12, 0, 4, 0, 1, 0, 140},
      {96, 80, KB_INIT_CONVERGED, 30, 10, 20, 0, 0, 0, 0, 1, 20},
      {96, 80, KB_INIT_CONVERGED, 30, 10, 20, 0, 0, 0, 0, 2, 20},
      {256, 256, KB_INIT_CONVERGED, 50, 0, 0, 1, 0, 2, 0, 4, 30},     // sparse rows: partition + heal
      {160, 128, KB_INIT_CONVERGED, 20, 30, 12, 0, 4, 0, 0, 4, 140},  // sparse rows: churn, rebases
      {300, 300, KB_INIT_JOIN, 20, 0, 0, 0, 5, 0, 0, 4, 20},          // sparse rows: empty base
  };
  int k = 0;
  for (const Sc& c : list) {
    kb_config cfg;
    kbo_config_default(&cfg);
    cfg.capacity = c.cap; cfg.initial_nodes = c.init; cfg.init_mode = c.mode; cfg.seed = 7 + k;
    cfg.loss_threshold = (uint32_t)((uint64_t)c.loss_pm * 4294967296ull / 1000);
    cfg.churn_threshold = (uint32_t)((uint64_t)c.churn_pm * 4294967296ull / 1000);
    cfg.fault_end_round = c.faults ? (int32_t)c.faults : -1;
    cfg.failed_mode = c.fmode; cfg.id_len = c.idlen; cfg.track_latency = c.lat; cfg.variant = c.variant;
    if (c.groups) { cfg.partition_groups = c.groups; cfg.partition_start = 3; cfg.partition_end = 12; }
    kbo_sim* s = nullptr;
    CHECK(kbo_sim_create(&cfg, &s) == KB_OK);
    if (!s) return 1;
    const uint32_t C = c.cap;
    if (c.init == 0) {
      const char* names[4] = {"top-left", "top-right", "bottom-left", "bottom-right"};
      for (uint32_t i = 0; i < 4 && i < C; ++i) {
        CHECK(kbo_sim_set_identity(s, i, (const uint8_t*)names[i], strlen(names[i])) == KB_OK);
        CHECK(kbo_sim_start_node(s, i) == KB_OK);
      }
    }
    CHECK(kbo_sim_watch(s, 0) == KB_OK);
    CHECK(kbo_sim_watch(s, C - 1) == KB_OK);
    uint32_t moved = 0;                 // node 1's instance: stopped at round 3, restarted at round 5
    for (uint32_t r = 0; r < c.rounds; ++r) {
      if (r == 1) { kb_wire_addr a = {{192, 0, 2, 1}, 4000, 0}; CHECK(kbo_sim_probe(s, &a) == KB_OK); }
      if (r == 3 && C > 4) {
        const uint8_t again[32] = {'a', 'g', 'a', 'i', 'n', '-', 'a', 'g', 'a', 'i', 'n'};
        CHECK(kbo_sim_stop_node(s, 1) == KB_OK);
        CHECK(kbo_sim_set_identity(s, 1, again, c.idlen) == KB_OK);
      }
      if (r == 5 && C > 4) {
        const int rc = kbo_sim_restart_node(s, 1, &moved);
        CHECK(rc == KB_OK || rc == KB_CAPACITY);
        if (rc == KB_OK) CHECK(kbo_sim_watch(s, moved) == KB_OK);
      }
      if (r == 10 && c.groups) {
        for (uint32_t i = 0; i < C; i += 16) { const uint32_t t = (i + C / 2) % C; const int rc = kbo_sim_ping_addrs(s, i, &t, 1); CHECK(rc == KB_OK || rc == KB_INVALID_OPERATION); }
      }
      CHECK(kbo_sim_step(s, 1) == KB_OK);
      drain(s, 0); drain(s, C - 1);
      if (moved) drain(s, moved);
      if (r % 7 == 0 || r + 1 == c.rounds) inspect(s, C);
    }
    std::vector<uint32_t> ids;
    for (uint32_t i = 0; i < C; i += 3) ids.push_back(i);
    (void)kbo_fingerprint_of_set(ids.data(), ids.size(), nullptr, 0, nullptr);
    CHECK(kbo_sim_destroy(s) == KB_OK);
    ++k;
  }
  printf("scenarios: %d run, %d failures\n", k, fails);
  return fails != 0;
}

// decode one datagram on every channel, with and without an entries buffer; a successful unicast decode of
// KnownPeers must address its entries and identities inside the datagram
static void decode_all(const uint8_t* dg, size_t len) {
  for (int ch = 0; ch < 3; ++ch) {
    kb_wire_msg m;
    const int rc0 = kb_wire_decode(dg, len, ch, &m, nullptr, 0);
    std::vector<kb_wire_entry> e(8);
    const int rc1 = kb_wire_decode(dg, len, ch, &m, e.data(), e.size());
    CHECK((rc0 == KB_OK) == (rc1 == KB_OK || rc1 == KB_CAPACITY));
    if (rc1 == KB_OK || rc1 == KB_CAPACITY) {
      CHECK((size_t)m.identity_off + m.identity_len <= len);
      for (uint32_t q = 0; q < m.n_entries && q < e.size(); ++q) CHECK((size_t)e[q].id_off + e[q].id_len <= len);
    }
  }
  kb_wire_msg m;
  (void)kb_wire_decode(dg, len, 7, &m, nullptr, 0);                 // an unknown channel is refused
  (void)kb_wire_decode(dg, len, -1, &m, nullptr, 0);
}

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t)rs; }

// a valid encoding of a random message (round-trip checked), for the mutation fuzz
static std::vector<uint8_t> random_valid() {
  uint8_t idents[512];
  for (auto& x : idents) x = (uint8_t)rnd();
  kb_wire_entry ent[12];
  kb_wire_msg m;
  memset(&m, 0, sizeof m);
  const uint32_t kinds[] = {KB_WIRE_PING, KB_WIRE_PING_REQUEST, KB_WIRE_ACK, KB_WIRE_KNOWN_PEERS,
                            KB_WIRE_KNOWN_PEERS_REQUEST, KB_WIRE_JOIN, KB_WIRE_FAILED, KB_WIRE_PROBE, KB_WIRE_PROBE_RESPONSE};
  m.kind = kinds[rnd() % 9];
  m.identity_off = rnd() % 64; m.identity_len = rnd() % 33;
  for (int k = 0; k < 4; ++k) m.peer.ip[k] = (uint8_t)rnd();
  m.peer.port = (uint16_t)rnd(); m.fingerprint = rnd(); m.num_peers = rnd();
  if (m.kind == KB_WIRE_KNOWN_PEERS) {
    m.n_entries = rnd() % 12;
    for (uint32_t q = 0; q < m.n_entries; ++q) {
      for (int k = 0; k < 4; ++k) ent[q].addr.ip[k] = (uint8_t)rnd();
      ent[q].addr.port = (uint16_t)rnd(); ent[q].addr.pad = 0;
      ent[q].id_off = 100 + rnd() % 300; ent[q].id_len = rnd() % 33;
    }
  }
  size_t sz = 0;
  CHECK(kb_wire_encode(&m, ent, idents, nullptr, 0, &sz) == KB_OK);
  std::vector<uint8_t> dg(sz);
  CHECK(kb_wire_encode(&m, ent, idents, dg.data(), dg.size(), &sz) == KB_OK);
  const int ch = m.kind >= KB_WIRE_PROBE_RESPONSE ? KB_WIRE_CHANNEL_PROBE_RESPONSE : m.kind >= KB_WIRE_JOIN ? KB_WIRE_CHANNEL_BROADCAST
                                                                                                  : KB_WIRE_CHANNEL_UNICAST;
  kb_wire_msg d;
  std::vector<kb_wire_entry> de(16);
  CHECK(kb_wire_decode(dg.data(), dg.size(), ch, &d, de.data(), de.size()) == KB_OK);
  const bool has_id = m.kind != KB_WIRE_FAILED && m.kind != KB_WIRE_PROBE;    // Failed / Probe carry an address only
  CHECK(d.kind == m.kind && d.identity_len == (has_id ? m.identity_len : 0u) && d.n_entries == m.n_entries);
  if (d.identity_len) CHECK(memcmp(dg.data() + d.identity_off, idents + m.identity_off, m.identity_len) == 0);
  for (uint32_t q = 0; q < d.n_entries; ++q)
    CHECK(de[q].id_len == ent[q].id_len && memcmp(&de[q].addr, &ent[q].addr, 6) == 0 &&
          memcmp(dg.data() + de[q].id_off, idents + ent[q].id_off, ent[q].id_len) == 0);
  return dg;
}

static int fuzz(long n) {
  for (long it = 0; it < n; ++it) {
    std::vector<uint8_t> dg;
    if (it % 3 == 0) {                                               // random bytes, random length
      dg.resize(rnd() % 96);
      for (auto& x : dg) x = (uint8_t)rnd();
    } else {                                                         // a valid datagram, mutated
      dg = random_valid();
      const int muts = 1 + rnd() % 4;
      for (int k = 0; k < muts && !dg.empty(); ++k) {
        switch (rnd() % 4) {
          case 0: dg[rnd() % dg.size()] ^= (uint8_t)(1u << (rnd() % 8)); break;
          case 1: dg.resize(rnd() % (dg.size() + 1)); break;
          case 2: { const size_t p = rnd() % dg.size(); for (int b = 0; b < 8 && p + b < dg.size(); ++b) dg[p + b] = 0xFF; break; }
          default: dg.push_back((uint8_t)rnd()); break;
        }
      }
    }
    // decode from an exactly sized heap buffer: any read past the end is a sanitizer error
    uint8_t* heap = (uint8_t*)malloc(dg.size() ? dg.size() : 1);
    if (!dg.empty()) memcpy(heap, dg.data(), dg.size());
    decode_all(heap, dg.size());
    free(heap);
  }
  printf("fuzz: %ld datagrams, %d failures\n", n, fails);
  return fails != 0;
}

static int decode_stdin() {
  long count = 0;
  for (;;) {
    uint8_t h[4];
    if (fread(h, 1, 4, stdin) != 4) break;
    const uint32_t len = (uint32_t)h[0] | (uint32_t)h[1] << 8 | (uint32_t)h[2] << 16 | (uint32_t)h[3] << 24;
    uint8_t* dg = (uint8_t*)malloc(len ? len : 1);
    if (len && fread(dg, 1, len, stdin) != len) { free(dg); fprintf(stderr, "short input\n"); return 2; }
    decode_all(dg, len);
    free(dg);
    ++count;
  }
  printf("decode: %ld datagrams, %d failures\n", count, fails);
  return fails != 0;
}

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s scenarios | decode | fuzz N\n", argv[0]); return 2; }
  if (!strcmp(argv[1], "scenarios")) return scenarios();
  if (!strcmp(argv[1], "decode")) return decode_stdin();
  if (!strcmp(argv[1], "fuzz")) return fuzz(argc > 2 ? atol(argv[2]) : 100000);
  return 2;
}
