// kaboodle_sim.hpp — thin header-only C++ wrapper over the C ABI (include/kaboodle_sim.h) with the
// shape of the reference's `Kaboodle` surface (src/lib.rs:65-369): a `Mesh` owns one simulated mesh
// on one GPU, `Mesh::Peer` is the per-instance view (start/stop/ping_addrs/fingerprint/peers/...).
// Errors become `kb::Error` (status code + kb_last_error text), mirroring KaboodleError
// (src/errors.rs:8-24).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "kaboodle_sim.h"

namespace kb {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char* fn) {
  if (rc != KB_OK) {
    const char* e = kb_last_error();
    throw Error(rc, std::string(fn) + ": " + (e ? e : ""));
  }
}

inline std::string format_addr(uint32_t id) {                 // canonical simulated SocketAddr
  char buf[32];
  check(kb_format_addr(id, buf, sizeof buf), "kb_format_addr");
  return buf;
}

class Mesh {
 public:
  explicit Mesh(const kb_config& cfg) { check(kb_sim_create(&cfg, &h_), "kb_sim_create"); }
  static kb_config defaults() { kb_config c; kb_config_default(&c); return c; }
  ~Mesh() { if (h_) kb_sim_destroy(h_); }
  Mesh(const Mesh&) = delete;
  Mesh& operator=(const Mesh&) = delete;
  Mesh(Mesh&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}

  void step(uint32_t rounds = 1) { check(kb_sim_step(h_, rounds), "kb_sim_step"); }
  kb_stats stats() const { kb_stats s; check(kb_sim_stats(h_, &s), "kb_sim_stats"); return s; }
  uint32_t true_fingerprint() const { uint32_t f; check(kb_sim_true_fingerprint(h_, &f), "kb_sim_true_fingerprint"); return f; }
  kb_sim* handle() const { return h_; }

  // the per-instance view: method names of src/lib.rs
  class Peer {
   public:
    Peer(kb_sim* h, uint32_t id) : h_(h), id_(id) {}
    // :136 — a stopped peer comes back at a fresh address (src/kaboodle.rs:138-152) with its map
    void start() { check(kb_sim_restart_node(h_, id_, &id_), "kb_sim_restart_node"); }
    void stop() { check(kb_sim_stop_node(h_, id_), "kb_sim_stop_node"); }               // :159
    bool is_running() const { int r; check(kb_sim_is_running(h_, id_, &r), "kb_sim_is_running"); return r != 0; }
    std::string self_addr() const { return format_addr(id_); }                          // :312
    void ping_addrs(const std::vector<uint32_t>& ids) {                                 // :268
      check(kb_sim_ping_addrs(h_, id_, ids.data(), ids.size()), "kb_sim_ping_addrs");
    }
    void set_identity(const std::vector<uint8_t>& ident) {                              // :323
      check(kb_sim_set_identity(h_, id_, ident.data(), ident.size()), "kb_sim_set_identity");
    }
    uint32_t fingerprint() const { uint32_t f; check(kb_sim_fingerprint(h_, id_, &f), "kb_sim_fingerprint"); return f; }
    std::vector<uint32_t> peers() const {                                               // :339 (ids)
      size_t n = 0;
      check(kb_sim_peers(h_, id_, nullptr, 0, &n), "kb_sim_peers");
      std::vector<uint32_t> v(n);
      check(kb_sim_peers(h_, id_, v.data(), v.size(), &n), "kb_sim_peers");
      v.resize(n);
      return v;
    }
    // Kaboodle::peers as the reference returns it (:339-345): address -> identity bytes
    std::vector<std::pair<std::string, std::vector<uint8_t>>> peers_with_identity() const {
      std::vector<std::pair<std::string, std::vector<uint8_t>>> out;
      for (uint32_t p : peers()) out.emplace_back(format_addr(p), identity_of(h_, p));
      return out;
    }
    std::vector<uint8_t> identity() const { return identity_of(h_, id_); }
    std::vector<kb_peer_state> peer_states() const {                                   // :348
      size_t n = 0;
      check(kb_sim_peer_states(h_, id_, nullptr, 0, &n), "kb_sim_peer_states");
      std::vector<kb_peer_state> v(n);
      check(kb_sim_peer_states(h_, id_, v.data(), v.size(), &n), "kb_sim_peer_states");
      v.resize(n);
      return v;
    }
    // events.rs:18-125 behind discover_peers / discover_departures / discover_fingerprint_changes
    // (:186-263): watch() once, then events() after each step drains one batch
    struct Events { std::vector<uint32_t> discovered, departed; bool fingerprint_changed; uint32_t fingerprint; };
    void watch() { check(kb_sim_watch(h_, id_), "kb_sim_watch"); }
    Events events() {
      Events e;
      size_t nd = 0, np = 0;
      int ch = 0;
      check(kb_sim_events(h_, id_, nullptr, 0, &nd, nullptr, 0, &np, &e.fingerprint, &ch), "kb_sim_events");
      e.discovered.resize(nd);
      e.departed.resize(np);
      check(kb_sim_events(h_, id_, e.discovered.data(), nd, &nd, e.departed.data(), np, &np, &e.fingerprint, &ch),
            "kb_sim_events");
      e.fingerprint_changed = ch != 0;
      return e;
    }
   private:
    static std::vector<uint8_t> identity_of(kb_sim* h, uint32_t id) {
      uint8_t buf[32];
      size_t len = 0;
      check(kb_sim_identity(h, id, buf, sizeof buf, &len), "kb_sim_identity");
      return std::vector<uint8_t>(buf, buf + len);
    }
    kb_sim* h_;
    uint32_t id_;
  };
  Peer peer(uint32_t id) const { return Peer(h_, id); }

  // real instances in the mesh: an external peer's records out, its datagrams in
  struct Record { kb_unicast rec; std::vector<uint32_t> ids; };
  void set_external(uint32_t id) { check(kb_sim_set_external(h_, id), "kb_sim_set_external"); }
  void inject(const kb_unicast& rec, const std::vector<uint32_t>& ids = {}) {
    kb_unicast m = rec;
    m.pay_len = (uint32_t)ids.size();
    check(kb_sim_inject(h_, &m, ids.empty() ? nullptr : ids.data()), "kb_sim_inject");
  }
  std::vector<Record> exported() {                    // drains: (round, wave, sender, seq) order
    size_t n = 0, ni = 0;
    check(kb_sim_exported(h_, nullptr, 0, &n, nullptr, 0, &ni), "kb_sim_exported");
    std::vector<kb_unicast> v(n);
    std::vector<uint32_t> ids(ni);
    check(kb_sim_exported(h_, v.data(), v.size(), &n, ids.data(), ids.size(), &ni), "kb_sim_exported");
    std::vector<Record> out;
    for (size_t k = 0; k < n; ++k)
      out.push_back({v[k], std::vector<uint32_t>(ids.begin() + v[k].pay_off, ids.begin() + v[k].pay_off + v[k].pay_len)});
    return out;
  }

 private:
  kb_sim* h_ = nullptr;
};

}  // namespace kb
