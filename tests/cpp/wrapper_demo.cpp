// Exercises include/kaboodle_sim.hpp: pure helpers always; with a GPU, the config-1 2x2 mesh
// (2x2-layout.kdl identities) stepped until every peer reports the golden fingerprint 0x981285c8.
#include "kaboodle_sim.hpp"
#include <cstdio>
#include <cstring>

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && !strcmp(argv[1], "--gpu");
  printf("addr %s\n", kb::format_addr(50001).c_str());
  uint32_t ids[4] = {3, 1, 2, 0};
  printf("fp %08x\n", kb_fingerprint_of_set(ids, 4, nullptr, 0, nullptr));
  kb_config c = kb::Mesh::defaults();
  c.capacity = 4;
  c.initial_nodes = 0;
  try {
    kb::Mesh m(c);
    const char* names[4] = {"top-left", "top-right", "bottom-left", "bottom-right"};
    for (uint32_t i = 0; i < 4; ++i) {
      auto p = m.peer(i);
      p.set_identity(std::vector<uint8_t>(names[i], names[i] + strlen(names[i])));
      p.start();
    }
    m.peer(0).watch();
    m.step(6);
    auto ev = m.peer(0).events();                 // first batch: all four discovered (events.rs:59-79)
    printf("events 0: disc %zu dep %zu changed %d fp %08x\n", ev.discovered.size(), ev.departed.size(),
           (int)ev.fingerprint_changed, ev.fingerprint);
    for (uint32_t i = 0; i < 4; ++i) printf("peer %u fp %08x n %zu\n", i, m.peer(i).fingerprint(), m.peer(i).peers().size());
    // an external peer (a real instance behind a bridge): its Ping in, the Ack out
    kb_config c2 = kb::Mesh::defaults();
    c2.capacity = 8; c2.initial_nodes = 4; c2.init_mode = KB_INIT_CONVERGED;
    kb::Mesh x(c2);
    x.set_external(6);
    x.step(1);
    kb_unicast ping{};
    ping.sender = 6; ping.dest = 1; ping.kind = KB_WIRE_PING;
    x.inject(ping);
    x.step(1);
    size_t acks = 0;
    for (const auto& r : x.exported()) acks += r.rec.dest == 6 && r.rec.sender == 1 && r.rec.kind == KB_WIRE_ACK;
    printf("external acks %zu\n", acks);
    printf("mesh ok\n");
  } catch (const kb::Error& e) {
    printf("error %d %s\n", e.code, e.what());
    return gpu ? 1 : (e.code == KB_NO_DEVICE ? 0 : 1);
  }
  return 0;
}
