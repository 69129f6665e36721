"""Per-round message volume of the benched workload, and the collective volume of a row-sharded mesh
(DESIGN.md §6), from the CPU oracle's counters (kb_stats):

  messages of each unicast kind per round (Ping, PingRequest, Ack, KnownPeers, KnownPeersRequest), the
  KnownPeers ids they carry, and the Join/Failed broadcast entries, averaged over rounds [warm, warm+k) of
  configs[2] at the given peer counts (converged start, 1% loss, 0.1%/round churn, sim_sender).

A sharded round moves, per delivery wave, the records whose destination row lives on another rank (32 B
each, plus 4 B per KnownPeers id), and once per round the broadcast lists (all-gather of 16 B entries).
With destinations uniform over ranks, (world-1)/world of the records cross ranks.

    python tools/round_volume.py [peers ...] [--out profiles/r03_round_volume.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import parity  # noqa: E402
from kaboodle_amd._ffi import KB_INIT_CONVERGED, Sim, SimConfig  # noqa: E402

KINDS = ("sent_ping", "sent_ping_req", "sent_ack", "sent_known_peers", "sent_kpr")
REC, ID, BREC = 32, 4, 16


def measure(peers, warm, k, seed=1):
    cfg = SimConfig(capacity=peers + max(1024, peers // 8), initial_nodes=peers, init_mode=KB_INIT_CONVERGED,
                    loss=0.01, churn=0.001, fault_end_round=warm + k + 1, seed=seed)
    with Sim(parity.oracle_lib(omp=True), cfg) as o:
        o.step(warm)
        s0 = o.stats()
        t0 = time.time()
        o.step(k)
        s1 = o.stats()
        dt = time.time() - t0
    per = {n: (s1[n] - s0[n]) / k for n in KINDS + ("sent_kp_ids", "bcast_join", "bcast_failed", "join_responses",
                                                   "removed_failed", "drop_loss", "drop_dead", "drop_window")}
    per["records"] = sum(per[n] for n in KINDS)
    per["record_bytes"] = REC * per["records"] + ID * per["sent_kp_ids"]
    per["bcast_entries"] = per["bcast_join"] + per["bcast_failed"]
    return {"peers": peers, "rounds": [warm, warm + k], "oracle_s": round(dt, 1), "per_round": per}


def sharded_volume(m, world):
    """bytes per round a row-sharded mesh of `world` ranks moves between ranks (whole node / per rank)"""
    p = m["per_round"]
    x = p["record_bytes"] * (world - 1) / world
    g = BREC * p["bcast_entries"] * (world - 1)          # each rank receives every other rank's entries
    return {"world": world, "records_cross_bytes": int(x), "bcast_allgather_bytes_per_rank": int(g),
            "per_rank_in_bytes": int(x / world + g)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("peers", nargs="*", type=int, default=[8192, 16384, 32768, 65536])
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_round_volume.json"))
    a = ap.parse_args()
    rows = []
    for n in a.peers:
        m = measure(n, a.warm, a.rounds)
        m["sharded"] = [sharded_volume(m, w) for w in (2, 4, 8)]
        rows.append(m)
        p = m["per_round"]
        print(f"{n:8d} peers: records {p['records']:.0f}/round ({p['records'] / n:.2f}/peer), KP ids "
              f"{p['sent_kp_ids']:.0f}, bcast Join {p['bcast_join']:.0f} Failed {p['bcast_failed']:.0f}, "
              f"{p['record_bytes'] / 1e6:.1f} MB of records ({m['oracle_s']} s)", flush=True)
    json.dump({"tool": "tools/round_volume.py", "workload": "configs[2] shape: converged start, 1% loss, "
               "0.1%/round churn, sim_sender", "rows": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
