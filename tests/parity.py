"""Parity harness: drive the HIP library and the CPU oracle through identical ABI calls and compare the
complete simulator state (stamp rows, per-node scalars, suspect and curious tables, fingerprints,
counters) after every round.  Used by tests/test_gpu_parity.py and runnable as a script on the GPU box:

    python tests/parity.py            # the standard matrix, prints one line per case
"""
from __future__ import annotations

import os
import sys
from dataclasses import replace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kaboodle_amd._ffi import (KB_INIT_CONVERGED, KB_INIT_JOIN, KB_FAILED_SOCKET_FAITHFUL,  # noqa: E402
                               Sim, SimConfig, SimLib)

ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libkb_oracle.so")
ORACLE_OMP_SO = os.path.join(ROOT, "oracle", "_build", "libkb_oracle_omp.so")
GPU_SO = os.path.join(ROOT, "kaboodle_amd", "libkaboodle_sim.so")

CONFIG1_IDS = [b"top-left", b"top-right", b"bottom-left", b"bottom-right"]   # 2x2-layout.kdl:6-20


def oracle_lib(omp: bool = False) -> SimLib:
    return SimLib(ORACLE_OMP_SO if omp else ORACLE_SO, "kbo_")


def gpu_lib() -> SimLib:
    return SimLib(GPU_SO, "kb_")


def state_of(sim: Sim, full_rows: bool = True) -> dict:
    st = {"stats": sim.stats(), "scalars": sim.scalars(), "fps": sim.fingerprints(),
          "truefp": sim.true_fingerprint()}
    C = sim.capacity
    if full_rows:
        st["rows"] = sim.rows()
    st["susp"] = [sim.suspects(i) for i in range(C)]
    st["cur"] = [sim.curious(i) for i in range(C)]
    st["probe"] = sim.probe_responses()          # drained: the round's ProbeResponses
    st["bcasts"] = sim.broadcasts()              # the broadcast lists the next round delivers
    return st


def diff_states(a: dict, b: dict) -> list[str]:
    out = []
    for k in ("stats",):
        for f, v in a[k].items():
            if b[k][f] != v:
                out.append(f"stats.{f}: {v} != {b[k][f]}")
    if a["truefp"] != b["truefp"]:
        out.append(f"truefp {a['truefp']:#x} != {b['truefp']:#x}")
    for k in ("scalars", "fps"):
        if not np.array_equal(a[k], b[k]):
            bad = np.argwhere(a[k] != b[k])
            out.append(f"{k}: {len(bad)} mismatches, first {bad[:4].tolist()}")
    if "rows" in a and "rows" in b and not np.array_equal(a["rows"], b["rows"]):
        bad = np.argwhere(a["rows"] != b["rows"])
        i, j = bad[0]
        out.append(f"rows: {len(bad)} mismatches, first node {i} peer {j}: {a['rows'][i, j]} != {b['rows'][i, j]}")
    for k in ("susp", "cur"):
        for i, (x, y) in enumerate(zip(a[k], b[k])):
            if x != y:
                out.append(f"{k}[{i}]: {x} != {y}")
                break
    for k in ("probe", "bcasts"):
        if k in a and k in b and a[k] != b[k]:
            out.append(f"{k}: {len(a[k])} vs {len(b[k])} entries, first {a[k][:2]} vs {b[k][:2]}")
    return out


def setup(sim: Sim, case: dict) -> None:
    for i, ident in case.get("identities", {}).items():
        sim.set_identity(i, ident)
    for i in case.get("start", []):
        sim.start_node(i)


def diff_peer_states(o: Sim, g: Sim, nodes) -> list[str]:
    """Kaboodle::peer_states (src/lib.rs:348-354) of `nodes` on both implementations: (peer, state,
    since round, latency) for every entry; it must also list exactly the ids peers() reports."""
    out = []
    for i in nodes:
        a, b = o.peer_states_array(int(i)), g.peer_states_array(int(i))
        if a.tobytes() != b.tobytes():              # the arrays carry the bytes past identity_len too: decide on tuples
            a, b = o.peer_states(int(i)), g.peer_states(int(i))
            if a != b:
                bad = [(x, y) for x, y in zip(a, b) if x != y][:2]
                out.append(f"peer_states[{i}]: {len(a)} vs {len(b)} entries, first differing {bad}")
                break
            b = g.peer_states_array(int(i))
        if not np.array_equal(b["peer"], np.asarray(g.peers(int(i)), dtype=np.uint32)):
            out.append(f"peer_states[{i}] ids != peers()")
            break
    return out


def with_cfg(case: dict, **kw) -> dict:
    """The case with config fields replaced (e.g. debug_flags=KB_DBG_ALL)."""
    return {**case, "cfg": replace(case["cfg"], **kw)}


def run_case(case: dict, rounds: int, check_every: int = 1, full_rows: bool = True, verbose: bool = False,
             shards: int = 0, gpu: Sim | None = None, peer_states: bool = False):
    """Run `case` on both implementations; returns (ok, message, final gpu stats).  shards=k runs the
    GPU mesh as k row shards exchanging every wave (kb_sim_create_local); `gpu` = an already created
    GPU handle for the case (e.g. an RCCL rank); peer_states: also compare peer_states() of every node."""
    cfg = case["cfg"]
    o = Sim(oracle_lib(), cfg)
    g = gpu if gpu is not None else Sim(gpu_lib(), cfg, shards=shards)
    setup(o, case)
    setup(g, case)
    for r in range(rounds):
        apply_events((o, g), case, r)
        o.step(1)
        g.step(1)
        if (r + 1) % check_every == 0 or r == rounds - 1:
            d = diff_states(state_of(o, full_rows), state_of(g, full_rows))
            if not d and peer_states:
                d = diff_peer_states(o, g, range(cfg.capacity))
            if d:
                return False, f"round {r}: " + "; ".join(d[:6]), g.stats()
            if verbose:
                st = g.stats()
                print(f"  round {r}: agree {st['agree']}/{st['alive']} ok", flush=True)
    return True, "ok", g.stats()


def compare_sampled(o: Sim, g: Sim, rng, nrows: int = 24) -> list[str]:
    """Full-size comparison after a round: counters, every fingerprint and per-node scalar, and for a
    random sample of nodes the whole stamp row, suspect/curious tables and peer_states."""
    out = []
    so, sg = o.stats(), g.stats()
    out += [f"stats.{k}: {v} != {sg[k]}" for k, v in so.items() if sg[k] != v]
    fo, fg = o.fingerprints(), g.fingerprints()
    if not np.array_equal(fo, fg):
        out.append(f"fingerprints: {int((fo != fg).sum())} differ, first {np.argwhere(fo != fg)[:3].ravel().tolist()}")
    if not np.array_equal(o.scalars(), g.scalars()):
        out.append("scalars differ")
    for i in rng.choice(o.capacity, nrows, replace=False):
        i = int(i)
        if not np.array_equal(o.row(i), g.row(i)):
            out.append(f"row {i} differs")
        if o.suspects(i) != g.suspects(i) or o.curious(i) != g.curious(i):
            out.append(f"suspect/curious table {i} differs")
        out += diff_peer_states(o, g, [i])
        if out:
            break
    return out


def apply_events(sims, case: dict, r: int) -> dict:
    """The case's API calls of round r on every implementation; returns {old address: new address} of
    the restarts (each implementation must allocate the same fresh id)."""
    moved = {}
    for kind, node, arg in case.get("events", {}).get(r, []):
        got = set()
        for s in sims:
            if kind == "stop":
                s.stop_node(node)
            elif kind == "start":
                s.start_node(node)
            elif kind == "restart":
                got.add(s.restart_node(node))
            elif kind == "ident":
                s.set_identity(node, arg)
            elif kind == "probe":
                s.probe(arg)
            elif kind == "ping":
                s.ping_addrs(node, arg)
        if kind == "restart":
            assert len(got) == 1, f"restart of {node}: implementations allocated {got}"
            moved[node] = got.pop()
    return moved


def run_events_case(case: dict, rounds: int, watched, drain_every: int = 1, shards: int = 0,
                    libs=None, gpu: Sim | None = None):
    """Event streams (src/events.rs:18-125) on both implementations: every node in `watched` is
    observed from creation and drained every `drain_every` rounds.  Each batch must be identical
    across implementations and equal to the net diff of the oracle's peer lists.  libs = (oracle,
    other) SimLibs; default (oracle, HIP library); `gpu` = an already created handle (e.g. an RCCL
    rank).  Returns (ok, message, batches compared)."""
    cfg = case["cfg"]
    la, lb = libs if libs is not None else (oracle_lib(), gpu_lib())
    o = Sim(la, cfg)
    g = gpu if gpu is not None else Sim(lb, cfg, shards=shards)
    for s in (o, g):
        for i in watched:
            s.watch(i)
    setup(o, case)
    setup(g, case)
    prev = {i: set() for i in watched}
    last_fp = {i: 0 for i in watched}
    n = 0
    watched = list(watched)
    for r in range(rounds):
        for a, b in apply_events((o, g), case, r).items():     # the observer follows the instance
            if a in watched:
                watched[watched.index(a)] = b
                prev[b], last_fp[b] = prev.pop(a), last_fp.pop(a)
        o.step(1)
        g.step(1)
        if (r + 1) % drain_every and r != rounds - 1:
            continue
        for i in watched:
            eo, eg = o.events(i), g.events(i)
            if eo != eg:
                return False, f"round {r} node {i}: oracle {eo[:2]} fp {eo[2]:#x}/{eo[3]} != {eg[:2]} fp {eg[2]:#x}/{eg[3]}", n
            now = set(o.peers(i))
            want_d, want_p = sorted(now - prev[i]), sorted(prev[i] - now)
            want_ch = bool(now) and eo[2] != last_fp[i]
            if (eo[0], eo[1], eo[3]) != (want_d, want_p, want_ch):
                return False, f"round {r} node {i}: events {eo} != peer-list diff {want_d} {want_p} {want_ch}", n
            if want_ch:
                last_fp[i] = eo[2]
            prev[i] = now
            n += 1
    return True, "ok", n


K_PING, K_PINGREQ, K_ACK, K_KP, K_KPR = range(5)
K_JOIN = 16                              # KB_WIRE_JOIN: an external peer's Join broadcast


def external_replies(exported, me_known, r: int, proactive_to=None):
    """What a real instance at an external address sends back into the mesh for the records it received
    (src/kaboodle.rs:394-548, a scripted stand-in for a real instance): Ping -> Ack{self, fp, n};
    PingRequest(p) -> Ping p; KnownPeersRequest -> KnownPeers of the peers it knows; Ack / KnownPeers learn
    their senders; every 10th round (from round 1) each external peer broadcasts Join, as maybe_broadcast_join
    re-broadcasts (src/kaboodle.rs:228-251).  Returns [(sender, dest, kind, a, fp, n, ids)] in order, at most 33
    unicast records per external peer."""
    out = []
    for (_, _, sender, dest, _, kind, a, fp, n, ids) in exported:
        me_known.setdefault(dest, set()).add(sender)
        if kind == K_PING:
            out.append((dest, sender, K_ACK, dest, 0xC0FFEE00 + dest, len(me_known[dest]) + 1, []))
        elif kind == K_PINGREQ:
            out.append((dest, a, K_PING, 0, 0, 0, []))
        elif kind == K_KPR:
            out.append((dest, sender, K_KP, 0, 0, 0, sorted(me_known[dest] - {sender})[:40]))
        elif kind == K_KP:
            me_known[dest].update(ids)
    if proactive_to is not None:
        for x, targets in proactive_to.items():
            t = targets[r % len(targets)]
            out.append((x, t, K_PING, 0, 0, 0, []))
            if r % 5 == 2:
                out.append((x, t, K_KPR, 0, 0xBADF00D, 1, []))
    per = {}
    kept = []
    for m in out:
        per[m[0]] = per.get(m[0], 0) + 1
        if per[m[0]] <= 33:
            kept.append(m)
    if proactive_to is not None and r % 10 == 1:
        kept += [(x, 0, K_JOIN, 0, 0, 0, []) for x in proactive_to]
    return kept


def run_external_case(case: dict, rounds: int, externals, libs, shards: int = 0) -> tuple[bool, str, int]:
    """The case with external peers (kb_sim_set_external) answered by external_replies: every implementation
    gets the same injections (they depend only on the exports, which must be identical) and must keep the same
    complete state every round.  Returns (ok, message, exported records compared)."""
    cfg = case["cfg"]
    sims = [Sim(libs[0], cfg)] + [Sim(lb, cfg, shards=shards) for lb in libs[1:]]
    for sm in sims:
        setup(sm, case)
        for x in externals:
            sm.set_external(x)
    known = [dict() for _ in sims]
    targets = {x: [(x * 7 + k * 13) % cfg.initial_nodes for k in range(5)] for x in externals}
    nx = 0
    for r in range(rounds):
        apply_events(sims, case, r)
        for sm in sims:
            sm.step(1)
        ex = [sm.exported() for sm in sims]
        for e in ex[1:]:
            if e != ex[0]:
                return False, f"round {r}: exports differ: {ex[0][:3]} vs {e[:3]}", nx
        nx += len(ex[0])
        st = [state_of(sm) for sm in sims]
        for k in range(1, len(sims)):
            d = diff_states(st[0], st[k])
            if d:
                return False, f"round {r}: " + "; ".join(d[:6]), nx
        for k, sm in enumerate(sims):
            for m in external_replies(ex[k], known[k], r, targets):
                sm.inject(*m[:6], ids=m[6])
    for sm in sims:
        sm.close()
    return True, "ok", nx


def standard_cases() -> list[tuple[str, dict, int]]:
    cases = []
    cases.append(("config1_2x2", {"cfg": SimConfig(capacity=4, initial_nodes=0),
                                  "identities": {i: n for i, n in enumerate(CONFIG1_IDS)},
                                  "start": [0, 1, 2, 3]}, 6))
    cases.append(("join_64", {"cfg": SimConfig(capacity=64, initial_nodes=64)}, 8))
    cases.append(("config2_join_1k", {"cfg": SimConfig(capacity=1024, initial_nodes=1024)}, 6))
    cases.append(("converged_loss_256", {"cfg": SimConfig(capacity=256, initial_nodes=256, init_mode=KB_INIT_CONVERGED,
                                                          loss=0.05, seed=7)}, 30))
    cases.append(("churn_loss_512", {"cfg": SimConfig(capacity=640, initial_nodes=512, init_mode=KB_INIT_CONVERGED,
                                                      loss=0.01, churn=0.01, fault_end_round=25, seed=3)}, 40))
    cases.append(("join_loss_300_ids", {"cfg": SimConfig(capacity=300, initial_nodes=300, loss=0.02, id_len=5,
                                                         seed=11)}, 20))
    cases.append(("socket_faithful", {"cfg": SimConfig(capacity=200, initial_nodes=200, init_mode=KB_INIT_CONVERGED,
                                                       loss=0.05, failed_mode=KB_FAILED_SOCKET_FAITHFUL, seed=5)}, 20))
    cases.append(("partition_heal", {"cfg": SimConfig(capacity=256, initial_nodes=256, init_mode=KB_INIT_CONVERGED,
                                                      loss=0.02, partition_groups=2, partition_start=3,
                                                      partition_end=12, seed=9),
                                     "events": {12: [("ping", i, [(i + 128) % 256]) for i in range(0, 256, 16)]}}, 30))
    cases.append(("stop_start", {"cfg": SimConfig(capacity=128, initial_nodes=100, init_mode=KB_INIT_CONVERGED,
                                                  seed=2),
                                 "events": {2: [("stop", 5, None), ("stop", 17, None)], 4: [("start", 120, None)],
                                            9: [("restart", 5, None)], 12: [("stop", 100, None)],
                                            14: [("restart", 100, None), ("restart", 17, None)]}}, 20))
    cases.append(("rebase_window", {"cfg": SimConfig(capacity=192, initial_nodes=192, init_mode=KB_INIT_CONVERGED,
                                                     loss=0.01, churn=0.002, seed=4)}, 140))
    cases.append(("waves_2", {"cfg": SimConfig(capacity=256, initial_nodes=256, loss=0.03, max_waves=2, seed=13)}, 15))
    # 200 peers ping_addrs the same peer before their first tick: one in-order inbox of 200 Pings in
    # wave 0 (k_sort_inbox + k_proc's sorted path; with KB_DBG_PROC_UNSORTED the selection path)
    cases.append(("hot_inbox", {"cfg": SimConfig(capacity=256, initial_nodes=256, loss=0.02, seed=17),
                                "events": {0: [("ping", i, [0]) for i in range(1, 201)]}}, 8))
    # Kaboodle::set_identity on stopped peers (src/lib.rs:323-336), uniform and non-uniform lengths, restarted
    cases.append(("identity_change", {"cfg": SimConfig(capacity=160, initial_nodes=150, init_mode=KB_INIT_CONVERGED,
                                                       loss=0.02, id_len=6, seed=23),
                                      "events": {2: [("stop", 9, None), ("stop", 70, None)],
                                                 3: [("ident", 9, b"qwerty"), ("ident", 70, b"short"),
                                                     ("restart", 9, None)],
                                                 5: [("ident", 155, b"fresh-peer-id"), ("start", 155, None),
                                                     ("restart", 70, None)]}}, 16))
    # SwimBroadcast::Probe from outside the mesh (src/discovery.rs:30-89): ProbeResponses of the peers that
    # should_respond, in a small mesh (everyone answers: n <= 2) and a lossy converged one (about 1 %)
    cases.append(("probes", {"cfg": SimConfig(capacity=400, initial_nodes=396, init_mode=KB_INIT_CONVERGED, loss=0.03,
                                              churn=0.01, fault_end_round=8, seed=29),
                             "events": {1: [("probe", 0, ("192.0.2.10", 41000))],
                                        3: [("probe", 0, ("192.0.2.10", 41000)), ("probe", 0, ("198.51.100.3", 5000))],
                                        6: [("probe", 0, ("192.0.2.11", 41001))] * 3}}, 10))
    cases.append(("probe_tiny", {"cfg": SimConfig(capacity=4, initial_nodes=2, seed=2),
                                 "events": {0: [("probe", 0, ("192.0.2.1", 9000))], 2: [("probe", 0, ("192.0.2.1", 9000))],
                                            3: [("start", 3, None)], 5: [("probe", 0, ("192.0.2.2", 9001))]}}, 8))
    # fresh ids: churn joins and restarts skip an address the API already bound (49, started) or
    # gave an identity (51), so no two instances ever share an address
    cases.append(("fresh_ids", {"cfg": SimConfig(capacity=64, initial_nodes=48, init_mode=KB_INIT_CONVERGED, loss=0.02,
                                                 churn=0.02, fault_end_round=24, seed=12),
                                "events": {1: [("start", 49, None), ("ident", 51, b"x")], 3: [("stop", 7, None)],
                                           5: [("restart", 7, None)], 6: [("stop", 20, None)], 9: [("restart", 20, None)]}},
                  28))
    # stamps from before round 0 (early joiners' KnownPeers inserts) crossing three window rebases
    cases.append(("old_stamps", {"cfg": SimConfig(capacity=160, initial_nodes=128, init_mode=KB_INIT_CONVERGED, loss=0.02,
                                                  churn=0.03, fault_end_round=12, seed=31)}, 200))
    return cases


def main() -> int:
    fails = 0
    only = sys.argv[1:]
    for name, case, rounds in standard_cases():
        if only and name not in only:
            continue
        ok, msg, st = run_case(case, rounds)
        print(f"{'PASS' if ok else 'FAIL'} {name:24s} rounds={rounds:4d} {msg} "
              f"(agree {st['agree']}/{st['alive']}, sent ping {st['sent_ping']} kpr {st['sent_kpr']} "
              f"kp {st['sent_known_peers']} removed {st['removed_timeout']}+{st['removed_failed']})", flush=True)
        fails += not ok
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
