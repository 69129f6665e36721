"""configs[4] on one MI355X: the partition + heal scenario (converged start, 5 % loss, two halves cut
off for rounds 3-11, healed at round 12 by every 256th peer pinging the other half, socket_faithful) on the GPU's
sparse rows (KB_VARIANT_SPARSE_ROWS) at 4,194,304 peers, with per-round time, agreement, the layout's footprint,
the kernel breakdown and the property checks of tests/test_gpu_sparse_big.py on sampled rows.

    python tools/sparse_big.py --nodes 4194304 --rounds 24 --out profiles/r05_sparse_4m.json

Reconvergence after the heal: --fault-end R ends the loss at round R, --until-converged runs until every live
view's fingerprint equals the true set's (or --rounds / --budget-s).

The Failed lists' lost deliveries are not counted by default (KB_STAT_NO_SF_FAILED_DROPS): in socket_faithful mode
a Failed broadcast changes no state, so the count is a statistic only, and at 4M it is one Philox
word per (receiver, entry), ≈ 10^12 a round, 96 % of the round.  --count-sf-failed-drops counts them (the
scenario's drop_bcast exactly as the oracle counts it; the kernel is VALU-bound).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def scenario(n: int, every: int = 256, seed: int = 9, row_cap: int = 2048, rounds_part=(3, 12), fault_end: int = -1,
             stat_flags: int = 0):
    from kaboodle_amd._ffi import KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_VARIANT_SPARSE_ROWS, SimConfig
    a, b = rounds_part
    cfg = SimConfig(capacity=n, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.05, partition_groups=2,
                    partition_start=a, partition_end=b, seed=seed, failed_mode=KB_FAILED_SOCKET_FAITHFUL,
                    variant=KB_VARIANT_SPARSE_ROWS, sparse_row_cap=row_cap, fault_end_round=fault_end,
                    stat_flags=stat_flags)
    return {"cfg": cfg, "events": {b: [("ping", i, [(i + n // 2) % n]) for i in range(0, n, every)]}}


def fp_of_peers(sim, lib, i: int) -> tuple[int, int]:
    """(the row's fingerprint, generate_fingerprint of its peers() list computed from scratch)"""
    import ctypes as C
    ids = np.asarray(sim.peers(i), dtype=np.uint32)
    f = lib.lib.kb_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    want = f(ids.ctypes.data_as(C.POINTER(C.c_uint32)), len(ids), None, 0, None)   # empty identities (id_len 0)
    return sim.fingerprint(i), int(want)


def check_invariants(st: dict, n: int, rounds: int) -> list[str]:
    out = []
    if st["alive"] != n:
        out.append(f"alive {st['alive']} != {n}")
    if st["alive_rounds"] != n * rounds:
        out.append(f"alive_rounds {st['alive_rounds']} != {n * rounds}")
    if st["bcast_failed"] != st["removed_timeout"]:
        out.append(f"every A2 removal is one Failed broadcast: {st['bcast_failed']} != {st['removed_timeout']}")
    if st["removed_failed"] or st["drop_dead"] or st["churn_joins"] or st["bcast_join"]:
        out.append("socket_faithful, no churn: no Failed honoured, no dead receivers, no joins")
    return out


def run(n: int, rounds: int, every: int, row_cap: int, check_rows: int, seed: int = 9, verbose: bool = True,
        fault_end: int = -1, stat_flags: int = 0, until_converged: bool = False, budget_s: float = 0.0,
        print_every: int = 1, fp_every: int = 4) -> dict:
    import kaboodle_amd
    import parity
    from kaboodle_amd._ffi import Sim
    lib = kaboodle_amd.lib()                                  # honours KB_LIB_PATH (A/B builds)
    case = scenario(n, every, seed, row_cap, fault_end=fault_end, stat_flags=stat_flags)
    t0 = time.time()
    g = Sim(lib, case["cfg"])
    t_create = time.time() - t0
    g.set_profiling(1)
    rng = np.random.default_rng(seed)
    traj, prev = [], g.stats()
    all_ms = []                                              # every round's time (traj keeps every print_every-th)
    fails = []
    heal = case["cfg"].partition_end
    converged_round, stopped_by, t_start = None, "rounds", time.time()
    for r in range(rounds):
        parity.apply_events((g,), case, r)
        t = time.time()
        g.step(1)
        dt = time.time() - t
        all_ms.append(dt * 1e3)
        st = g.stats()
        rec = {"round": r, "ms": round(dt * 1e3, 1), "agree": st["agree"],
               "failed_bcasts": st["bcast_failed"] - prev["bcast_failed"],
               "drop_bcast": st["drop_bcast"] - prev["drop_bcast"], "drop_partition": st["drop_partition"] - prev["drop_partition"],
               "sent": sum(st[k] - prev[k] for k in ("sent_ping", "sent_ping_req", "sent_ack", "sent_known_peers", "sent_kpr")),
               "kpr": st["sent_kpr"] - prev["sent_kpr"], "oversize": st["drop_oversize"] - prev["drop_oversize"]}
        done = until_converged and r >= heal and st["agree"] == st["alive"]
        if done:
            converged_round, stopped_by = r, "converged"
        if budget_s and time.time() - t_start > budget_s and not done:
            stopped_by = "budget"
        last = done or stopped_by == "budget" or r == rounds - 1
        if r % fp_every == fp_every - 1 or last:
            fp = g.sparse_footprint()
            rec.update({"entries": fp["exceptions"] + fp["stamps"],
                        "exceptions_per_row": round(fp["exceptions"] / n, 3), "stamps_per_row": round(fp["stamps"] / n, 2),
                        "max_row_entries": fp["max_row_entries"], "bytes_per_row": round(fp["bytes"] / n, 1)})
            for i in rng.choice(n, check_rows, replace=False):
                got, want = fp_of_peers(g, lib, int(i))
                if got != want:
                    fails.append(f"round {r} row {i}: fingerprint {got:#x} != generate_fingerprint(peers()) {want:#x}")
        prev = st
        if r % print_every == 0 or last or r <= heal + 2:
            traj.append(rec)
            if verbose:
                print(json.dumps(rec), flush=True)
        if last:
            break
    rounds = r + 1
    st = g.stats()
    fails += check_invariants(st, n, rounds)
    # a bench-style line for this layout: peer-rounds/s over the run, and the HBM roofline of the
    # layout's own algorithmic bytes per round — every row's entry list read once (4 B per entry, the sampled
    # footprints' mean), 32 B per message record, 4 B per KnownPeers payload id
    # (over every round run: the trajectory keeps only every print_every-th round and all rounds up to the heal,
    # a sample biased toward the cheap early rounds)
    wall = sum(all_ms) / 1e3
    sent = sum(st[k] for k in ("sent_ping", "sent_ping_req", "sent_ack", "sent_known_peers", "sent_kpr"))
    ents = [t["entries"] for t in traj if "entries" in t]
    b_round = (4.0 * (sum(ents) / len(ents) if ents else 0.0) + 32.0 * sent / max(rounds, 1)
               + 4.0 * st["sent_kp_ids"] / rounds)
    ms_round = wall * 1e3 / max(len(all_ms), 1)
    bench_line = {"metric": "simulated peer-rounds/sec", "value": n * len(all_ms) / wall if wall else None,
                  "unit": "peer-rounds/s", "ms_per_round": round(ms_round, 3), "rounds_timed": len(all_ms),
                  "roofline": {"bound": "hbm", "bytes_per_round": int(b_round),
                               "achieved": round(b_round / (ms_round / 1e3) / 1e9, 1) if ms_round else None,
                               "peak": 8000.0, "unit": "GB/s",
                               "frac": round(b_round / (ms_round / 1e3) / 8e12, 4) if ms_round else None}}
    kb = g.kernel_breakdown()
    round_ms, nr = g.kernel_time(1)
    g.close()
    return {"nodes": n, "rounds": rounds, "row_cap": row_cap, "create_s": round(t_create, 1), "fault_end_round": fault_end,
            "stat_flags": stat_flags, "converged_round": converged_round, "stopped_by": stopped_by,
            "wall_s": round(time.time() - t_start, 1), "bench_line": bench_line, "trajectory": traj,
            "kernels_ms_per_round": {k: round(v["ms"] / rounds, 3) for k, v in sorted(kb.items(), key=lambda x: -x[1]["ms"])},
            "gpu_round_ms_mean": round(round_ms / max(nr, 1), 2), "final_stats": st, "failures": fails}


def digest_diff(a, b, rng, nrows: int) -> list[str]:
    """Two GPU handles of one mesh (e.g. unsharded and as row shards): counters, every fingerprint and per-node
    scalar, and for sampled nodes the whole row, suspect/curious tables and peer_states."""
    out = []
    sa, sb = a.stats(), b.stats()
    out += [f"stats.{k}: {v} != {sb[k]}" for k, v in sa.items() if sb[k] != v]
    fa, fb = a.fingerprints(), b.fingerprints()
    if not np.array_equal(fa, fb):
        out.append(f"fingerprints: {int((fa != fb).sum())} differ, first {np.argwhere(fa != fb)[:3].ravel().tolist()}")
    if not np.array_equal(a.scalars(), b.scalars()):
        out.append("scalars differ")
    for i in rng.choice(a.capacity, nrows, replace=False):
        i = int(i)
        if not np.array_equal(a.row(i), b.row(i)):
            out.append(f"row {i} differs")
        if a.suspects(i) != b.suspects(i) or a.curious(i) != b.curious(i):
            out.append(f"suspect/curious table {i} differs")
        if a.peer_states_array(i).tobytes() != b.peer_states_array(i).tobytes() and a.peer_states(i) != b.peer_states(i):
            out.append(f"peer_states {i} differ")
        if out:
            break
    return out


def run_twin(case: dict, rounds: int, shards: int, nrows: int = 4, check_rows: int = 2, seed: int = 3,
             verbose: bool = False, externals=(), join_rounds=()) -> dict:
    """The mesh unsharded and as `shards` in-process row shards (kb_sim_create_local: every wave's records
    all-to-all-v'd between the shards, the broadcast lists all-gathered), stepped in lock step: digest_diff every
    round, and generate_fingerprint(peers()) on sampled rows of the sharded mesh.  The two handles are resident
    together (the sparse layout: a few GB per mesh at 1M-4M peers)."""
    import kaboodle_amd
    import parity
    from kaboodle_amd._ffi import Sim
    lib = kaboodle_amd.lib()
    cfg = case["cfg"]
    a, b = Sim(lib, cfg), Sim(lib, cfg, shards=shards)
    for x in externals:                        # real instances outside the mesh (kb_sim_set_external)
        a.set_external(x)
        b.set_external(x)
    rng = np.random.default_rng(seed)
    fails, traj = [], []
    exported = {"records": 0, "ids": 0, "kp_to_ext": 0}
    for r in range(rounds):
        parity.apply_events((a, b), case, r)
        if r in join_rounds:                   # each external instance broadcasts Join (src/kaboodle.rs:228-251)
            for x in externals:
                a.inject(x, 0, parity.K_JOIN, 0, 0, 0)
                b.inject(x, 0, parity.K_JOIN, 0, 0, 0)
        ta = time.time(); a.step(1); ta = time.time() - ta
        tb = time.time(); b.step(1); tb = time.time() - tb
        d = digest_diff(a, b, rng, nrows)
        if externals:
            ea, eb = a.exported(), b.exported()
            if ea != eb:
                d.append(f"exports differ: {len(ea)} vs {len(eb)} records")
            exported["records"] += len(ea)
            exported["ids"] += sum(len(e[9]) for e in ea)
            exported["kp_to_ext"] += sum(1 for e in ea if e[5] == parity.K_KP)
        if d:
            fails.append(f"round {r}: " + "; ".join(d[:4]))
            break
        for i in rng.choice(cfg.capacity, check_rows, replace=False):
            got, want = fp_of_peers(b, lib, int(i))
            if got != want:
                fails.append(f"round {r} row {i}: fingerprint {got:#x} != generate_fingerprint(peers()) {want:#x}")
        st = b.stats()
        rec = {"round": r, "ms_unsharded": round(ta * 1e3, 1), "ms_sharded": round(tb * 1e3, 1), "agree": st["agree"],
               "drop_partition": st["drop_partition"], "bcast_failed": st["bcast_failed"]}
        traj.append(rec)
        if verbose:
            print(json.dumps(rec), flush=True)
    st = b.stats()
    fp = b.sparse_footprint()
    a.close()
    b.close()
    return {"nodes": cfg.capacity, "shards": shards, "rounds": len(traj), "trajectory": traj, "final_stats": st,
            "footprint": fp, "exported": exported, "failures": fails}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=4 * 1024 * 1024)
    ap.add_argument("--rounds", type=int, default=24)
    ap.add_argument("--every", type=int, default=256)
    ap.add_argument("--row-cap", type=int, default=2048)
    ap.add_argument("--check-rows", type=int, default=4)
    ap.add_argument("--out", default="")
    ap.add_argument("--fault-end", type=int, default=-1, help="loss ends at this round (-1: never)")
    ap.add_argument("--until-converged", action="store_true")
    ap.add_argument("--budget-s", type=float, default=0.0)
    ap.add_argument("--print-every", type=int, default=1)
    ap.add_argument("--fp-every", type=int, default=4)
    ap.add_argument("--count-sf-failed-drops", action="store_true")
    ap.add_argument("--no-sf-failed-drops", action="store_true", help="the default (kept for older scripts)")
    a = ap.parse_args()
    from kaboodle_amd._ffi import KB_STAT_NO_SF_FAILED_DROPS
    res = run(a.nodes, a.rounds, a.every, a.row_cap, a.check_rows, fault_end=a.fault_end,
              stat_flags=0 if a.count_sf_failed_drops else KB_STAT_NO_SF_FAILED_DROPS, until_converged=a.until_converged,
              budget_s=a.budget_s, print_every=a.print_every, fp_every=a.fp_every)
    res["scenario"] = ("configs[4]: converged start, 5% loss" + (f" until round {a.fault_end}" if a.fault_end >= 0 else "")
                       + ", 2-way partition rounds 3-11, heal at 12 (every "
                       f"{a.every}th peer pings across), socket_faithful, sparse rows on one MI355X"
                       + ("" if a.count_sf_failed_drops else "; Failed-list drops not counted (KB_STAT_NO_SF_FAILED_DROPS)"))
    print(json.dumps({k: v for k, v in res.items() if k != "trajectory"}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)
    return 1 if res["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
