"""Measured effect of the declared deviations, on the CPU oracle (its semantic variants,
kb_config.variant; the HIP library runs round semantics v1 only):

  same-window broadcasts  v1 delivers a round's Join/Failed broadcasts at the next round start; the
                          reference handles them inside the same receive window (src/kaboodle.rs:770-778)
  exact LRU               v1 keeps a one-byte stamp window: peers older than ~190 rounds tie as "ancient"
                          and A3 breaks the tie by a rotating sweep front; the reference orders by exact
                          Instants (src/kaboodle.rs:662-675)

    python tools/deviations.py [out.json]        (writes profiles/r03_deviations.json by default)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import parity  # noqa: E402
from kaboodle_amd._ffi import (KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_VARIANT_EXACT_LRU,  # noqa: E402
                               KB_VARIANT_SAME_WINDOW_BCAST, Sim, SimConfig)

CONFIG1_IDS = parity.CONFIG1_IDS


def first_converged(cfg, cap, setup=None):
    with Sim(parity.oracle_lib(omp=True), cfg) as o:
        if setup:
            setup(o)
        for _ in range(cap):
            o.step(1)
            st = o.stats()
            if st["first_converged_round"] >= 0:
                return st["first_converged_round"], st
        return None, o.stats()


def trajectory(cfg, marks=(5, 10, 20, 50, 100)):
    """agreement fraction (views equal to the running set) and the mean |view| gap at fixed rounds"""
    import numpy as np
    out = {}
    with Sim(parity.oracle_lib(omp=True), cfg) as o:
        r = 0
        for m in marks:
            o.step(m - r)
            r = m
            st = o.stats()
            sc = o.scalars()
            live = sc[:, 0] != 0
            gap = float(np.abs(sc[live, 1].astype(np.int64) - int(live.sum())).mean())
            out[m] = {"agree_frac": round(st["agree"] / max(st["alive"], 1), 4), "view_gap_mean": round(gap, 2)}
    return out


def tail_converged(cfg, fault_rounds, cap):
    """rounds after the faults stop until every live view equals the running set (None at the cap)"""
    with Sim(parity.oracle_lib(omp=True), cfg) as o:
        o.step(fault_rounds)
        for k in range(cap):
            o.step(1)
            st = o.stats()
            if st["agree"] == st["alive"]:
                return k + 1, st
        return None, o.stats()


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r03_deviations.json")
    res = {"tool": "tools/deviations.py", "oracle": "oracle/kb_oracle.c (OpenMP)", "rows": []}
    t0 = time.time()

    def cfg1_setup(o):
        for i, n in enumerate(CONFIG1_IDS):
            o.set_identity(i, n)
            o.start_node(i)

    # (1) broadcast delivery: next round (v1) vs the same receive window
    cases = [("configs[0] 2x2 mesh (identities, no loss)", lambda v: SimConfig(capacity=4, initial_nodes=0, variant=v), cfg1_setup, 20)]
    for seed in (1, 2, 3):
        cases.append((f"configs[1] 1K join, no loss, seed {seed}",
                      lambda v, seed=seed: SimConfig(capacity=1024, initial_nodes=1024, seed=seed, variant=v), None, 60))
    for name, mk, setup, cap in cases:
        a, _ = first_converged(mk(0), cap, setup)
        b, _ = first_converged(mk(KB_VARIANT_SAME_WINDOW_BCAST), cap, setup)
        res["rows"].append({"deviation": "broadcast delivery", "case": name, "metric": "first converged round",
                            "v1_next_round": a, "same_window": b})
        print(res["rows"][-1], flush=True)

    # lossy meshes do not converge inside a few hundred rounds in either reading: compare trajectories
    for mode, fm in (("sim_sender", 0), ("socket_faithful", KB_FAILED_SOCKET_FAITHFUL)):
        for seed in (1, 2):
            mk = lambda v, seed=seed, fm=fm: SimConfig(capacity=1024, initial_nodes=1024, seed=seed, loss=0.02,
                                                       failed_mode=fm, variant=v)
            res["rows"].append({"deviation": "broadcast delivery", "case": f"configs[1] with 2% loss, {mode}, seed {seed}",
                                "metric": "agreement fraction / mean view-size gap at rounds 5..100",
                                "v1_next_round": trajectory(mk(0)), "same_window": trajectory(mk(KB_VARIANT_SAME_WINDOW_BCAST))})
            print(res["rows"][-1], flush=True)

    # (2) A3 order: one-byte stamp window with ancient ties (v1) vs exact instants (LRU)
    for seed in (1, 2):
        n = 1536
        mk = lambda v, seed=seed: SimConfig(capacity=n + 256, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.01,
                                            churn=0.001, fault_end_round=25, seed=seed,
                                            failed_mode=KB_FAILED_SOCKET_FAITHFUL, variant=v)
        cap = 4 * n
        a, sa = tail_converged(mk(0), 25, cap)
        b, sb = tail_converged(mk(KB_VARIANT_EXACT_LRU), 25, cap)
        res["rows"].append({"deviation": "A3 ordering (stamp window)",
                            "case": f"{n} peers, socket_faithful, 1% loss + 0.1%/round churn until round 25, seed {seed}",
                            "metric": "quiet rounds until every live view equals the running set (cap 4N)",
                            "v1_ancient_ties": a, "exact_lru": b,
                            "v1_agree_at_end": f"{sa['agree']}/{sa['alive']}", "exact_agree_at_end": f"{sb['agree']}/{sb['alive']}"})
        print(res["rows"][-1], flush=True)
    res["seconds"] = round(time.time() - t0, 1)
    json.dump(res, open(out_path, "w"), indent=1)
    print("wrote", out_path)


if __name__ == "__main__":
    main()
