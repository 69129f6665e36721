"""Rounds to fingerprint convergence of the bench workload (BASELINE.json metric, second half).

    python tools/converge.py [--mode sim|sock] [--nodes 65536] [--faults 25] [--cap-factor 2] [--out FILE]

Runs configs[2] exactly as bench.py does (converged start, 1 % loss, 0.1 %/round churn, faults until
round F = 25 = warmup + steps of the driver's bench), then keeps stepping the quiescent tail (no loss,
no churn) on the GPU until every live peer's fingerprint equals the fingerprint of the true live set
(kb_stats.agree == alive) or the cap of cap_factor * N rounds.  Every 256 tail rounds it
records the agreement and the mean view-size gap |known_i| - live into the trajectory and prints a
progress line.  `--mode sock` = failed_mode socket_faithful (Failed never honoured, as over real
sockets: src/networking.rs:44-55); `sim` = sim_sender (honoured).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def kb_src_sha16():
    """the sources the in-tree library is built from (None for an A/B build loaded through KB_LIB_PATH)"""
    import kaboodle_amd
    from kaboodle_amd import build as kb_build
    return kb_build.src_sha16() if os.path.abspath(kaboodle_amd.LIB_PATH) == os.path.abspath(kb_build.OUT) else None


def lib_sha16() -> str:
    """the library build this record was made with (bench.py attaches a tail record only when it matches)"""
    import hashlib
    import kaboodle_amd
    return hashlib.sha256(open(kaboodle_amd.LIB_PATH, "rb").read()).hexdigest()[:16]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("sim", "sock"), default="sim")
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--faults", type=int, default=25)
    ap.add_argument("--cap-factor", type=float, default=2.0)
    ap.add_argument("--every", type=int, default=256)
    ap.add_argument("--budget-s", type=float, default=1e9, help="stop early after this many seconds")
    ap.add_argument("--lru", choices=("window", "exact"), default="window",
                    help="A3's order: the 1-byte stamp window with the sweep front (declared), or the exact instants "
                         "(KB_VARIANT_EXACT_LRU, src/kaboodle.rs:662-675)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import kaboodle_amd
    from kaboodle_amd._ffi import (KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_VARIANT_EXACT_LRU,
                                   SimConfig)
    kaboodle_amd.require_gpu()
    n, F = a.nodes, a.faults
    cfg = SimConfig(capacity=n + max(4096, int(n * 0.001 * (F + 8) * 1.5)), initial_nodes=n,
                    init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.001, fault_end_round=F, seed=1,
                    failed_mode=KB_FAILED_SOCKET_FAITHFUL if a.mode == "sock" else KB_FAILED_SIM_SENDER,
                    variant=KB_VARIANT_EXACT_LRU if a.lru == "exact" else 0)
    cap = int(a.cap_factor * n)
    t0 = time.time()
    traj = []

    def sample(m, r):
        st = m.stats()
        sc = m.scalars()
        live = sc[:, 0] != 0
        gap = sc[live, 1].astype(np.int64) - int(live.sum())
        rec = {"round": r, "agree": st["agree"], "alive": st["alive"], "agree_frac": round(st["agree"] / max(st["alive"], 1), 6),
               "view_gap_mean": round(float(np.abs(gap).mean()), 2), "view_gap_signed_mean": round(float(gap.mean()), 2),
               "view_exact_frac": round(float((gap == 0).mean()), 6), "wall_s": round(time.time() - t0, 1)}
        traj.append(rec)
        return st

    conv = None
    with kaboodle_amd.Mesh(cfg) as m:
        m.step(F)
        st = sample(m, F - 1)
        print(f"[converge {a.mode}] faults over at round {F}: agree {st['agree']}/{st['alive']}", flush=True)
        r = F
        while r < F + cap and time.time() - t0 < a.budget_s:
            m.step(1)
            s = m.stats()
            if s["alive"] and s["agree"] == s["alive"]:
                conv = r
                sample(m, r)
                break
            r += 1
            if (r - F) % a.every == 0:
                st = sample(m, r - 1)
                print(f"[converge {a.mode}] round {r - 1}: agree {st['agree']}/{st['alive']}, "
                      f"mean view gap {traj[-1]['view_gap_mean']}, {time.time() - t0:.0f} s", flush=True)
        if conv is None:
            sample(m, r - 1)
            # the few nodes still disagreeing: what their views lack or keep
            sc = m.scalars()
            live = np.nonzero(sc[:, 0] != 0)[0]
            lset = set(int(x) for x in live)
            tfp = m.true_fingerprint() if hasattr(m, "true_fingerprint") else None
            fps = m.fingerprints()
            bad = [int(i) for i in live if tfp is not None and fps[i] != tfp][:8]
            for i in bad:
                ids = set(m.peers(i)) if hasattr(m, "peers") else set()
                extra, missing = sorted(ids - lset)[:10], sorted(lset - ids)[:10]
                st = [e for e in m.peer_states(i) if e[0] in extra][:10] if hasattr(m, "peer_states") else []
                print(f"[converge {a.mode}] node {i} disagrees: extra {extra} missing {missing} extra states {st}", flush=True)
                traj.append({"round": r - 1, "node": i, "extra": extra, "missing": missing})
    out = {"workload": f"configs[2]: {n} peers, converged start, 1% loss, 0.1%/round churn, faults until round {F}",
           "failed_mode": "socket_faithful" if a.mode == "sock" else "sim_sender", "fault_end_round": F,
           "a3_order": a.lru,
           "converged_round": conv, "tail_rounds_to_converge": None if conv is None else conv - F + 1,
           "tail_rounds_run": traj[-1]["round"] - F + 1, "cap_rounds": cap,
           "stopped_by": "converged" if conv is not None else ("cap" if traj[-1]["round"] >= F + cap - 1 else "budget"),
           "wall_s": round(time.time() - t0, 1), "lib_sha16": lib_sha16(), "lib_src_sha16": kb_src_sha16(), "trajectory": traj}
    txt = json.dumps(out)
    print(json.dumps({k: v for k, v in out.items() if k != "trajectory"}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
