"""configs[4]'s representation measured: the partition + heal scenario in socket_faithful mode
(converged start, 5 % loss, two halves cut off for rounds 3-11, healed at round 12 by every 256th peer
pinging the other half) on the oracle's sparse rows (KB_VARIANT_SPARSE_ROWS: shared base, per-row exceptions,
explicit non-ancient stamps), checked bit-exact against the dense oracle on sampled rows where that fits in
host memory, with the per-row footprint every few rounds.  The per-row figures then size a 4M-peer mesh
on 8 GPUs.

    python tools/sparse_plan.py --nodes 16384 65536 --rounds 160 --out profiles/r04_sparse_plan.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from dataclasses import replace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(n: int, rounds: int, dense_upto: int, every: int) -> dict:
    import parity
    from test_sparse import SPARSE, footprint
    from kaboodle_amd._ffi import KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, Sim, SimConfig
    cfg = SimConfig(capacity=n, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.05, partition_groups=2,
                    partition_start=3, partition_end=12, seed=9, failed_mode=KB_FAILED_SOCKET_FAITHFUL)
    case = {"cfg": cfg, "events": {12: [("ping", i, [(i + n // 2) % n]) for i in range(0, n, 256)]}}
    lib = parity.oracle_lib(omp=True)
    s = Sim(lib, replace(cfg, variant=SPARSE))
    d = Sim(lib, cfg) if n <= dense_upto else None
    rng = np.random.default_rng(5)
    traj, t0 = [], time.time()
    for r in range(rounds):
        parity.apply_events((s, d) if d else (s,), case, r)
        s.step(1)
        if d:
            d.step(1)
            diff = parity.compare_sampled(d, s, rng, nrows=16)
            assert not diff, f"n={n} round {r}: " + "; ".join(diff[:4])
        if r % every == every - 1 or r == rounds - 1 or r in (5, 11):
            fp = footprint(s)
            st = s.stats()
            traj.append({"round": r, "agree": st["agree"], "alive": st["alive"],
                         "exceptions_per_row": round(fp["exceptions"] / n, 3), "stamps_per_row": round(fp["stamps"] / n, 2),
                         "max_row_entries": fp["max_row_entries"], "bytes_per_row": round(fp["bytes"] / n, 1),
                         "wall_s": round(time.time() - t0, 1)})
            print(f"n={n} round {r}: {traj[-1]}", flush=True)
    s.close()
    if d:
        d.close()
    return {"nodes": n, "rounds": rounds, "dense_checked": d is not None, "trajectory": traj}


def plan(res: list[dict]) -> dict:
    """4M peers on 8 MI355X from the largest measured size: per-row sparse bytes at the worst sampled round,
    the fixed per-row tables the dense simulator already keeps (suspect, curious, ping queue slots,
    checkpoints, freshness log), and the shared base tables, per GPU holding 1/8 of the rows."""
    big = max(res, key=lambda x: x["nodes"])
    worst = max(t["bytes_per_row"] for t in big["trajectory"])
    peers, gpus = 4 * 1024 * 1024, 8
    rows = peers // gpus
    fixed = 8 * 16 + 8 * 32 + 8 * 4 + 64 * 8 + 8 + 2048 * 4 + 16 * 4 + 64     # susp, cur, paq, segp, sdirty, flog, fstart, scalars
    sparse = int(worst * 2)                                                  # headroom x2 for growth between rebuilds
    base = peers // 8 + 3 * 4 * peers                                        # base bits, prefix counts + folds, Z^k
    per_gpu = rows * (sparse + fixed) + base
    dense_stamps = rows * peers
    return {"peers": peers, "gpus": gpus, "rows_per_gpu": rows, "measured_at_nodes": big["nodes"],
            "sparse_bytes_per_row_worst": worst, "sparse_bytes_per_row_budget": sparse, "fixed_bytes_per_row": fixed,
            "base_tables_bytes": base, "bytes_per_gpu": per_gpu, "gb_per_gpu": round(per_gpu / 1e9, 2),
            "dense_stamp_bytes_per_gpu": dense_stamps, "dense_gb_per_gpu": round(dense_stamps / 1e9, 1),
            "hbm_gb_per_gpu": 288}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, nargs="+", default=[16384, 65536])
    ap.add_argument("--rounds", type=int, default=160)
    ap.add_argument("--dense-upto", type=int, default=16384)
    ap.add_argument("--every", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = [run(n, a.rounds, a.dense_upto, a.every) for n in a.nodes]
    out = {"scenario": "configs[4] shape: converged start, 5% loss, 2-way partition rounds 3-11, heal at 12 "
                       "(every 256th peer pings across), socket_faithful", "results": res, "plan_4M_8gpu": plan(res)}
    print(json.dumps(out["plan_4M_8gpu"]), flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
