"""Per-round wall time of the benched workload (dev tool, GPU): python tools/round_series.py [rounds] [exact|window]

bench.py's configs[2] mesh (same capacity, seed, faults), stepped one round at a time with a device sync
after each, so the transient of the converged start (KnownPeersRequest replies under the size cap while
the freshness windows fill, rounds < SHARE_AGE) shows next to the steady state."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import kaboodle_amd  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 40
order = sys.argv[2] if len(sys.argv) > 2 else "exact"          # A3 order (bench.py's --a3-order; default exact)
sys.argv = [sys.argv[0], "--steps", str(rounds - 5), "--warmup", "5", "--a3-order", order]
a = bench.parse()
cfg = bench.rank_config(a, 0, 1, 0)
out = []
with kaboodle_amd.Mesh(cfg) as m:
    m.step(1)
    for r in range(1, rounds):
        t = time.perf_counter()
        m.step(1)
        dt = time.perf_counter() - t
        st = m.stats()
        out.append({"round": r, "ms": round(dt * 1e3, 3), "sent_kp_ids": st["sent_kp_ids"], "sent_kpr": st["sent_kpr"],
                     "drop_oversize": st["drop_oversize"]})
        print(json.dumps(out[-1]), flush=True)
