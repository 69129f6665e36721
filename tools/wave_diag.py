"""Per-wave diagnostics of the benched workload (dev tool, GPU): KB_DEBUG_WAVES=1 KB_DEV=64 python tools/wave_diag.py [rounds]

Runs bench.py's configs[2] mesh (same capacity, seed, faults) for `rounds` rounds; the library prints, per
round and wave, inbox sizes, k_proc's node count, prologue insertions, fingerprint refreshes and (KB_DEV=64)
k_proc's per-part wall time.  Only the last round's lines are worth reading (the workload drifts)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import kaboodle_amd  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 25
a = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
sys.argv = [sys.argv[0], "--steps", str(rounds - 5), "--warmup", "5"]
a = bench.parse()
cfg = bench.rank_config(a, 0, 1, 0)
with kaboodle_amd.Mesh(cfg) as m:
    m.step(rounds)
    st = m.stats()
    print(f"round {st['round']}: agree {st['agree']}/{st['alive']}", flush=True)
