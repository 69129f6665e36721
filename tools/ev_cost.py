"""What the per-launch HIP events cost the round (dev tool, GPU): the benched workload stepped with
profiling level 1 (events on the kernels with byte counters, as bench.py's timed rounds) and level 0 (no
events), alternating, each on a fresh mesh over the same rounds: wall time per round.   python tools/ev_cost.py [STEPS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import kaboodle_amd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
a = bench.parse([])
cfg = bench.rank_config(a, 0, 1, 0)
for level in (1, 0, 1, 0):                      # the same deterministic rounds each time
    with kaboodle_amd.Mesh(cfg) as m:
        m.set_profiling(level)
        m.step(a.warmup)
        t = time.perf_counter()
        m.step(steps)
        dt = time.perf_counter() - t
    print(f"profiling level {level}: {dt / steps * 1e3:.3f} ms per round", flush=True)
