"""Per-wave kernel time of the benched workload (dev tool, GPU): bench.py's configs[2] mesh, W warmup rounds, then
K rounds with an event pair on every launch (set_profiling(2), as bench.py's replay), and each receive-window
kernel's ms per round split by delivery wave.

    python tools/wave_times.py [--steps 20] [--warmup 5] [--out gpurun_out/wave_times.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import kaboodle_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--out", default="")
ns = ap.parse_args()
sys.argv = [sys.argv[0], "--steps", str(ns.steps), "--warmup", str(ns.warmup)]
a = bench.parse()
cfg = bench.rank_config(a, 0, 1, 0)
with kaboodle_amd.Mesh(cfg) as m:
    m.set_profiling(2)
    m.step(a.warmup)
    m.reset_kernel_time()
    m.step(a.steps)
    bd = m.kernel_breakdown()
out = {"workload": "configs[2]: 65536 peers (bench.py's mesh)", "steps": ns.steps, "warmup": ns.warmup, "kernels": {}}
for name in ("k_route", "k_scan_tiles", "k_scan_apply", "k_scatter", "k_kp", "k_sortfast", "k_proc"):
    if name in bd:
        k = bd[name]
        out["kernels"][name] = {"ms_per_round": round(k["ms"] / ns.steps, 4),
                                "per_wave_ms": [round(x / ns.steps, 4) for x in k["wave_ms"]]}
        print(name, json.dumps(out["kernels"][name]), flush=True)
waves = len(next(iter(out["kernels"].values()))["per_wave_ms"])
out["window_per_wave_ms"] = [round(sum(v["per_wave_ms"][w] for v in out["kernels"].values()), 4) for w in range(waves)]
print("window per wave", out["window_per_wave_ms"], flush=True)
if ns.out:
    with open(ns.out, "w") as f:
        json.dump(out, f, indent=1)
