"""Per-wave kernel durations of a few rounds from a rocprofv3 kernel trace (dev tool).

    python tools/wave_prof.py <kernel_trace.csv>

Dispatches are taken in start order; a round starts at k_alive_bits, and every k_route / k_route_x
starts a wave.  Prints, per round, the duration of each kernel instance tagged with its wave index.
"""
import csv
import sys
from collections import defaultdict


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("kb::", "")
    return n


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rounds, cur, wave = [], None, -1
for r in rows:
    k = short(r["Kernel_Name"])
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k == "k_alive_bits":
        cur = defaultdict(float)
        rounds.append(cur)
        wave = -1
    if cur is None:
        continue
    if k in ("k_route", "k_route_x"):
        wave += 1
    cur[(wave, k)] += us
for n, rd in enumerate(rounds):
    tot = sum(rd.values())
    print(f"round {n}: {tot:8.1f} us of kernels")
    pre = sorted(((k, v) for (w, k), v in rd.items() if w < 0), key=lambda x: -x[1])
    print("   pre-wave: " + ", ".join(f"{k} {v:.0f}" for k, v in pre if v >= 20))
    for w in range(0, 1 + max(w for w, _ in rd)):
        items = sorted(((k, v) for (ww, k), v in rd.items() if ww == w), key=lambda x: -x[1])
        print(f"   wave {w}: {sum(v for _, v in items):7.1f}  " + ", ".join(f"{k} {v:.0f}" for k, v in items if v >= 10))
