"""Per-wave wall spans vs summed kernel durations from a rocprofv3 kernel trace (dev tool): how much of each
delivery wave is kernel time and how much is the gap between dependent launches.

    python tools/wave_span.py <kernel_trace.csv> [first_round]
"""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.split("(")[0].replace("void ", "").replace("kb::", "")


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rounds, cur, wave = [], None, -1
for r in rows:
    k = short(r["Kernel_Name"])
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if k == "k_alive_bits":
        cur = defaultdict(list)
        rounds.append(cur)
        wave = -1
    if cur is None:
        continue
    if k in ("k_route", "k_route_x"):
        wave += 1
    cur[wave].append((a, b, k))
agg = defaultdict(lambda: [0.0, 0.0, 0])
for rd in rounds[first:-1]:
    for w, ks in rd.items():
        span = (max(b for _, b, _ in ks) - min(a for a, _, _ in ks)) / 1e3
        busy = sum(b - a for a, b, _ in ks) / 1e3
        agg[w][0] += span; agg[w][1] += busy; agg[w][2] += len(ks)
n = max(1, len(rounds[first:-1]))
for w in sorted(agg):
    s, b, c = agg[w]
    print(f"wave {w:2d}: span {s / n:7.1f} us  kernels {b / n:7.1f} us  launches {c / n:5.1f}  gap/launch {(s - b) / max(c, 1):5.2f} us")
