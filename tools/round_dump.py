"""Every kernel of one round of a rocprofv3 kernel trace, in dispatch order, with its wave index and the
idle gap before it (dev tool): round_dump.py <kernel_trace.csv> [round index, default: second to last]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    return n.split("(")[0].replace("void ", "").replace("kb::", "")


rounds, cur, wave, prev_end = [], None, -1, None
for r in rows:
    k = short(r["Kernel_Name"])
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if k == "k_alive_bits":
        cur, wave = [], -1
        rounds.append(cur)
    if cur is not None:
        if k in ("k_route", "k_route_x"):
            wave += 1
        cur.append((wave, k, (e - s) / 1e3, (s - prev_end) / 1e3 if prev_end else 0.0))
    prev_end = e
rd = rounds[int(sys.argv[2]) if len(sys.argv) > 2 else -2]
for w, k, d, g in rd:
    print(f"{w:2d} {k:28s} {d:8.1f} us   gap {g:6.1f}")
print(f"total {sum(x[2] for x in rd):.1f} us of kernels, {sum(x[3] for x in rd):.1f} us of gaps")
