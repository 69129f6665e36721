"""Busy time, span and the largest idle gaps between the kernels of each round of a rocprofv3 kernel
trace (dev tool): round_gaps.py <kernel_trace.csv>.  A round starts at k_alive_bits."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    return n.split("(")[0].replace("void ", "").replace("kb::", "")


idx = [k for k, r in enumerate(rows) if short(r["Kernel_Name"]) == "k_alive_bits"]
for a, b in zip(idx, idx[1:]):
    seg = rows[a:b]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    gaps = [((int(q["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3, short(q["Kernel_Name"])) for p, q in zip(seg, seg[1:])]
    print(f"kernels {len(seg)} busy {busy:.0f} us span {span:.0f} us gaps {span - busy:.0f} us; largest:",
          [(round(g), k) for g, k in sorted(gaps, reverse=True)[:5]])
