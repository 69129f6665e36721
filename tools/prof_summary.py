"""Summaries of rocprofv3 CSV output (dev tool).

  prof_summary.py stats <dir> [K]        kernel_stats.csv -> compact table (name, calls, avg us, total %), and
                                         k_sweep's average over its last K launches of the kernel trace
                                         (bench's timed steps; the table's average includes the warmup)
  prof_summary.py pmc <dir> <kernel> [bench args]
                                         counter_collection.csv of the FETCH_SIZE / WRITE_SIZE passes ->
                                         JSON with HBM bytes per launch of <kernel> (FETCH_SIZE x2, gfx950)
"""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "kb::"):
        n = n.replace(pre, "")
    return n


def stats(d, k_last=0):
    rs = rows(os.path.join(d, "**", "*kernel_stats.csv"))
    rs.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print(f"{'kernel':40s} {'calls':>7s} {'avg_us':>10s} {'pct':>6s}")
    for r in rs:
        print(f"{short(r['Name'])[:40]:40s} {r['Calls']:>7s} {float(r['AverageNs'])/1e3:10.2f} {float(r['Percentage']):6.2f}")
    if k_last:
        for kn in ("k_rowpass<true>", "k_rowpass<false>", "k_fold"):
            tr = [r for r in rows(os.path.join(d, "**", "*kernel_trace.csv")) if short(r["Kernel_Name"]) == kn]
            tr.sort(key=lambda r: int(r["Start_Timestamp"]))
            dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr][-k_last:]
            if dur:
                print(f"{kn} over its last {len(dur)} launches (the timed steps): avg {sum(dur) / len(dur):.2f} us")


def pmc(d, kernel, args):
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(d, c, "**", "*counter_collection.csv"))
                if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == c]
        res[c] = sum(vals) / len(vals) if vals else None
        res[c + "_dispatches"] = len(vals)
    # rocprofv3 reports both in KB; gfx950 FETCH_SIZE counts half of a wide streaming read (guide, HBM section)
    fetch = res["FETCH_SIZE"] * 1024 * 2 if res["FETCH_SIZE"] is not None else None
    write = res["WRITE_SIZE"] * 1024 if res["WRITE_SIZE"] is not None else None
    nodes, loss, churn, steps, warmup = 65536, 0.01, 0.001, 50, 5
    for k, v in zip(args[::2], args[1::2]):
        if k == "--nodes":
            nodes = int(v)
        elif k == "--steps":
            steps = int(v)
        elif k == "--warmup":
            warmup = int(v)
    workload = f"configs[2]: {nodes} peers, converged start, {loss:.0%} loss, {churn:.1%}/round churn"
    capacity = nodes + max(4096, int(nodes * churn * (steps + warmup + 8) * 1.5))      # bench.rank_config
    out = {"kernel": kernel.split("<")[0], "workload": workload, "capacity": capacity, "raw_kb": res,
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": (fetch or 0) + (write or 0) if fetch is not None else None,
           "correction": "FETCH_SIZE(KB)*1024*2 (gfx950 half-count of 16B/lane streaming reads) + WRITE_SIZE(KB)*1024"}
    print(json.dumps(out, indent=1))


def sq(d):
    """per-kernel averages of SQ counters (one pass of up to 8 SQ counters)"""
    agg = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        k = short(r["Kernel_Name"])
        a = agg.setdefault(k, {})
        a.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    names = sorted({n for a in agg.values() for n in a})
    print(f"{'kernel':28s} " + " ".join(f"{n[3:][:14]:>14s}" for n in names))
    for k, a in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
        print(f"{k[:28]:28s} " + " ".join(f"{(sum(a[n]) / len(a[n]) if n in a else 0):14.0f}" for n in names))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0)
    elif sys.argv[1] == "sq":
        sq(sys.argv[2])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4:])
