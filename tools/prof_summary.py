"""Summaries of rocprofv3 CSV output (dev tool).

  prof_summary.py stats <dir>                     kernel_stats.csv -> compact table (name, calls, avg us, total %)
  prof_summary.py rounds <dir> <warmup> <steps>   kernel_trace.csv -> per-round kernel time over the timed rounds
                                                  only (bench's timed region), kernels named as bench.py names them
  prof_summary.py pmc <dir> <tag-json-fields...>  counter_collection.csv of the FETCH_SIZE / WRITE_SIZE passes
                                                  (<dir>/FETCH_SIZE, <dir>/WRITE_SIZE) -> JSON: HBM bytes per launch
                                                  and per round of every kernel over the timed rounds
  prof_summary.py sq <dir>                        per-kernel averages of SQ counters

Rounds are delimited by the dispatches of k_round_end (the last kernel of every round): the timed rounds
of `bench.py --warmup W --steps K` are the dispatches after the W-th k_round_end up to the (W+K)-th.
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


def bench_name(name):
    """The kernel as bench.py's breakdown names it (template arguments and LDS/HBM variants folded)."""
    n = short(name).split("<")[0]
    return {"k_bfail_prep_lds": "k_bfail_prep"}.get(n, n)


def timed_window(rs, warmup, steps, id_key):
    """(first, last] dispatch ids of the timed rounds, from the k_round_end dispatches."""
    ends = sorted(int(r[id_key]) for r in rs if bench_name(r["Kernel_Name"]) == "k_round_end")
    if len(ends) < warmup + steps:
        raise SystemExit(f"only {len(ends)} rounds in the trace, need {warmup + steps}")
    return (ends[warmup - 1] if warmup else -1), ends[warmup + steps - 1]


def stats(d):
    rs = rows(os.path.join(d, "**", "*kernel_stats.csv"))
    rs.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print(f"{'kernel':40s} {'calls':>7s} {'avg_us':>10s} {'pct':>6s}")
    for r in rs:
        print(f"{short(r['Name'])[:40]:40s} {r['Calls']:>7s} {float(r['AverageNs'])/1e3:10.2f} {float(r['Percentage']):6.2f}")


def per_round(d, warmup, steps):
    tr = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    lo, hi = timed_window(tr, warmup, steps, "Dispatch_Id")
    agg = {}
    span = [None, None]
    for r in tr:
        k = int(r["Dispatch_Id"])
        if not lo < k <= hi:
            continue
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        span[0] = a if span[0] is None else min(span[0], a)
        span[1] = b if span[1] is None else max(span[1], b)
        e = agg.setdefault(bench_name(r["Kernel_Name"]), [0, 0.0])
        e[0] += 1
        e[1] += (b - a) / 1e6
    out = {"warmup": warmup, "steps": steps, "kernels": {}}
    tot = 0.0
    for n, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out["kernels"][n] = {"ms_per_round": round(ms / steps, 4), "launches_per_round": round(c / steps, 2),
                             "avg_launch_us": round(ms / c * 1e3, 2)}
        tot += ms
    out["kernel_ms_per_round"] = round(tot / steps, 4)
    out["first_to_last_dispatch_ms_per_round"] = round((span[1] - span[0]) / 1e6 / steps, 4)
    print(json.dumps(out, indent=1))


# kernels whose HBM reads are 16 B/lane coalesced streams (row stamps staged / copied as uint4)
STREAM16 = {"k_rowpass", "k_resp_wave"}


def pmc(d, fields):
    meta = json.loads(fields) if fields else {}
    warmup, steps = meta.get("warmup", 5), meta.get("steps", 20)
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rs = [r for r in rows(os.path.join(d, c, "**", "*counter_collection.csv")) if r.get("Counter_Name") == c]
        lo, hi = timed_window(rs, warmup, steps, "Dispatch_Id")
        for r in rs:
            if lo < int(r["Dispatch_Id"]) <= hi:
                e = res.setdefault(bench_name(r["Kernel_Name"]), {}).setdefault(c, [0, 0.0])
                e[0] += 1
                e[1] += float(r["Counter_Value"])
    kern = {}
    for n, e in res.items():
        if "FETCH_SIZE" not in e or "WRITE_SIZE" not in e:
            continue
        launches = e["FETCH_SIZE"][0]
        # rocprofv3 reports both in KB.  gfx950 FETCH_SIZE counts half of a wide (16 B/lane) coalesced
        # streaming read (guide, HBM section): doubled only for the kernels whose reads are that shape; the
        # gathers (k_fold's byte-table lookups, the handlers' member words) are reported raw
        raw = e["FETCH_SIZE"][1] * 1024
        fetch = raw * (2 if n in STREAM16 else 1)
        write = e["WRITE_SIZE"][1] * 1024
        kern[n] = {"launches_per_round": launches / steps, "fetch_bytes_per_launch": int(fetch / launches),
                   "fetch_raw_bytes_per_launch": int(raw / launches), "fetch_doubled": n in STREAM16,
                   "write_bytes_per_launch": int(write / launches),
                   "hbm_bytes_per_launch": int((fetch + write) / launches),
                   "hbm_bytes_per_round": int((fetch + write) / steps)}
    out = dict(meta)
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kaboodle_amd", "libkaboodle_sim.so")
    out["lib_sha16"] = (hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]   # the build the counters measured
                        if os.path.exists(lib) else None)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from kaboodle_amd import build as kb_build                   # and its sources (bench.py matches either)
    out["lib_src_sha16"] = kb_build.src_sha16()
    out["kernels"] = dict(sorted(kern.items(), key=lambda kv: -kv[1]["hbm_bytes_per_round"]))
    out["correction"] = ("FETCH_SIZE(KB)*1024, x2 only for " + ", ".join(sorted(STREAM16)) +
                         " (gfx950 half-count of 16 B/lane streaming reads; other kernels raw) + WRITE_SIZE(KB)*1024")
    out["window"] = f"the {steps} timed rounds after {warmup} warmup rounds (k_round_end dispatches delimit rounds)"
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
        stats(sys.argv[2])
    elif sys.argv[1] == "rounds":
        per_round(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    elif sys.argv[1] == "sq":
        sq(sys.argv[2])
    else:
        pmc(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
