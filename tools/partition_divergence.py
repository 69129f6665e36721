"""configs[4] evidence: how far the rows of a partitioned-then-healed mesh are from a shared
base, measured on the GPU at 64K peers (the scenario of tests/test_gpu_fullsize.py::test_partition_heal_64k:
5 % loss, halves cut off for rounds 3-11, healed at round 12 by ping_addrs across the halves).

For sampled rows at several rounds: membership exceptions against (a) one global base set (bitwise
majority of the sampled rows) and (b) a per-partition base (majority of the rows of the same half); the
entries whose stamp is not "ancient" (Known(t) inside the window, or WaitingFor*), which a base+exceptions
form must also store per row.  Written to profiles/r03_partition_divergence.json.

    python tools/partition_divergence.py [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import kaboodle_amd  # noqa: E402
from kaboodle_amd._ffi import KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, SimConfig  # noqa: E402

N = 65536
MARKS = [2, 6, 11, 13, 16, 24, 40, 80, 160]
SAMPLE = 192                        # rows per half


def measure(mode):
    cfg = SimConfig(capacity=N, initial_nodes=N, init_mode=KB_INIT_CONVERGED, loss=0.05, partition_groups=2,
                    partition_start=3, partition_end=12, seed=9, failed_mode=mode)
    rng = np.random.default_rng(5)
    rows_a = np.sort(rng.choice(N // 2, SAMPLE, replace=False))
    rows_b = np.sort(rng.choice(N // 2, SAMPLE, replace=False)) + N // 2
    out = []
    with kaboodle_amd.Mesh(cfg) as m:
        r = 0
        for mark in MARKS:
            while r < mark:
                if r == 12:
                    for i in range(0, N, 256):
                        if m.is_running(i):
                            m.ping_addrs(i, [(i + N // 2) % N])
                m.step(1)
                r += 1
            ids_a = [i for i in rows_a if m.is_running(int(i))]
            ids_b = [i for i in rows_b if m.is_running(int(i))]
            ra = np.stack([m.row(int(i)) for i in ids_a])
            rb = np.stack([m.row(int(i)) for i in ids_b])
            allr = np.concatenate([ra, rb])
            mem = allr != 0
            base_g = mem.sum(0) * 2 > len(mem)
            base_a = (ra != 0).sum(0) * 2 > len(ra)
            base_b = (rb != 0).sum(0) * 2 > len(rb)
            exc_g = (mem != base_g[None, :]).sum(1)
            exc_p = np.concatenate([((ra != 0) != base_a[None, :]).sum(1), ((rb != 0) != base_b[None, :]).sum(1)])
            fresh = ((allr > 2)).sum(1)               # Known(t) inside the stamp window (self included)
            susp = (allr == 1).sum(1)
            st = m.stats()
            e = {"round": mark, "agree_frac": round(st["agree"] / max(st["alive"], 1), 4),
                 "view_size_mean": float(mem.sum(1).mean()),
                 "exceptions_vs_global_base": {"mean": float(exc_g.mean()), "max": int(exc_g.max())},
                 "exceptions_vs_partition_base": {"mean": float(exc_p.mean()), "max": int(exc_p.max())},
                 "base_sizes": {"global": int(base_g.sum()), "half_a": int(base_a.sum()), "half_b": int(base_b.sum())},
                 "non_ancient_stamps": {"mean": float(fresh.mean()), "max": int(fresh.max())},
                 "suspects": {"mean": float(susp.mean()), "max": int(susp.max())}}
            out.append(e)
            print(mode, json.dumps(e), flush=True)
    return out


def main():
    t0 = time.time()
    kaboodle_amd.require_gpu()
    res = {"tool": "tools/partition_divergence.py", "peers": N, "sampled_rows": 2 * SAMPLE,
           "scenario": "5% loss, 2 halves cut off for rounds 3-11, healed at round 12 (every 256th peer pings the other half)",
           "sim_sender": measure(KB_FAILED_SIM_SENDER), "socket_faithful": measure(KB_FAILED_SOCKET_FAITHFUL)}
    res["seconds"] = round(time.time() - t0, 1)
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "r03_partition_divergence.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
