"""Large single-GPU meshes (configs[3]'s per-GPU footprint): time rounds and record
per-round digests of an unsharded mesh, or of the same mesh as k LocalXfer row shards, so the two runs can
be compared after the fact (both cannot be resident at once at ~372K peers: ~160 GB each).

    python tools/big_mesh.py --nodes 372736 --rounds 6 [--shards 8] [--dbg 31] --out gpurun_out/big.json

Per round: wall ms, the round's GPU ms (HIP events), counters, and a digest = sha256 over every
fingerprint, the per-node scalars and the counters.  At the end: sampled rows (stamp bytes digested) and
the generate_fingerprint of each sampled row's peers() against its fingerprint (src/kaboodle.rs:71-83)."""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def digest(m) -> str:
    h = hashlib.sha256()
    h.update(m.fingerprints().tobytes())
    h.update(m.scalars().tobytes())
    h.update(json.dumps(m.stats(), sort_keys=True).encode())
    return h.hexdigest()[:16]


def fp_of_set(ids) -> int:
    import kaboodle_amd
    f = kaboodle_amd.lib().lib.kb_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    a = np.ascontiguousarray(np.asarray(ids, dtype=np.uint32))
    return int(f(a.ctypes.data_as(C.POINTER(C.c_uint32)), len(a), None, 0, None))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=372736)
    ap.add_argument("--reserve", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--loss", type=float, default=0.01)
    ap.add_argument("--churn", type=float, default=0.0001)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--shards", type=int, default=0)
    ap.add_argument("--dbg", type=int, default=0)
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--prof", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import kaboodle_amd
    from kaboodle_amd._ffi import KB_INIT_CONVERGED, SimConfig
    kaboodle_amd.require_gpu()
    cfg = SimConfig(capacity=a.nodes + a.reserve, initial_nodes=a.nodes, init_mode=KB_INIT_CONVERGED, loss=a.loss,
                    churn=a.churn, seed=a.seed, debug_flags=a.dbg)
    t0 = time.perf_counter()
    m = kaboodle_amd.Mesh(cfg, shards=a.shards)
    m.set_profiling(a.prof) if not a.shards else None
    rec = {"nodes": a.nodes, "capacity": cfg.capacity, "shards": a.shards, "dbg": a.dbg, "loss": a.loss,
           "churn": a.churn, "seed": a.seed, "create_s": round(time.perf_counter() - t0, 2), "rounds": []}
    print(f"created {cfg.capacity} ids, shards {a.shards}: {rec['create_s']} s", flush=True)
    for r in range(a.rounds):
        if not a.shards:
            m.reset_kernel_time()
        t1 = time.perf_counter()
        m.step(1)
        wall = (time.perf_counter() - t1) * 1e3
        st = m.stats()
        e = {"round": r, "wall_ms": round(wall, 2), "digest": digest(m), "alive": st["alive"], "agree": st["agree"],
             "removed_failed": st["removed_failed"], "join_responses": st["join_responses"],
             "sent_kp_ids": st["sent_kp_ids"]}
        if not a.shards:
            e["gpu_ms"] = round(m.kernel_time(1)[0], 2)
            e["kernels"] = {k: round(v["ms"], 3) for k, v in sorted(m.kernel_breakdown().items(), key=lambda kv: -kv[1]["ms"])}
            e["rowpass_bytes"] = m.kernel_bytes(0)
        rec["rounds"].append(e)
        print(json.dumps(e), flush=True)
    rng = np.random.default_rng(a.seed)
    rows = {}
    fps = m.fingerprints()
    for i in sorted(int(x) for x in rng.choice(a.nodes, a.rows, replace=False)):
        row = m.row(i)
        p = m.peers(i)
        ok = not m.is_running(i) or fp_of_set(p) == int(fps[i])
        rows[str(i)] = {"sha": hashlib.sha256(row.tobytes()).hexdigest()[:16], "n": len(p), "fp_ok": bool(ok)}
    rec["rows"] = rows
    rec["paths"] = m.debug_paths()
    m.close()
    print(json.dumps({"rows": rows, "paths": rec["paths"]}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(rec, open(a.out, "w"), indent=1)
    return 0 if all(v["fp_ok"] for v in rows.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
