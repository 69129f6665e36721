"""The sharded round's overhead on ONE MI355X: the configs[2] bench workload (64K peers, 1 % loss, 0.1 %/round
churn, latency on) as one mesh row-sharded over W rank PROCESSES that share the device and exchange every
delivery wave over the IPC transport (kb_ipc_unique_id), against the same mesh unsharded.

This is not a scaling measurement — every rank runs on the same GPU, so the work does not spread — it measures
what the sharded data path adds per round on one device: the per-wave count hand-offs to the host, the
all-to-all-v of records and KnownPeers ids, the broadcast-list all-gather, and W processes' kernels
interleaved on one device.  Every rank's results must equal the unsharded mesh's (the round's counters are
compared).

    python tools/ipc_ranks.py --worlds 1 2 4 --steps 20 --warmup 5 --out gpurun_out/ipc_ranks.json
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _args(ns):
    return argparse.Namespace(nodes=ns.nodes, loss=0.01, churn=0.001, seed=ns.seed, warmup=ns.warmup, steps=ns.steps,
                              replicas=False, weak=False, failed_mode="sim_sender", a3_order=ns.a3_order)


def _xbytes(lib, g):
    """bytes this rank's waves sent to other ranks (kb_sim_debug_counters[3]; 0 on builds without the counter)"""
    import ctypes as C
    buf = (C.c_uint64 * 5)()
    return int(buf[3]) if lib.lib.kb_sim_debug_counters(g.h, buf, 5) == 0 else 0


def _rank(rank, world, port, ns, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import parity
        from kaboodle_amd._ffi import Sim, ipc_unique_id
        lib = parity.gpu_lib()
        a = _args(ns)
        cfg = bench.rank_config(a, rank, world, 0)
        uid = bench.share_uid(rank, lambda: ipc_unique_id(lib))
        g = Sim(lib, cfg, rank=rank, world=world, uid=uid)
        g.step(a.warmup)
        g.stats()                                         # collective: drains the warmup
        s0, x0 = g.host_syncs(), _xbytes(lib, g)
        dist.barrier()
        t0 = time.perf_counter()
        g.step(a.steps)
        st = g.stats()                                    # collective; waits for the last round
        dt = time.perf_counter() - t0
        dist.barrier()
        q.put((rank, dt, g.host_syncs() - s0, st, None, _xbytes(lib, g) - x0))
        g.close()
    except Exception as e:  # noqa: BLE001 — reported to the parent
        q.put((rank, 0.0, 0, None, repr(e), 0))
    finally:
        dist.destroy_process_group()


def unsharded(ns):
    import bench
    import parity
    from kaboodle_amd._ffi import Sim
    lib = parity.gpu_lib()
    a = _args(ns)
    cfg = bench.rank_config(a, 0, 1, 0)
    with Sim(lib, cfg) as g:
        g.step(a.warmup)
        g.stats()
        s0 = g.host_syncs()
        t0 = time.perf_counter()
        g.step(a.steps)
        st = g.stats()
        dt = time.perf_counter() - t0
        return dt, g.host_syncs() - s0, st


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--a3-order", choices=("window", "exact"), default="exact")
    ap.add_argument("--out", default="")
    ns = ap.parse_args()
    import multiprocessing as mp
    res = {"workload": f"configs[2]: {ns.nodes} peers, converged start, 1% loss, 0.1%/round churn, latency on",
           "a3_order": ns.a3_order,
           "steps": ns.steps, "warmup": ns.warmup, "device": "one MI355X shared by every rank", "runs": {}}
    base = None
    for w in ns.worlds:
        if w == 1:
            dt, syncs, st = unsharded(ns)
            base = st
            res["runs"]["1"] = {"ms_per_round": round(1e3 * dt / ns.steps, 3), "host_syncs_per_round": syncs / ns.steps,
                                "transport": "none (unsharded)"}
        else:
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            port = _free_port()
            procs = [ctx.Process(target=_rank, args=(k, w, port, ns, q)) for k in range(w)]
            for p in procs:
                p.start()
            out = {}
            for _ in procs:
                rank, dt, syncs, st, err, xb = q.get(timeout=600)
                if err:
                    raise SystemExit(f"world {w} rank {rank}: {err}")
                out[rank] = (dt, syncs, st, xb)
            for p in procs:
                p.join(timeout=60)
            dts = [out[k][0] for k in range(w)]
            same = base is None or all(out[k][2] == base for k in range(w))
            res["runs"][str(w)] = {"ms_per_round": round(1e3 * max(dts) / ns.steps, 3),
                                   "host_syncs_per_round": out[0][1] / ns.steps, "transport": "IPC (kb_ipc_unique_id)",
                                   "bytes_to_other_ranks_per_round_per_rank": [round(out[k][3] / ns.steps) for k in range(w)],
                                   "counters_equal_unsharded": same}
            if not same:
                raise SystemExit(f"world {w}: counters differ from the unsharded mesh")
        print(w, json.dumps(res["runs"][str(w)]), flush=True)
    if ns.out:
        with open(ns.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
