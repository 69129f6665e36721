"""kb_sim_create_rank across PROCESSES on one MI355X.  RCCL refuses two ranks on one GPU, so the
ranks exchange over the IPC test transport (kb_ipc_unique_id: IPC-mapped device windows and a shared-memory
rendezvous) with the same collective discipline as RCCL: every rank makes the same mesh-changing calls and steps
and reads the counters together; row inspection is answered by the rank holding the row.  The unique id is made
on rank 0 and reaches the other rank over torch.distributed (gloo), as bench.py shares the RCCL id.

Two (or four) processes, each holding its share of the rows, must reproduce the oracle every round: counters, every fingerprint
and per-node scalar, whole rows, suspect and curious tables, and the broadcast lists — the reference's UDP
transport between instances (src/kaboodle.rs:188-226) carried between processes."""
import os
import socket

import numpy as np
import pytest

import parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {n: (c, r) for n, c, r in parity.standard_cases()}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case(name, sparse):
    case, rounds = CASES[name]
    if sparse:
        from kaboodle_amd._ffi import KB_VARIANT_SPARSE_ROWS
        case = parity.with_cfg(case, variant=KB_VARIANT_SPARSE_ROWS, track_latency=0)
    return case, rounds


def _rank_main(rank, world, port, name, q, sparse=False):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import parity as par
        from kaboodle_amd._ffi import Sim, ipc_unique_id
        lib = par.gpu_lib()
        uid = bench.share_uid(rank, lambda: ipc_unique_id(lib))
        case, rounds = _case(name, sparse)
        g = Sim(lib, case["cfg"], rank=rank, world=world, uid=uid)
        _, _, lo, hi = g.shard_info()
        par.setup(g, case)
        out = []
        for r in range(rounds):
            par.apply_events((g,), case, r)
            g.step(1)
            st = g.stats()                                   # collective: every rank reads the counters together
            rec = {"stats": st, "fps": g.fingerprints()[lo:hi].tolist(), "scalars": g.scalars()[lo:hi].tolist(),
                   "alive": g.scalars()[:, 0].tolist(), "bcasts": g.broadcasts(),
                   "rows": {i: g.row(i).tolist() for i in range(lo, hi)},
                   "susp": {i: g.suspects(i) for i in range(lo, hi)}, "cur": {i: g.curious(i) for i in range(lo, hi)}}
            out.append(rec)
        g.close()
        q.put((rank, lo, hi, out, None))
    except Exception as e:  # noqa: BLE001 — reported to the parent
        q.put((rank, 0, 0, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,world,sparse", [("churn_loss_512", 2, False), ("stop_start", 2, False),
                                               ("partition_heal", 2, False), ("fresh_ids", 2, False),
                                               ("identity_change", 2, False), ("churn_loss_512", 4, False),
                                               ("partition_heal", 4, False),
                                               # configs[4]'s sparse rows as rank processes
                                               ("churn_loss_512", 2, True), ("stop_start", 2, True)])
def test_processes_equal_oracle(name, world, sparse):
    import multiprocessing as mp
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    from kaboodle_amd._ffi import Sim
    case, rounds = _case(name, sparse)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(k, world, port, name, q, sparse)) for k in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, lo, hi, out, err = q.get(timeout=500)
        assert err is None, f"rank {rank}: {err}"
        res[rank] = (lo, hi, out)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = Sim(parity.oracle_lib(), case["cfg"])
    parity.setup(o, case)
    assert res[0][0] == 0 and res[world - 1][1] == case["cfg"].capacity                    # the rows, split in `world`
    assert all(res[k][1] == res[k + 1][0] for k in range(world - 1))
    for r in range(rounds):
        parity.apply_events((o,), case, r)
        o.step(1)
        so = parity.state_of(o)
        for rank, (lo, hi, out) in res.items():
            g = out[r]
            assert g["stats"] == so["stats"], f"{name} round {r} rank {rank}: counters differ"
            assert g["fps"] == so["fps"][lo:hi].tolist(), f"{name} round {r} rank {rank}: fingerprints differ"
            assert g["scalars"] == so["scalars"][lo:hi].tolist(), f"{name} round {r} rank {rank}: scalars differ"
            assert g["alive"] == so["scalars"][:, 0].tolist()
            assert [tuple(b) for b in g["bcasts"]] == [tuple(b) for b in so["bcasts"]], f"{name} round {r}: broadcast lists"
            for i in range(lo, hi):
                assert np.array_equal(np.asarray(g["rows"][i], np.uint8), so["rows"][i]), f"{name} round {r}: row {i}"
                assert [tuple(x) for x in g["susp"][i]] == so["susp"][i] and [tuple(x) for x in g["cur"][i]] == so["cur"][i]
    o.close()
