"""The N > 1 bench path on CPU: world_size-2 gloo process groups (127.0.0.1).  Each rank runs its
replica of the workload (here through the CPU oracle, since there is no GPU in this container), timed as
bench.py times it (barrier, the steps, barrier), and the whole-job numbers are reduced exactly as bench.py does
on RCCL: max wall time, summed peer-rounds.  The GPU exchange between rank processes is tests/test_gpu_multiproc.py."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import argparse
    import bench
    import parity
    from kaboodle_amd._ffi import Sim
    a = argparse.Namespace(nodes=96, loss=0.02, churn=0.01, seed=1, warmup=1, steps=4, replicas=True)
    cfg = bench.rank_config(a, rank, world, rank)
    with Sim(parity.oracle_lib(), cfg) as o:
        o.step(a.warmup)
        units = 0
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps * (1 + 2 * rank)):       # rank 1 does three times the work: the max must be its time
            o.step(1)
            units += o.stats()["alive"]
        dist.barrier()
        dt = time.perf_counter() - t0
        mine = dt
        fps = o.fingerprints().tolist()
    tot_dt, tot_units = bench.aggregate(dt, float(units), world)
    out[rank] = (cfg.seed, units, tot_dt, tot_units, fps[:8], mine)
    dist.barrier()
    dist.destroy_process_group()


def test_replicas_reduce_like_bench():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    (s0, u0, dt0, tu0, fp0, m0), (s1, u1, dt1, tu1, fp1, m1) = out[0], out[1]
    assert s0 != s1                                     # distinct replicas
    assert fp0 != fp1
    assert dt0 == dt1 == max(m0, m1) > 0                # max over ranks of the measured times
    assert tu0 == tu1 == float(u0 + u1)                 # summed units


def _shard_worker(rank, world, port, out):
    """The sharded bench setup on gloo: the RCCL id made on rank 0 reaches every rank, and every rank
    derives the same mesh (capacity, seed) of nodes x world peers."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import argparse
    import bench
    a = argparse.Namespace(nodes=96, loss=0.01, churn=0.001, seed=5, warmup=2, steps=3, replicas=False, weak=False)
    uid = bench.share_uid(rank, lambda: bytes(range(128)))
    cfg = bench.rank_config(a, rank, world, rank)
    ra = argparse.Namespace(**{**a.__dict__, "replicas": True})
    rcfg = bench.rank_config(ra, rank, world, rank)
    wa = argparse.Namespace(**{**a.__dict__, "weak": True})
    wcfg = bench.rank_config(wa, rank, world, rank)
    out[rank] = (uid, cfg.capacity, cfg.initial_nodes, cfg.seed, rcfg.initial_nodes, rcfg.seed,
                 bench.sharded(a, world), bench.sharded(ra, world), wcfg.initial_nodes, wcfg.seed)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_setup_over_gloo():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_shard_worker, args=(world, port, out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    assert r0[0] == r1[0] == bytes(range(128))          # rank 0's id on every rank
    assert r0[1:4] == r1[1:4]                            # one mesh: same capacity, size and seed
    assert r0[2] == 96                                   # strong: the same mesh split over the ranks
    assert r0[8] == r1[8] == 96 * world and r0[9] == r1[9]  # --weak: nodes rows per rank, one mesh
    assert r0[4] == r1[4] == 96 and r0[5] != r1[5]        # replicas: per-rank mesh, distinct seeds
    assert r0[6] and not r0[7]
