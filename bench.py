"""bench.py — simulated peer-rounds/s of the MI355X SWIM-round simulator (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--nodes 65536] [--loss 0.01] [--churn 0.001]

Workload (BASELINE.json configs[2]): 65,536 simulated Kaboodle peers on one MI355X, started converged,
1% per-delivery loss and 0.1%/round churn (leaves + joins with fresh ids).  A "step" is one complete
simulated round (lifecycle, broadcasts, tick A1-A4 for every live peer, and all receive waves) through
the C ABI `kb_sim_step`; the timed region holds K steps with all state resident in HBM.

value = live peers x rounds / max-over-ranks wall time, for the whole job.
N > 1 (torchrun, one process per GPU): the same `nodes`-peer mesh row-sharded across the N GPUs
(kb_sim_create_rank): every delivery wave is an RCCL all-to-all-v of the records between
shards and the Join/Failed lists an all-gather.  Strong scaling: the workload is fixed (configs[2]) and
each GPU holds nodes/N rows.  --weak makes `nodes` the rows per GPU (a mesh of nodes x N peers, e.g.
configs[3]: --weak --nodes 131072 on 8 GPUs = 1M peers); its rows get wider with N, because every peer
tracks every peer, so per-GPU work grows with N.  --replicas runs N independent meshes instead
(distinct seeds, no collective on the data path).

Also reported, on the same JSON line:
  kernels       every kernel of the round: HIP-event ms per round (each launch timed by its own dispatch
                packet on the simulator's stream), launches per round, wave-0 share, and for the kernels
                with an in-kernel byte counter (k_rowpass, k_fold, k_resp_wave, k_proc) the algorithmic
                bytes and GB/s.  The timed rounds carry events on the three once-per-round ones only (an
                event pair costs ≈5 us of dispatch overhead; k_proc's eight launches a round would add
                ≈0.05 ms); the other kernels' times, k_proc's included, come from an untimed replay of
                the same rounds (same seed: the simulation is deterministic, bit for bit) with events on
                every launch.  The kernels the simulator runs on its side stream, beside the Join responses
                (SIDE_KERNELS, marked "stream": "side"), overlap the round's other kernels and are left out of
                the sum; `gaps` = round_gpu_ms minus the other kernels (launch gaps, host hand-offs, and what
                the overlap costs them), so those rows sum to round_gpu_ms;
  roofline      the kernel with the most time per round: algorithmic bytes per launch (counted in-kernel)
                / its mean HIP-event launch duration, against 8 TB/s; `traffic` = measured HBM bytes per
                launch from the rocprofv3 PMC summary committed under profiles/ for this exact command
                (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, timed rounds only), else null;
  cpu_baseline  the CPU oracle (oracle/, OpenMP build, same semantics and seeds) on a bounded sample of
                the same workload, on rank 0 only; `single_thread`: the same oracle on one thread for the
                rounds that follow;
  seeds         seeds 2 and 3 of the same workload, timed the same way (N = 1);
  convergence   after the timed rounds faults stop (fault_end_round); untimed rounds continue until every
                live peer's fingerprint equals the fingerprint of the true live set (or a cap).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md "HBM [CDNA4]")
LAT_TABLE_MAX = 64 << 30        # bytes of latency table per GPU beyond which --latency is dropped
KT_ROUND = 1                    # kb_sim_kernel_time kind of the whole round
# kernels on the simulator's side stream (kb_sim.hip step_round: side_fork / side_join), overlapping the round's
SIDE_KERNELS = ("k_alive_bits", "k_truefp_part", "k_truefp_fin", "k_lat_sweep", "k_a3_exact")
CHURN_RESERVE = 8192            # fresh ids kept for churn joins: capacity does not depend on --steps


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=65536, help="peers of the mesh (per GPU with --weak)")
    ap.add_argument("--weak", action="store_true", help="N > 1: nodes rows per GPU, a mesh of nodes x N peers")
    ap.add_argument("--replicas", action="store_true", help="N > 1: independent meshes instead of one sharded mesh")
    ap.add_argument("--rank-mesh", action="store_true",
                    help="N = 1: run the mesh through the RCCL rank path (a 1-rank communicator) to check it")
    ap.add_argument("--loss", type=float, default=0.01)
    ap.add_argument("--churn", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--conv-cap", type=int, default=100, help="max untimed quiescent rounds for convergence")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--cpu1-seconds", type=float, default=15.0, help="single-thread CPU sample budget (0: skip)")
    ap.add_argument("--seeds", default="2,3", help="extra seeds of the same workload timed the same way (N = 1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="do not keep PeerInfo.latency (track_latency 0)")
    ap.add_argument("--no-conv", action="store_true")
    ap.add_argument("--no-replay", action="store_true", help="skip the profiled replay (kernel breakdown)")
    ap.add_argument("--no-modes", action="store_true", help="skip the socket_faithful line (N = 1)")
    ap.add_argument("--failed-mode", choices=("sim_sender", "socket_faithful"), default="sim_sender",
                    help="Q1: Failed(p) honoured (sim_sender, the headline) or never (socket_faithful)")
    ap.add_argument("--a3-order", choices=("window", "exact"), default="exact",
                    help="A3's five oldest: the reference's exact instants (exact, the default: KB_VARIANT_EXACT_LRU, "
                         "src/kaboodle.rs:662-675) or the 1-byte stamp window with a sweep front (window, the declared "
                         "deviation of DESIGN.md §2.11)")
    return ap.parse_args(argv)


def lib_sha16() -> str:
    import hashlib
    import kaboodle_amd
    return hashlib.sha256(open(kaboodle_amd.LIB_PATH, "rb").read()).hexdigest()[:16]


def same_build(d: dict) -> bool:
    """A record made with this library: the same binary (lib_sha16), or the same sources and build command
    (lib_src_sha16, kaboodle_amd/build.py: a rebuild of unchanged sources is not byte-identical).  An A/B build
    loaded through KB_LIB_PATH matches by its binary only."""
    import kaboodle_amd
    from kaboodle_amd import build as kb_build
    if d.get("lib_sha16") == lib_sha16():
        return True
    return (os.path.abspath(kaboodle_amd.LIB_PATH) == os.path.abspath(kb_build.OUT) and d.get("lib_src_sha16") is not None
            and d.get("lib_src_sha16") == kb_build.src_sha16())


def pmc_summary(cfg_key: str, capacity: int, steps: int, warmup: int, failed_mode: str, a3_order: str):
    """The latest committed PMC summary (tools/gpu_measure.sh -> profiles/*pmc*.json) taken on exactly this
    workload, capacity, step and warmup counts, with this very library build (lib_sha16): {kernel:
    {hbm_bytes_per_launch, hbm_bytes_per_round, ...}} over the timed rounds, and the summary's path."""
    best, src = None, None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if (d.get("workload") == cfg_key and d.get("capacity") == capacity and d.get("steps") == steps and
                d.get("warmup") == warmup and d.get("failed_mode", "sim_sender") == failed_mode and "kernels" in d
                and d.get("a3_order", "window") == a3_order
                and same_build(d)):
            best, src = d["kernels"], os.path.relpath(p, ROOT)
    return best, src


def committed_tail(cfg_key: str, mode: str, a3_order: str = "window"):
    """The full quiescent tail of this workload (tools/converge.py, run to agreement or a cap of 2-4 N rounds
    on an MI355X; profiles/*converge*.json): too long for the bench's minutes, so read from the record —
    only a record made with this very library build (lib_sha16), like pmc_summary.  a3_order "exact": the
    same tail with A3 in the reference's exact-instant order (KB_VARIANT_EXACT_LRU)."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*converge*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if (d.get("workload", "").startswith(cfg_key) and d.get("failed_mode") == mode and same_build(d)
                and d.get("a3_order", "window") == a3_order):
            best = {k: d[k] for k in ("converged_round", "tail_rounds_to_converge", "tail_rounds_run", "cap_rounds",
                                      "stopped_by") if k in d}
            best["source"] = os.path.relpath(p, ROOT)
            samples = [t for t in d.get("trajectory", []) if "agree_frac" in t]
            if samples:
                best["final_agree_frac"] = samples[-1]["agree_frac"]
                best["final_view_gap_mean"] = samples[-1]["view_gap_mean"]
    return best


def timed_rounds(mesh, steps: int, world: int):
    """Steps `steps` rounds between barriers; returns (wall s, sum of live peers over the rounds, stats
    before, stats after)."""
    import torch
    import torch.distributed as dist
    s0 = mesh.stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        mesh.step(1)                                 # synchronous: returns after the round's kernels
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    s1 = mesh.stats()                                # sharded: the whole mesh (collective)
    # live peers of every simulated round, counted on the device during the round (kb_stats.alive_rounds)
    return dt, s1["alive_rounds"] - s0["alive_rounds"], s0, s1


def round_model_bytes(s0: dict, s1: dict, alive_mean: float, steps: int) -> float:
    """SURVEY.md §8(d)'s dense per-round model: every live peer reads its row of the stamp table
    (N bytes), plus 32 B per message record and 4 B per KnownPeers entry moved."""
    msgs = sum(s1[k] - s0[k] for k in ("sent_ping", "sent_ping_req", "sent_ack", "sent_known_peers", "sent_kpr"))
    ids = s1["sent_kp_ids"] - s0["sent_kp_ids"]
    return (alive_mean * alive_mean * steps + 32.0 * msgs + 4.0 * ids) / steps


def cpu_baseline(cfg, budget_s: float, nodes: int, budget_1t: float) -> dict:
    """The OpenMP oracle on a bounded sample of the same workload (rank 0, N=1 only); then the same oracle
    restricted to one thread on the rounds that follow (BASELINE.md's single-thread CPU figure)."""
    import ctypes as C
    from kaboodle_amd._ffi import Sim
    so = os.path.join(ROOT, "oracle", "_build", "libkb_oracle_omp.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from kaboodle_amd._ffi import SimLib
    lib = SimLib(so, "kbo_")
    lib.lib.kbo_num_threads.restype = C.c_int
    cores = int(lib.lib.kbo_num_threads())

    def sample(o, budget, cap, least=1):
        t0 = time.perf_counter()
        rounds, alive_sum = 0, 0
        while True:
            o.step(1)
            rounds += 1
            alive_sum += o.stats()["alive"]
            if (time.perf_counter() - t0 >= budget and rounds >= least) or rounds >= cap:
                return rounds, alive_sum, time.perf_counter() - t0

    with Sim(lib, cfg) as o:
        o.step(1)                                # one warmup round (first touch of the dense table)
        rounds, alive_sum, dt = sample(o, budget_s, 200)
        one = None
        if budget_1t > 0:
            lib.lib.kbo_set_num_threads(1)
            r1, a1, dt1 = sample(o, budget_1t, 50, least=3)   # at least 3 rounds (~17 s each at 64K)
            lib.lib.kbo_set_num_threads(cores)
            one = {"value": a1 / dt1, "unit": "peer-rounds/s", "cores": 1,
                   "sample": f"the next {r1} rounds of the same run on one thread ({dt1:.1f} s)"}
    return {"value": alive_sum / dt, "unit": "peer-rounds/s", "cores": cores, "kind": "port",
            "sample": f"{rounds} rounds of the same {nodes}-peer workload after 1 warmup round "
                      f"(oracle/kb_oracle.c, OpenMP over peers, {dt:.1f} s)",
            "single_thread": one}


def sharded(a, world: int) -> bool:
    return (world > 1 and not getattr(a, "replicas", False)) or getattr(a, "rank_mesh", False)


def rank_config(a, rank: int, world: int, local: int):
    """This rank's mesh: one mesh of nodes x world peers shared by every rank (sharded), or a replica of
    the nodes-peer workload with a rank-distinct seed (world 1, --replicas)."""
    from kaboodle_amd._ffi import KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, SimConfig
    total = a.warmup + a.steps
    shard = sharded(a, world)
    peers = a.nodes * world if (shard and getattr(a, "weak", False)) else a.nodes
    reserve = max(CHURN_RESERVE, int(peers * a.churn * (total + 8) * 1.5))   # 8192 up to ~80 churn rounds at 64K
    from kaboodle_amd._ffi import KB_VARIANT_EXACT_LRU
    mode = KB_FAILED_SOCKET_FAITHFUL if getattr(a, "failed_mode", "sim_sender") == "socket_faithful" else KB_FAILED_SIM_SENDER
    return SimConfig(capacity=peers + reserve, initial_nodes=peers, init_mode=KB_INIT_CONVERGED, loss=a.loss,
                     churn=a.churn, fault_end_round=total, seed=a.seed + (0 if shard else 1000 * rank),
                     device=local if world > 1 else -1, failed_mode=mode,
                     track_latency=int(latency_on(a, peers + reserve, world if shard else 1)),
                     variant=KB_VARIANT_EXACT_LRU if getattr(a, "a3_order", "window") == "exact" else 0)


def latency_on(a, capacity: int, shards: int) -> bool:
    """PeerInfo.latency is kept (as the reference always does, src/kaboodle.rs:789-817) unless --no-latency,
    or unless its table (2 B per row x id) would take more than LAT_TABLE_MAX of one GPU's HBM (configs[3]:
    131K rows x 1M ids = 275 GB on top of the stamps)."""
    rows = -(-capacity // shards)
    width = -(-capacity // 8192) * 8192
    return not getattr(a, "no_latency", False) and 2 * rows * width <= LAT_TABLE_MAX


def share_uid(rank: int, make) -> bytes:
    """Rank 0 makes the RCCL unique id of the mesh's communicator; every rank receives it."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return make()
    obj = [make() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def aggregate(dt: float, units: float, world: int, device="cpu"):
    """Whole-job numbers: max wall time over ranks, units summed over ranks."""
    if world == 1:
        return dt, units
    import torch
    import torch.distributed as dist
    t = torch.tensor([dt, units], dtype=torch.float64, device=device)
    tm = t[:1].clone()
    tu = t[1:].clone()
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    dist.all_reduce(tu, op=dist.ReduceOp.SUM)
    return float(tm[0]), float(tu[0])


def main() -> int:
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    import kaboodle_amd
    from kaboodle_amd._ffi import SimConfig
    kaboodle_amd.require_gpu()

    total = a.warmup + a.steps
    shard = sharded(a, world)
    cfg = rank_config(a, rank, world, local)
    capacity = cfg.capacity
    peers = cfg.initial_nodes
    workload = f"configs[2]: {a.nodes} peers, converged start, {a.loss:.0%} loss, {a.churn:.1%}/round churn"
    if shard:
        weak = getattr(a, "weak", False)
        workload = (f"{'configs[2] per GPU' if weak else 'configs[2]'}, one mesh: {peers} peers row-sharded "
                    f"{(peers + world - 1) // world}/GPU over {world} GPUs, "
                    f"converged start, {a.loss:.0%} loss, {a.churn:.1%}/round churn")
        mesh = kaboodle_amd.Mesh(cfg, rank=rank, world=world, uid=share_uid(rank, kaboodle_amd.rccl_unique_id))
    else:
        mesh = kaboodle_amd.Mesh(cfg)

    mesh.step(a.warmup)
    torch.cuda.synchronize()
    mesh.reset_kernel_time()
    syncs0 = mesh.host_syncs()
    dt, alive_sum, st0, st = timed_rounds(mesh, a.steps, world)
    syncs = mesh.host_syncs() - syncs0
    bd = mesh.kernel_breakdown()
    round_ms, round_n = mesh.kernel_time(KT_ROUND)
    model_bytes = round_model_bytes(st0, st, alive_sum / max(a.steps, 1), a.steps)

    # sharded: every rank saw the whole mesh's count, so it enters the sum once
    dt, alive_total = aggregate(dt, float(alive_sum if (rank == 0 or not shard) else 0), world, device="cuda")

    conv = None
    if not a.no_conv:
        # (1) BASELINE configs[1]: 1024 peers all joining at round 0, no faults -> rounds to convergence
        r2 = -1
        if rank == 0 or not shard:
            with kaboodle_amd.Mesh(SimConfig(capacity=1024, initial_nodes=1024, seed=a.seed + 1000 * rank,
                                             device=local if world > 1 else -1)) as m2:
                for _ in range(64):
                    m2.step(1)
                    s2 = m2.stats()
                    if s2["first_converged_round"] >= 0:
                        r2 = s2["first_converged_round"]
                        break
        # (2) this workload's quiescent tail: faults ended at round `total`; step untimed until every live
        # peer agrees or the cap (Q2 + honoured Failed remove live peers mesh-wide)
        r_conv, extra = -1, 0
        while r_conv < 0 and extra < a.conv_cap:
            mesh.step(1)
            extra += 1
            s3 = mesh.stats()
            if s3["agree"] == s3["alive"]:
                r_conv = s3["round"] - 1
        s3 = mesh.stats()
        conv = {"config2_join_1k_converged_round": r2 if r2 >= 0 else None,
                "workload_fault_end_round": total,
                "workload_converged_round": r_conv if r_conv >= 0 else None,
                "workload_tail_rounds_run": extra,
                "workload_agree_frac_at_fault_end": round(st["agree"] / max(st["alive"], 1), 4),
                "workload_agree_frac_final": round(s3["agree"] / max(s3["alive"], 1), 4),
                "workload_full_tail": committed_tail(f"configs[2]: {a.nodes} peers", a.failed_mode, a.a3_order)}
        if not shard:
            # how far the views are from agreement: |known_i| against the running count (0 = right size)
            import numpy as np
            sc = mesh.scalars()
            live = sc[:, 0] != 0
            gap = np.abs(sc[live, 1].astype(np.int64) - int(live.sum()))
            conv["workload_view_size_match_frac_final"] = round(float((gap == 0).mean()), 4)
            conv["workload_view_size_mean_gap_final"] = round(float(gap.mean()), 2)

    # every kernel's time: an untimed replay of the same rounds (deterministic) with events on every launch
    if world == 1 and not a.no_replay:
        mesh.close()
        with kaboodle_amd.Mesh(cfg) as rp:
            rp.set_profiling(2)
            rp.step(a.warmup)
            rp.reset_kernel_time()
            rp.step(a.steps)
            for name, k in rp.kernel_breakdown().items():
                if name not in bd:
                    bd[name] = k

    out = None
    if rank == 0:
        nr = max(round_n, 1)
        pmc, pmc_src = pmc_summary(workload, capacity, a.steps, a.warmup, a.failed_mode, a.a3_order)
        table = {}
        for name, k in sorted(bd.items(), key=lambda kv: -kv[1]["ms"]):
            e = {"ms_per_round": round(k["ms"] / nr, 4), "launches_per_round": round(k["launches"] / nr, 2),
                 "wave0_ms_per_round": round(k["wave_ms"][0] / nr, 4)}
            if k["bytes"] is not None and k["launches"]:
                per_launch = k["bytes"] / k["launches"]
                avg_ms = k["ms"] / k["launches"]
                ach = per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
                e.update({"algorithmic_bytes_per_launch": int(per_launch), "avg_launch_ms": round(avg_ms, 4),
                          "achieved_GBs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4)})
            if pmc and name in pmc:
                e["traffic_per_launch"] = pmc[name].get("hbm_bytes_per_launch")
            table[name] = e
        for name in SIDE_KERNELS:
            if name in table:
                table[name]["stream"] = "side"
        kern_sum = sum(v["ms_per_round"] for n, v in table.items() if n not in SIDE_KERNELS)
        gaps = round(round_ms / nr - kern_sum, 4)
        counted = [n for n, v in table.items() if "achieved_GBs" in v]
        # the critical-path kernel: side-stream kernels overlap others, and their event spans stretch with them
        top = max((n for n in table if n not in SIDE_KERNELS), key=lambda n: table[n]["ms_per_round"])
        dominant = top if top in counted else max(counted, key=lambda n: table[n]["ms_per_round"])
        dk, db = table[dominant], bd[dominant]
        roof = {"bound": "hbm", "kernel": dominant, "achieved": dk["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dk["frac"], "traffic": dk.get("traffic_per_launch"),
                "traffic_source": pmc_src if dk.get("traffic_per_launch") is not None else None,
                "algorithmic_bytes_per_launch": dk["algorithmic_bytes_per_launch"], "avg_launch_ms": dk["avg_launch_ms"],
                "launches": db["launches"], "ms_per_round": dk["ms_per_round"],
                "note": None if top == dominant else f"{top} takes more time per round but has no byte counter"}
        out = {
            "metric": "simulated peer-rounds/sec (whole node) + rounds to fingerprint convergence",
            "value": alive_total / dt, "unit": "peer-rounds/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak" if (getattr(a, "weak", False) or (world > 1 and not shard)) else "strong",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (Philox-keyed loss/churn/targets, seed-determined)",
            "config": {"workload": workload, "failed_mode": a.failed_mode, "a3_order": a.a3_order, "peers": peers, "peers_per_gpu": (peers + world - 1) // world if shard else peers,
                       "capacity": capacity,
                       "loss": a.loss, "churn": a.churn,
                       "parallelism": (f"rowshard{world}" if shard else f"replicas{world}") if world > 1 else "single",
                       "max_waves": cfg.max_waves, "latency_ewma": bool(cfg.track_latency)},
            "roofline": roof,
            "kernels": {**table, "gaps": {"ms_per_round": gaps}},
            "round_gpu_ms": round(round_ms / nr, 4),
            "host_syncs_per_round": round(syncs / max(a.steps, 1), 2),
            # the whole round against SURVEY.md §8(d)'s dense model (every live peer reads its N-byte
            # row, plus the message bytes), per wall-clock round
            "round_roofline": {"bytes_model_per_round": int(model_bytes),
                               "achieved": round(model_bytes / (dt / a.steps) / 1e9, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(model_bytes / (dt / a.steps) / 1e9 / HBM_PEAK_GBS, 4)},
            "convergence": conv,
        }
        if world == 1 and not a.no_cpu:
            ccfg = SimConfig(**{**cfg.__dict__, "device": -1})
            out["cpu_baseline"] = cpu_baseline(ccfg, a.cpu_seconds, a.nodes, a.cpu1_seconds)
        else:
            out["cpu_baseline"] = None
    mesh.close()
    modes = None
    if world == 1 and not a.no_modes and a.failed_mode == "sim_sender":
        # Q1's deployment-faithful reading (Failed never honoured, src/networking.rs:44-55): same
        # workload, seeds, K and W, its own mesh; timed the same way
        import copy
        b = copy.copy(a)
        b.failed_mode = "socket_faithful"
        with kaboodle_amd.Mesh(rank_config(b, rank, world, local)) as m2:
            m2.step(a.warmup)
            torch.cuda.synchronize()
            dt2, alive2, s20, s21 = timed_rounds(m2, a.steps, world)
            rb2 = round_model_bytes(s20, s21, alive2 / max(a.steps, 1), a.steps)
            modes = {"socket_faithful": {
                "value": alive2 / dt2, "ms_per_step": dt2 / a.steps * 1e3,
                "round_model_frac": round(rb2 / (dt2 / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "agree_frac_at_fault_end": round(s21["agree"] / max(s21["alive"], 1), 4),
                "workload_full_tail": committed_tail(f"configs[2]: {a.nodes} peers", "socket_faithful", b.a3_order),
                "workload_full_tail_" + ("window" if b.a3_order == "exact" else "exact_lru"):
                    committed_tail(f"configs[2]: {a.nodes} peers", "socket_faithful",
                                   "window" if b.a3_order == "exact" else "exact")}}
        # the other A3 order on the same workload, seeds, K and W: the reference's exact instants
        # (src/kaboodle.rs:662-675) against the 1-byte window, each kernel of its round from a profiled replay
        other = "window" if a.a3_order == "exact" else "exact"
        c = copy.copy(a)
        c.a3_order = other
        ccfg4 = rank_config(c, rank, world, local)
        with kaboodle_amd.Mesh(ccfg4) as m4:
            m4.step(a.warmup)
            torch.cuda.synchronize()
            dt4, alive4, s40, s41 = timed_rounds(m4, a.steps, world)
        ms_head = dt / a.steps * 1e3
        ent = {"value": alive4 / dt4, "ms_per_step": dt4 / a.steps * 1e3,
               "cost_vs_headline": round(dt4 / a.steps * 1e3 / ms_head, 3),
               "agree_frac_at_fault_end": round(s41["agree"] / max(s41["alive"], 1), 4),
               "workload_full_tail_socket_faithful": committed_tail(f"configs[2]: {a.nodes} peers", "socket_faithful", other)}
        if not a.no_replay:
            with kaboodle_amd.Mesh(ccfg4) as rp4:
                rp4.set_profiling(2)
                rp4.step(a.warmup)
                rp4.reset_kernel_time()
                rp4.step(a.steps)
                kb4 = rp4.kernel_breakdown()
                rms4, rn4 = rp4.kernel_time(KT_ROUND)
            ent["round_gpu_ms"] = round(rms4 / max(rn4, 1), 4)
            ent["kernels_ms_per_round"] = {n: round(k["ms"] / max(rn4, 1), 4)
                                           for n, k in sorted(kb4.items(), key=lambda kv: -kv[1]["ms"])[:12]}
        modes["exact_lru" if other == "exact" else "window"] = ent
    seeds = None
    if world == 1 and a.seeds:
        # seeds 2 and 3 of the same synthetic workload, same K and W, each its own mesh
        import copy
        seeds = {}
        for sd in (int(x) for x in a.seeds.split(",") if x.strip()):
            b = copy.copy(a)
            b.seed = sd
            with kaboodle_amd.Mesh(rank_config(b, rank, world, local)) as m3:
                m3.step(a.warmup)
                torch.cuda.synchronize()
                dt3, alive3, _, s31 = timed_rounds(m3, a.steps, world)
                seeds[str(sd)] = {"value": alive3 / dt3, "ms_per_step": dt3 / a.steps * 1e3,
                                  "agree_frac_at_fault_end": round(s31["agree"] / max(s31["alive"], 1), 4)}
    if out is not None:
        out["modes"] = modes
        out["seeds"] = seeds
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
