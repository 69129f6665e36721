"""Small scenarios shared by the pyref pin, the golden round-trace fixtures and the CPU tests.

Each scenario is plain data: a SimConfig, the rounds to run, identities/starts applied before round 0 and
per-round API events (applied before that round's step, in list order).  `pymesh_of` builds the
equivalent tests/pyref.py mesh so the same scenario drives the independent Python restatement.
"""
from __future__ import annotations

import zlib

import numpy as np

from kaboodle_amd._ffi import KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, Sim, SimConfig

CONFIG1_IDS = [b"top-left", b"top-right", b"bottom-left", b"bottom-right"]   # 2x2-layout.kdl:6-20


def _sc(name, cfg, rounds, identities=None, start=(), events=None):
    return {"name": name, "cfg": cfg, "rounds": rounds, "identities": identities or {}, "start": list(start),
            "events": events or {}}


SCENARIOS = [
    _sc("config1", SimConfig(capacity=4, initial_nodes=0), 6,
        identities={i: n for i, n in enumerate(CONFIG1_IDS)}, start=[0, 1, 2, 3]),
    _sc("join32", SimConfig(capacity=32, initial_nodes=32, seed=3), 8),
    _sc("conv_loss48", SimConfig(capacity=48, initial_nodes=48, init_mode=KB_INIT_CONVERGED, seed=7, loss=0.08), 30),
    _sc("churn40", SimConfig(capacity=60, initial_nodes=40, init_mode=KB_INIT_CONVERGED, seed=5, loss=0.03,
                             churn=0.03, fault_end_round=20), 35),
    _sc("join_loss_ids", SimConfig(capacity=40, initial_nodes=40, seed=9, loss=0.05, id_len=7), 20),
    _sc("socket_faithful", SimConfig(capacity=30, initial_nodes=30, init_mode=KB_INIT_CONVERGED, seed=2, loss=0.1,
                                     failed_mode=KB_FAILED_SOCKET_FAITHFUL), 20),
    _sc("partition", SimConfig(capacity=32, initial_nodes=32, init_mode=KB_INIT_CONVERGED, seed=4, loss=0.02,
                               partition_groups=2, partition_start=3, partition_end=10), 25,
        events={10: [("ping", i, [(i + 16) % 32]) for i in range(0, 32, 4)]}),
    # a stopped instance restarts at a fresh address (src/kaboodle.rs:138-152) with its map (src/lib.rs:104):
    # 3 comes back as id 20, the first fresh id; 22 is a first start
    _sc("stop_start", SimConfig(capacity=24, initial_nodes=20, init_mode=KB_INIT_CONVERGED, seed=6), 15,
        events={2: [("stop", 3, None)], 4: [("start", 22, None)], 8: [("restart", 3, None)]}),
    _sc("rebase", SimConfig(capacity=24, initial_nodes=24, init_mode=KB_INIT_CONVERGED, seed=8, loss=0.02,
                            churn=0.01), 140),
    _sc("waves2", SimConfig(capacity=40, initial_nodes=40, seed=13, loss=0.03, max_waves=2), 15),
    _sc("trunc_join", SimConfig(capacity=700, initial_nodes=700, seed=21), 3),
    # Join responses truncated from views of ~1200 ids: an odd permutation width (11 bits)
    _sc("trunc_odd", SimConfig(capacity=1300, initial_nodes=1200, init_mode=KB_INIT_CONVERGED, churn=0.01, seed=23), 3),
    # early joiners' KnownPeers inserts are stamped before round 0 (Known(r - 10), r < 10); three stamp-window
    # rebases later (rounds 64, 128, 192) they sit at the bottom of the window: the saturation edge of k_rebase
    _sc("old_stamps", SimConfig(capacity=160, initial_nodes=128, init_mode=KB_INIT_CONVERGED, loss=0.02, churn=0.03,
                                fault_end_round=12, seed=31), 200),
    # Kaboodle::set_identity on stopped peers (src/lib.rs:323-336): one keeps the uniform length, one does not;
    # both restart at fresh addresses (36, 37) under the new identity, while the views that still hold 5 and 11
    # keep the identities those addresses announced; 38 is set before its first start
    _sc("identity_change", SimConfig(capacity=40, initial_nodes=36, init_mode=KB_INIT_CONVERGED, seed=19, loss=0.03,
                                     id_len=4), 24,
        events={2: [("stop", 5, None), ("stop", 11, None)], 3: [("ident", 5, b"wxyz"), ("ident", 11, b"zz"),
                                                                ("restart", 5, None)],
                6: [("ident", 38, b"new-peer"), ("start", 38, None), ("restart", 11, None)]}),
]

BY_NAME = {s["name"]: s for s in SCENARIOS}


def pymesh_of(sc):
    import pyref
    c = sc["cfg"]
    part = (c.partition_groups, c.partition_start, c.partition_end) if c.partition_groups else None
    pm = pyref.PyMesh(c.capacity, c.initial_nodes, converged=c.init_mode == KB_INIT_CONVERGED, seed=c.seed,
                      loss=c.loss, churn=c.churn, fault_end=c.fault_end_round, max_waves=c.max_waves,
                      failed_honoured=c.failed_mode != KB_FAILED_SOCKET_FAITHFUL, id_len=c.id_len, partition=part)
    return pm


def setup(sim, sc):
    """identities then starts (works for Sim and PyMesh alike)"""
    for i, ident in sc["identities"].items():
        sim.set_identity(i, ident)
    for i in sc["start"]:
        sim.start_node(i)


def apply_events(sim, sc, r):
    for kind, node, arg in sc["events"].get(r, []):
        if kind == "stop":
            sim.stop_node(node)
        elif kind == "start":
            sim.start_node(node)
        elif kind == "restart":
            sim.restart_node(node)
        elif kind == "ident":
            sim.set_identity(node, arg)
        else:
            sim.ping_addrs(node, arg)


def _crc(b: bytes) -> int:
    return zlib.crc32(b)


def digest_sim(sim: Sim) -> dict:
    """Round digest of an ABI implementation (oracle or GPU)."""
    C = sim.capacity
    rows = sim.rows()
    susp = [s for i in range(C) for s in [(i,) + tuple(x) for x in sim.suspects(i)]]
    cur = [s for i in range(C) for s in [(i,) + tuple(x) for x in sim.curious(i)]]
    st = sim.stats()
    return {"rows": _crc(rows.astype(np.uint8).tobytes()), "fps": _crc(np.asarray(sim.fingerprints(), np.uint32).tobytes()),
            "susp": _crc(repr(susp).encode()), "cur": _crc(repr(cur).encode()), "agree": st["agree"],
            "alive": st["alive"], "stats": {k: st[k] for k in STAT_KEYS}}


def digest_pymesh(pm) -> dict:
    import pyref
    C = pm.C
    rows = np.array([pm.row(i) for i in range(C)], dtype=np.uint8)
    fps = np.array([pyref.view_fingerprint(p.known) if p.running else 0 for p in pm.peers], np.uint32)
    susp = [s for i in range(C) for s in [(i,) + tuple(x) for x in pm.suspects(i)]]
    cur = [s for i in range(C) for s in [(i,) + tuple(x) for x in pm.curious_view(i)]]
    return {"rows": _crc(rows.tobytes()), "fps": _crc(fps.tobytes()), "susp": _crc(repr(susp).encode()),
            "cur": _crc(repr(cur).encode()), "agree": pm.agree,
            "alive": sum(p.running for p in pm.peers), "stats": {k: pm.stats[k] for k in STAT_KEYS}}


STAT_KEYS = ("sent_ping", "sent_ping_req", "sent_ack", "sent_known_peers", "sent_kpr", "bcast_join", "bcast_failed",
             "drop_dead", "drop_loss", "drop_window", "drop_oversize", "drop_partition", "drop_bcast",
             "removed_timeout", "removed_failed", "join_responses", "curious_overflow", "churn_leaves", "churn_joins")
