"""ctypes binding of the C ABI declared in include/kaboodle_sim.h.

`SimLib(path, prefix)` binds one shared library that implements the ABI.  The product binds the
in-tree HIP library (`kaboodle_amd/libkaboodle_sim.so`, prefix ``kb_``); the test suite uses the same
class to bind the CPU oracle (prefix ``kbo_``) so both are driven through identical calls.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

KB_ABI_VERSION = 3
KB_OK, KB_INVALID_OPERATION, KB_IO_ERROR, KB_NO_DEVICE, KB_STOPPING_FAILED, KB_INVALID_ARGUMENT, KB_CAPACITY = range(7)
KB_INIT_JOIN, KB_INIT_CONVERGED = 0, 1
KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL = 0, 1
KB_DBG_PHASEB_HBM, KB_DBG_RESP_HBM, KB_DBG_KP_HBM, KB_DBG_KP_BIG_SMALL, KB_DBG_PROC_UNSORTED = 1, 2, 4, 8, 16
KB_DBG_ALL = 31                  # every wide-row variant
KB_DBG_WAVE_GRAPH = 32           # the receive window as a replayed HIP graph
KB_DBG_RESP_WAVE_HBM = 64        # Join responses by wave, rows read in place (rows > 110K ids)
KB_DBG_NO_UNION = 128            # row shards: Join responses as id lists, not one union per (source shard, joiner)
KB_VARIANT_SAME_WINDOW_BCAST, KB_VARIANT_EXACT_LRU = 1, 2   # the first oracle-only; the second on the GPU too (bench default)
KB_STAT_NO_SF_FAILED_DROPS = 1
KB_VARIANT_SPARSE_ROWS = 4       # the configs[4] layout: oracle and the HIP library (unsharded or row shards)
KB_LATENCY_NONE = 0xFFFFFFFF
KT_ROWPASS, KT_ROUND, KT_FOLD, KT_RESP, KT_PROC = 0, 1, 2, 3, 4   # kb_sim_kernel_time / kb_sim_kernel_bytes kinds
KB_WAVE_SLOTS = 9
STATE_NAMES = {0: "Known", 1: "WaitingForPing", 2: "WaitingForIndirectPing"}


class KbConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("capacity", C.c_uint32), ("initial_nodes", C.c_uint32),
        ("init_mode", C.c_uint32), ("seed", C.c_uint64), ("loss_threshold", C.c_uint32),
        ("churn_threshold", C.c_uint32), ("fault_end_round", C.c_int32), ("max_waves", C.c_uint32),
        ("failed_mode", C.c_uint32), ("id_len", C.c_uint32), ("partition_groups", C.c_uint32),
        ("partition_start", C.c_int32), ("partition_end", C.c_int32), ("device", C.c_int32),
        ("debug_flags", C.c_uint32), ("track_latency", C.c_uint32), ("variant", C.c_uint32),
        ("sparse_row_cap", C.c_uint32), ("stat_flags", C.c_uint32), ("reserved", C.c_uint32 * 1),
    ]


class KbPeerState(C.Structure):
    _fields_ = [("peer", C.c_uint32), ("state", C.c_uint32), ("since", C.c_int32), ("latency_ms", C.c_uint32),
                ("identity_len", C.c_uint32), ("identity", C.c_uint8 * 32)]


PEER_STATE_DTYPE = [("peer", "<u4"), ("state", "<u4"), ("since", "<i4"), ("latency_ms", "<u4"), ("identity_len", "<u4"),
                    ("identity", "u1", (32,))]    # KbPeerState's layout (52 B, no padding)


class KbStats(C.Structure):
    _fields_ = [
        ("round", C.c_int32), ("alive", C.c_uint32), ("agree", C.c_uint32),
        ("first_converged_round", C.c_int32), ("last_converged_round", C.c_int32), ("next_free_id", C.c_uint32),
        ("sent_ping", C.c_uint64), ("sent_ping_req", C.c_uint64), ("sent_ack", C.c_uint64),
        ("sent_known_peers", C.c_uint64), ("sent_kpr", C.c_uint64),
        ("bcast_join", C.c_uint64), ("bcast_failed", C.c_uint64),
        ("drop_dead", C.c_uint64), ("drop_loss", C.c_uint64), ("drop_window", C.c_uint64),
        ("drop_oversize", C.c_uint64), ("drop_partition", C.c_uint64), ("drop_bcast", C.c_uint64),
        ("removed_timeout", C.c_uint64), ("removed_failed", C.c_uint64), ("join_responses", C.c_uint64),
        ("curious_overflow", C.c_uint64), ("churn_leaves", C.c_uint64), ("churn_joins", C.c_uint64),
        ("sent_kp_ids", C.c_uint64), ("alive_rounds", C.c_uint64), ("probe_responses", C.c_uint64),
        ("exported", C.c_uint64), ("reserved", C.c_uint64 * 4),
    ]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "reserved"}


class KbKernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 24), ("ms", C.c_double), ("launches", C.c_uint64), ("bytes", C.c_uint64),
                ("has_bytes", C.c_uint32), ("pad", C.c_uint32), ("wave_ms", C.c_double * KB_WAVE_SLOTS)]


class KbWireAddrC(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 4), ("port", C.c_uint16), ("pad", C.c_uint16)]


class KbProbeResponse(C.Structure):
    _fields_ = [("responder", C.c_uint32), ("probe", C.c_uint32), ("round", C.c_int32), ("prober", KbWireAddrC),
                ("identity_len", C.c_uint32), ("identity", C.c_uint8 * 32)]


class KbUnicast(C.Structure):
    _fields_ = [("round", C.c_int32), ("wave", C.c_uint32), ("sender", C.c_uint32), ("dest", C.c_uint32),
                ("seq", C.c_uint32), ("kind", C.c_uint32), ("a", C.c_uint32), ("fp", C.c_uint32), ("n", C.c_uint32),
                ("pay_off", C.c_uint32), ("pay_len", C.c_uint32), ("pad", C.c_uint32)]


class KbBroadcast(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("sender", C.c_uint32), ("peer", C.c_uint32), ("pad", C.c_uint32)]


def wire_addr(addr) -> KbWireAddrC:
    """("a.b.c.d", port) -> kb_wire_addr"""
    ip, port = addr
    a = KbWireAddrC()
    for k, part in enumerate(ip.split(".")):
        a.ip[k] = int(part)
    a.port = port
    return a


class KbError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with status {code}")
        self.code = code


@dataclass
class SimConfig:
    """Python-side mirror of kb_config (defaults as kb_config_default)."""
    capacity: int = 1024
    initial_nodes: int = 1024
    init_mode: int = KB_INIT_JOIN
    seed: int = 1
    loss: float = 0.0            # per-delivery loss probability
    churn: float = 0.0           # per-node per-round leave probability
    fault_end_round: int = -1
    max_waves: int = 8
    failed_mode: int = KB_FAILED_SIM_SENDER
    id_len: int = 0
    partition_groups: int = 0
    partition_start: int = 0
    partition_end: int = 0
    device: int = -1
    debug_flags: int = 0         # KB_DBG_*: force the wide-row kernel variants (test surface)
    track_latency: int = 0       # 1: keep the ping-latency EWMA reported by peer_states
    variant: int = 0             # KB_VARIANT_*: SAME_WINDOW_BCAST (oracle-only deviation measurement), EXACT_LRU
                                 # (the reference's exact A3 order, oracle and GPU), SPARSE_ROWS (the configs[4]
                                 # layout, oracle and GPU, unsharded or as row shards)
    sparse_row_cap: int = 0      # KB_VARIANT_SPARSE_ROWS on the GPU: entries per row (0: min(capacity, 4096))
    stat_flags: int = 0          # KB_STAT_*: KB_STAT_NO_SF_FAILED_DROPS skips socket_faithful Failed drop counts

    def to_c(self) -> KbConfig:
        c = KbConfig()
        c.abi_version = KB_ABI_VERSION
        c.capacity, c.initial_nodes, c.init_mode = self.capacity, self.initial_nodes, self.init_mode
        c.seed = self.seed
        c.loss_threshold = min(int(round(self.loss * 2**32)), 2**32 - 1)
        c.churn_threshold = min(int(round(self.churn * 2**32)), 2**32 - 1)
        c.fault_end_round, c.max_waves, c.failed_mode = self.fault_end_round, self.max_waves, self.failed_mode
        c.id_len = self.id_len
        c.partition_groups, c.partition_start, c.partition_end = (
            self.partition_groups, self.partition_start, self.partition_end)
        c.device = self.device
        c.debug_flags, c.track_latency, c.variant = self.debug_flags, self.track_latency, self.variant
        c.sparse_row_cap, c.stat_flags = self.sparse_row_cap, self.stat_flags
        return c


_SIGS = {
    "sim_create": (C.c_int, [C.POINTER(KbConfig), C.POINTER(C.c_void_p)]),
    "sim_destroy": (C.c_int, [C.c_void_p]),
    "sim_step": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sim_start_node": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sim_stop_node": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sim_is_running": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_int)]),
    "sim_ping_addrs": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_size_t]),
    "sim_set_identity": (C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]),
    "sim_identity": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_size_t)]),
    "sim_fingerprint": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "sim_fingerprints": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t]),
    "sim_true_fingerprint": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "sim_peers": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t)]),
    "sim_peer_states": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(KbPeerState), C.c_size_t,
                                  C.POINTER(C.c_size_t)]),
    "sim_stats": (C.c_int, [C.c_void_p, C.POINTER(KbStats)]),
    "sim_dump_row": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint8), C.c_size_t]),
    "sim_dump_scalars": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.c_size_t]),
    "sim_dump_suspects": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_int32), C.c_size_t,
                                    C.POINTER(C.c_size_t)]),
    "sim_dump_curious": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_int32), C.c_size_t,
                                   C.POINTER(C.c_size_t)]),
    "sim_watch": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sim_events": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t),
                             C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_uint32),
                             C.POINTER(C.c_int)]),
    "sim_probe": (C.c_int, [C.c_void_p, C.POINTER(KbWireAddrC)]),
    "sim_probe_responses": (C.c_int, [C.c_void_p, C.POINTER(KbProbeResponse), C.c_size_t, C.POINTER(C.c_size_t)]),
    "sim_broadcasts": (C.c_int, [C.c_void_p, C.POINTER(KbBroadcast), C.c_size_t, C.POINTER(C.c_size_t)]),
    "sim_set_external": (C.c_int, [C.c_void_p, C.c_uint32]),
    "sim_inject": (C.c_int, [C.c_void_p, C.POINTER(KbUnicast), C.POINTER(C.c_uint32)]),
    "sim_exported": (C.c_int, [C.c_void_p, C.POINTER(KbUnicast), C.c_size_t, C.POINTER(C.c_size_t),
                               C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t)]),
    "format_addr": (C.c_int, [C.c_uint32, C.c_char_p, C.c_size_t]),
    "last_error": (C.c_char_p, []),
}
_OPTIONAL = {
    "sim_restart_node": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    # sharding (HIP library only; the oracle is the unsharded mesh every shard layout must reproduce)
    "rccl_unique_id": (C.c_int, [C.POINTER(C.c_uint8), C.c_size_t]),
    "ipc_unique_id": (C.c_int, [C.POINTER(C.c_uint8), C.c_size_t]),
    "sim_create_rank": (C.c_int, [C.POINTER(KbConfig), C.c_int32, C.c_int32, C.POINTER(C.c_uint8),
                                  C.POINTER(C.c_void_p)]),
    "sim_create_local": (C.c_int, [C.POINTER(KbConfig), C.c_int32, C.POINTER(C.c_void_p)]),
    "sim_shard_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint32)]),
    "sim_kernel_time": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "sim_reset_kernel_time": (C.c_int, [C.c_void_p]),
    "sim_kernel_bytes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)]),
    "sim_debug_paths": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "sim_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "sim_kernel_breakdown": (C.c_int, [C.c_void_p, C.POINTER(KbKernelTime), C.c_size_t, C.POINTER(C.c_size_t)]),
    "sim_host_syncs": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "sim_sparse_footprint": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t]),
}


class SimLib:
    """One loaded implementation of the ABI (functions named `<prefix><name>`)."""

    def __init__(self, path: str, prefix: str = "kb_"):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.path, self.prefix = path, prefix
        self.lib = C.CDLL(path)
        self.fn = {}
        for name, (res, args) in _SIGS.items():
            f = getattr(self.lib, prefix + name)
            f.restype, f.argtypes = res, args
            self.fn[name] = f
        for name, (res, args) in _OPTIONAL.items():
            f = getattr(self.lib, prefix + name, None)
            if f is not None:
                f.restype, f.argtypes = res, args
                self.fn[name] = f

    def call(self, name: str, *args) -> None:
        rc = self.fn[name](*args)
        if rc != KB_OK:
            err = self.fn["last_error"]()
            raise KbError(rc, f"{self.prefix}{name} ({err.decode(errors='replace') if err else ''})")


KB_UNIQUE_ID_BYTES = 128


def rccl_unique_id(lib: SimLib) -> bytes:
    """A fresh RCCL unique id (rank 0 makes it; the host broadcasts it to the other ranks)."""
    buf = (C.c_uint8 * KB_UNIQUE_ID_BYTES)()
    lib.call("rccl_unique_id", buf, KB_UNIQUE_ID_BYTES)
    return bytes(buf)


def ipc_unique_id(lib: SimLib) -> bytes:
    """A unique id for ranks in separate processes sharing one device (the IPC test transport)."""
    buf = (C.c_uint8 * KB_UNIQUE_ID_BYTES)()
    lib.call("ipc_unique_id", buf, KB_UNIQUE_ID_BYTES)
    return bytes(buf)


class Sim:
    """A simulated mesh (one handle) bound to a SimLib.

    shards=k (k >= 1): the mesh split into k row shards inside this process (kb_sim_create_local);
    rank/world/uid: this process's shard of a mesh spread over `world` processes (kb_sim_create_rank).
    A library without the sharding entry points (the oracle) always builds the unsharded mesh, which
    every shard layout must reproduce bit for bit.
    """

    def __init__(self, lib: SimLib, cfg: SimConfig, shards: int = 0, rank: int | None = None,
                 world: int | None = None, uid: bytes | None = None):
        self.lib, self.cfg = lib, cfg
        self._c = cfg.to_c()
        h = C.c_void_p()
        if world is not None and "sim_create_rank" in lib.fn:
            ub = (C.c_uint8 * KB_UNIQUE_ID_BYTES).from_buffer_copy(uid)
            lib.call("sim_create_rank", C.byref(self._c), rank, world, ub, C.byref(h))
        elif shards and "sim_create_local" in lib.fn:
            lib.call("sim_create_local", C.byref(self._c), shards, C.byref(h))
        else:
            lib.call("sim_create", C.byref(self._c), C.byref(h))
        self.h = h
        self.capacity = cfg.capacity

    def shard_info(self):
        """(rank, world, lo, hi): the rows this handle holds."""
        if "sim_shard_info" not in self.lib.fn:
            return 0, 1, 0, self.capacity
        r, w, lo, hi = C.c_int32(), C.c_int32(), C.c_uint32(), C.c_uint32()
        self.lib.call("sim_shard_info", self.h, C.byref(r), C.byref(w), C.byref(lo), C.byref(hi))
        return r.value, w.value, lo.value, hi.value

    def close(self) -> None:
        if self.h:
            self.lib.call("sim_destroy", self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- lifecycle --
    def step(self, rounds: int = 1) -> None:
        self.lib.call("sim_step", self.h, rounds)

    def start_node(self, node: int) -> None:
        self.lib.call("sim_start_node", self.h, node)

    def stop_node(self, node: int) -> None:
        self.lib.call("sim_stop_node", self.h, node)

    def restart_node(self, node: int) -> int:
        """Kaboodle::start for the instance at `node`: returns its address from then on (a fresh id when it
        had run and is stopped; kb_sim_restart_node)."""
        v = C.c_uint32()
        self.lib.call("sim_restart_node", self.h, node, C.byref(v))
        return v.value

    def is_running(self, node: int) -> bool:
        v = C.c_int()
        self.lib.call("sim_is_running", self.h, node, C.byref(v))
        return bool(v.value)

    def ping_addrs(self, node: int, peers) -> None:
        arr = (C.c_uint32 * len(peers))(*peers)
        self.lib.call("sim_ping_addrs", self.h, node, arr, len(peers))

    def set_identity(self, node: int, identity: bytes) -> None:
        self.lib.call("sim_set_identity", self.h, node, identity, len(identity))

    # -- inspection --
    def identity(self, node: int) -> bytes:
        """The identity bytes of id `node` (what every view reports for it)."""
        n = C.c_size_t()
        buf = (C.c_uint8 * 32)()
        self.lib.call("sim_identity", self.h, node, buf, 32, C.byref(n))
        return bytes(buf[: n.value])

    def fingerprint(self, node: int) -> int:
        v = C.c_uint32()
        self.lib.call("sim_fingerprint", self.h, node, C.byref(v))
        return v.value

    def fingerprints(self):
        import numpy as np
        out = np.zeros(self.capacity, dtype=np.uint32)
        self.lib.call("sim_fingerprints", self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), self.capacity)
        return out

    def true_fingerprint(self) -> int:
        v = C.c_uint32()
        self.lib.call("sim_true_fingerprint", self.h, C.byref(v))
        return v.value

    def peers(self, node: int):
        n = C.c_size_t()
        self.lib.call("sim_peers", self.h, node, None, 0, C.byref(n))
        arr = (C.c_uint32 * max(n.value, 1))()
        self.lib.call("sim_peers", self.h, node, arr, n.value, C.byref(n))
        return list(arr[: n.value])

    # -- event streams (src/events.rs:18-125) --
    def watch(self, node: int) -> None:
        """Attach an observer to `node` (empty, as Kaboodle::new does, src/lib.rs:112)."""
        self.lib.call("sim_watch", self.h, node)

    def events(self, node: int):
        """Drain one batch: (discovered, departed, fingerprint, fingerprint_changed)."""
        nd, npp, fp, ch = C.c_size_t(), C.c_size_t(), C.c_uint32(), C.c_int()
        self.lib.call("sim_events", self.h, node, None, 0, C.byref(nd), None, 0, C.byref(npp), C.byref(fp),
                      C.byref(ch))
        d = (C.c_uint32 * max(nd.value, 1))()
        p = (C.c_uint32 * max(npp.value, 1))()
        self.lib.call("sim_events", self.h, node, d, nd.value, C.byref(nd), p, npp.value, C.byref(npp),
                      C.byref(fp), C.byref(ch))
        return list(d[: nd.value]), list(p[: npp.value]), fp.value, bool(ch.value)

    def peer_states(self, node: int):
        n = C.c_size_t()
        self.lib.call("sim_peer_states", self.h, node, None, 0, C.byref(n))
        arr = (KbPeerState * max(n.value, 1))()
        self.lib.call("sim_peer_states", self.h, node, arr, n.value, C.byref(n))
        return [(a.peer, a.state, a.since, a.latency_ms, bytes(a.identity[: a.identity_len])) for a in arr[: n.value]]

    def peer_states_array(self, node: int):
        """peer_states as one numpy record array (the fields of kb_peer_state): peer_states() without a Python
        tuple per entry (64K-entry rows).  Identity bytes past identity_len are whatever the library wrote there
        (zero-filled buffer), so equal arrays mean equal peer_states(), not the converse."""
        import numpy as np
        n = C.c_size_t()
        self.lib.call("sim_peer_states", self.h, node, None, 0, C.byref(n))
        a = np.zeros(max(n.value, 1), dtype=PEER_STATE_DTYPE)
        self.lib.call("sim_peer_states", self.h, node, C.cast(a.ctypes.data, C.POINTER(KbPeerState)), n.value,
                      C.byref(n))
        return a[: n.value]

    # -- discovery (src/discovery.rs:30-89, src/kaboodle.rs:305-331) --
    def probe(self, prober) -> None:
        """Queue SwimBroadcast::Probe(prober) for the next round; prober = ("a.b.c.d", port) outside the mesh."""
        self.lib.call("sim_probe", self.h, C.byref(wire_addr(prober)))

    def probe_responses(self):
        """Drain the ProbeResponses: [(round, responder id, probe index, prober addr, identity)] in canonical order."""
        n = C.c_size_t()
        self.lib.call("sim_probe_responses", self.h, None, 0, C.byref(n))
        arr = (KbProbeResponse * max(n.value, 1))()
        self.lib.call("sim_probe_responses", self.h, arr, n.value, C.byref(n))
        return [(a.round, a.responder, a.probe, (".".join(str(a.prober.ip[k]) for k in range(4)), a.prober.port),
                 bytes(a.identity[: a.identity_len])) for a in arr[: n.value]]

    def broadcasts(self):
        """The last round's Join / Failed broadcasts: [("Join" | "Failed", sender id, peer id)], sender order."""
        n = C.c_size_t()
        self.lib.call("sim_broadcasts", self.h, None, 0, C.byref(n))
        arr = (KbBroadcast * max(n.value, 1))()
        self.lib.call("sim_broadcasts", self.h, arr, n.value, C.byref(n))
        return [("Join" if a.kind == 16 else "Failed", a.sender, a.peer) for a in arr[: n.value]]

    # -- external peers: real instances attached through a bridge --
    def set_external(self, node: int) -> None:
        """Mark a never-bound address as an external peer (kb_sim_set_external)."""
        self.lib.call("sim_set_external", self.h, node)

    def inject(self, sender: int, dest: int, kind: int, a: int = 0, fp: int = 0, n: int = 0, ids=()) -> None:
        """Queue a record from external peer `sender` to `dest` for the next round's wave 0 (kb_sim_inject);
        kind = wire kind 0..4 (Ping, PingRequest, Ack, KnownPeers, KnownPeersRequest), or 16: the external peer's
        Join broadcast, delivered in the next round's broadcast phase (dest unused)."""
        m = KbUnicast(sender=sender, dest=dest, kind=kind, a=a, fp=fp, n=n, pay_len=len(ids))
        arr = (C.c_uint32 * max(1, len(ids)))(*ids)
        self.lib.call("sim_inject", self.h, C.byref(m), arr)

    def exported(self):
        """Drain the records routed to external peers: [(round, wave, sender, dest, seq, kind, a, fp, n, ids)]."""
        n, ni = C.c_size_t(), C.c_size_t()
        self.lib.call("sim_exported", self.h, None, 0, C.byref(n), None, 0, C.byref(ni))
        arr = (KbUnicast * max(n.value, 1))()
        ids = (C.c_uint32 * max(ni.value, 1))()
        self.lib.call("sim_exported", self.h, arr, n.value, C.byref(n), ids, ni.value, C.byref(ni))
        return [(u.round, u.wave, u.sender, u.dest, u.seq, u.kind, u.a, u.fp, u.n, list(ids[u.pay_off:u.pay_off + u.pay_len]))
                for u in arr[: n.value]]

    def stats(self) -> dict:
        st = KbStats()
        self.lib.call("sim_stats", self.h, C.byref(st))
        return st.as_dict()

    def row(self, node: int):
        import numpy as np
        out = np.zeros(self.capacity, dtype=np.uint8)
        self.lib.call("sim_dump_row", self.h, node, out.ctypes.data_as(C.POINTER(C.c_uint8)), self.capacity)
        return out

    def rows(self):
        import numpy as np
        return np.stack([self.row(i) for i in range(self.capacity)])

    def scalars(self):
        import numpy as np
        out = np.zeros((self.capacity, 4), dtype=np.int32)
        self.lib.call("sim_dump_scalars", self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), out.size)
        return out

    def suspects(self, node: int):
        n = C.c_size_t()
        buf = (C.c_int32 * (3 * 8))()
        self.lib.call("sim_dump_suspects", self.h, node, buf, len(buf), C.byref(n))
        return [tuple(buf[3 * k: 3 * k + 3]) for k in range(n.value)]

    def curious(self, node: int):
        n = C.c_size_t()
        buf = (C.c_int32 * (6 * 8))()
        self.lib.call("sim_dump_curious", self.h, node, buf, len(buf), C.byref(n))
        return [tuple(buf[6 * k: 6 * k + 6]) for k in range(n.value)]

    def format_addr(self, node: int) -> str:
        buf = C.create_string_buffer(32)
        self.lib.call("format_addr", node, buf, 32)
        return buf.value.decode()

    # -- bench surface (HIP library only) --
    def kernel_time(self, kind: int = 0):
        ms, n = C.c_double(), C.c_uint64()
        self.lib.call("sim_kernel_time", self.h, kind, C.byref(ms), C.byref(n))
        return ms.value, n.value

    def reset_kernel_time(self) -> None:
        self.lib.call("sim_reset_kernel_time", self.h)

    def debug_paths(self) -> int:
        """OR of the kernel-variant bits (PATH_* of kb_common.h) that did work; 0 for the oracle."""
        if "sim_debug_paths" not in self.lib.fn:
            return 0
        v = C.c_uint32()
        self.lib.call("sim_debug_paths", self.h, C.byref(v))
        return v.value

    def kernel_bytes(self, kind: int = 0) -> int:
        """Algorithmic bytes the kernel `kind` (KT_ROWPASS / KT_FOLD / KT_RESP / KT_PROC) moved since
        reset_kernel_time."""
        v = C.c_uint64()
        self.lib.call("sim_kernel_bytes", self.h, kind, C.byref(v))
        return v.value

    def set_profiling(self, level: int) -> None:
        """Per-launch HIP events (kernel_breakdown): 0 none, 1 the byte-counted kernels (default), 2 every launch."""
        self.lib.call("sim_set_profiling", self.h, int(level))

    def kernel_breakdown(self) -> dict:
        """{kernel: {"ms", "launches", "bytes" (None if not counted), "wave_ms": [...]}} since reset_kernel_time."""
        n = C.c_size_t()
        self.lib.call("sim_kernel_breakdown", self.h, None, 0, C.byref(n))
        arr = (KbKernelTime * max(n.value, 1))()
        self.lib.call("sim_kernel_breakdown", self.h, arr, n.value, C.byref(n))
        return {a.name.decode(): {"ms": a.ms, "launches": a.launches, "bytes": a.bytes if a.has_bytes else None,
                                  "wave_ms": list(a.wave_ms)} for a in arr[: n.value]}

    def sparse_footprint(self) -> dict:
        """KB_VARIANT_SPARSE_ROWS: rows that adopted the base, exceptions, explicit stamps, entries of the largest
        row, bytes of the entries, rows (kb_sim_sparse_footprint)."""
        out = (C.c_uint64 * 6)()
        self.lib.call("sim_sparse_footprint", self.h, out, 6)
        keys = ("rows_based", "exceptions", "stamps", "max_row_entries", "bytes", "rows")
        return dict(zip(keys, (int(v) for v in out)))

    def host_syncs(self) -> int:
        """Host waits on the device since creation (stream synchronisations, pinned hand-offs)."""
        v = C.c_uint64()
        self.lib.call("sim_host_syncs", self.h, C.byref(v))
        return v.value
