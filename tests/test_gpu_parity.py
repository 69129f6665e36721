"""Parity of the HIP library with the CPU oracle, through the C ABI, on an MI355X.

Bar: bit-exact (all state is integer/byte): stamp rows, per-node scalars, suspect and curious tables,
fingerprints and every counter, after every round."""
import json
import os

import numpy as np
import pytest

import parity
import scenarios
from kaboodle_amd._ffi import (KB_DBG_ALL, KB_DBG_RESP_WAVE_HBM, KB_DBG_WAVE_GRAPH, KB_INIT_CONVERGED, KB_INVALID_OPERATION,
                               KB_VARIANT_EXACT_LRU, KbError, Sim, SimConfig)

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gpu():
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    return parity.gpu_lib()


@pytest.mark.parametrize("name,case,rounds", parity.standard_cases(), ids=[c[0] for c in parity.standard_cases()])
def test_parity_every_round(gpu, name, case, rounds):
    """Complete state every round, plus peer_states() of every node with the latency EWMA on (the
    rebase_window case crosses two 64-round stamp-window rebases)."""
    ok, msg, _ = parity.run_case(parity.with_cfg(case, track_latency=1), rounds, peer_states=True)
    assert ok, f"{name}: {msg}"


@pytest.mark.parametrize("name,case,rounds", parity.standard_cases(), ids=[c[0] for c in parity.standard_cases()])
def test_parity_wide_row_paths(gpu, name, case, rounds):
    """The standard matrix on the kernel variants a >= 1M-id mesh takes (configs[3]/[4]: broadcast phase
    and KnownPeers groups on the HBM bitset, Join responses from HBM scratch, BIG KnownPeers groups,
    k_proc's unsorted selection path), forced by kb_config.debug_flags at these sizes."""
    ok, msg, _ = parity.run_case(parity.with_cfg(case, debug_flags=KB_DBG_ALL), rounds)
    assert ok, f"{name} (debug_flags={KB_DBG_ALL}): {msg}"


@pytest.mark.parametrize("name,case,rounds", parity.standard_cases(), ids=[c[0] for c in parity.standard_cases()])
def test_parity_exact_lru(gpu, name, case, rounds):
    """A3 ordered by the exact instant of the last contact (KB_VARIANT_EXACT_LRU: src/kaboodle.rs:662-675 sorts
    by Instant) instead of the 1-byte stamp window: the instants of entries that saturate at a rebase are kept in
    a table, fresher ones are decoded from their bytes (rebase_window and old_stamps cross two and three
    rebases).  Complete state every round, latency on."""
    ok, msg, _ = parity.run_case(parity.with_cfg(case, variant=KB_VARIANT_EXACT_LRU, track_latency=1), rounds)
    assert ok, f"{name} (exact LRU): {msg}"


@pytest.mark.parametrize("name", ["stop_start", "rebase_window", "fresh_ids"])
def test_parity_exact_lru_sharded(gpu, name):
    """The exact instants move with a restart's map and stay row-local when sharded (x3)."""
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}[name]
    ok, msg, _ = parity.run_case(parity.with_cfg(case, variant=KB_VARIANT_EXACT_LRU), rounds, shards=3)
    assert ok, f"{name} (exact LRU, x3): {msg}"


def test_parity_exact_lru_block_bounds(gpu):
    """Rows of four 1024-id blocks over three rebases (k_a3_exact's bound-ordered block scan: the tied converged
    start, bounds tightened by scans, lowered by k_rebase, reset by a restart's move).  Complete state every 4th
    round and at the end."""
    case = {"cfg": SimConfig(capacity=4000, initial_nodes=3400, init_mode=KB_INIT_CONVERGED, churn=0.0005, loss=0.01,
                             seed=41, variant=KB_VARIANT_EXACT_LRU),
            "events": {70: [("stop", 17, None)], 75: [("restart", 17, None)], 150: [("stop", 2900, None)],
                       160: [("restart", 2900, None)]}}
    ok, msg, _ = parity.run_case(case, 200, check_every=4, full_rows=True)
    assert ok, f"exact LRU blocks: {msg}"


EXT_CASES = ["converged_loss_256", "churn_loss_512", "partition_heal", "stop_start", "join_64"]


@pytest.mark.parametrize("mode", ["dense", "x3", "sparse"])
@pytest.mark.parametrize("name", EXT_CASES)
def test_gpu_external_peers(gpu, name, mode):
    """External peers: two addresses beyond the case's ids stand for real instances; the records
    simulated peers address to them are exported (identically, every round) and a scripted real instance's
    replies are injected into the next round's wave 0 (parity.external_replies): complete state every round,
    unsharded, as 3 row shards (the sender's shard exports, the external's shard injects) and on sparse rows."""
    from dataclasses import replace
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}[name]
    c = case["cfg"]
    cfg = replace(c, capacity=c.capacity + 4, variant=4 if mode == "sparse" else 0)
    ok, msg, nx = parity.run_external_case({**case, "cfg": cfg}, rounds, [c.capacity + 1, c.capacity + 3],
                                           [parity.oracle_lib(), gpu], shards=3 if mode == "x3" else 0)
    assert ok and nx > 0, f"{name} ({mode}): {msg}"


TRUNC_CASES = {
    # views of > 567 ids: every Join response is a sampled (truncated) one, served by wave
    "trunc_1200": ({"cfg": SimConfig(capacity=1300, initial_nodes=1200, init_mode=KB_INIT_CONVERGED, churn=0.01, seed=23)}, 6),
    "trunc_loss_1800": ({"cfg": SimConfig(capacity=2000, initial_nodes=1800, init_mode=KB_INIT_CONVERGED, churn=0.005,
                                          loss=0.02, seed=5, id_len=3)}, 8),
}


@pytest.mark.parametrize("name", sorted(TRUNC_CASES))
def test_parity_resp_wave_rows_in_place(gpu, name):
    """Join responses by wave with the rows read in place (the path of rows too wide for a wave's LDS
    copy, configs[3]'s 1M-id rows), forced by KB_DBG_RESP_WAVE_HBM at these sizes; and the same cases on
    the default (LDS copy) wave path."""
    case, rounds = TRUNC_CASES[name]
    for flags, want in ((KB_DBG_RESP_WAVE_HBM, 256), (0, 64)):
        g = Sim(gpu, parity.with_cfg(case, debug_flags=flags)["cfg"])
        ok, msg, st = parity.run_case(parity.with_cfg(case, debug_flags=flags), rounds, gpu=g)
        assert ok, f"{name} (debug_flags={flags}): {msg}"
        assert st["join_responses"] > 0 and g.debug_paths() & want and not g.debug_paths() & (320 ^ want)
        g.close()


@pytest.mark.parametrize("name", ["partition_heal", "identity_change", "hot_inbox"])
def test_parity_wave_graph(gpu, name):
    """The receive window captured once as a HIP graph and replayed every round (KB_DBG_WAVE_GRAPH, the
    env KB_WAVE_GRAPH=1 path): same results, including across set_identity (which must drop the graph)."""
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}[name]
    ok, msg, _ = parity.run_case(parity.with_cfg(case, debug_flags=KB_DBG_WAVE_GRAPH, track_latency=1), rounds,
                                 peer_states=True)
    assert ok, f"{name} (wave graph): {msg}"


def test_identity_change_on_stopped_peer(gpu):
    """Kaboodle::set_identity (src/lib.rs:323-336) and start after stop (:136-156): refused while running
    (counting queued start/stop calls), allowed once stopped; the restarted instance binds a fresh address
    (src/kaboodle.rs:138-152) that inherits its map and announces the new bytes, while the views holding
    the old address keep the identity it announced.  Every fingerprint is generate_fingerprint over one
    identity per address (kb_fingerprint_of_set), on both implementations."""
    import ctypes as C
    cfg = SimConfig(capacity=512, initial_nodes=500, init_mode=KB_INIT_CONVERGED, id_len=6, seed=12)
    lib = C.CDLL(parity.GPU_SO)
    f = lib.kb_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    with Sim(parity.oracle_lib(), cfg) as o, Sim(gpu, cfg) as g:
        for s in (o, g):
            s.step(2)
        old7 = g.identity(7)
        news = set()
        for s in (o, g):
            with pytest.raises(KbError) as e:
                s.set_identity(7, b"abcdef")
            assert e.value.code == KB_INVALID_OPERATION
            s.stop_node(7)
            s.set_identity(7, b"abcdef")           # stop queued: no longer running as the API sees it
            with pytest.raises(KbError):
                s.start_node(7)                    # it ran: a restart binds a fresh address
            news.add(s.restart_node(7))
            with pytest.raises(KbError):
                s.set_identity(7, b"ghijkl")       # the instance moved on: address 7 stays stopped, but
        new = news.pop()                           # ... its restart is queued under the new address
        assert new == 500 and not news
        o.step(1)
        g.step(1)
        assert g.identity(7) == o.identity(7) == old7 and g.identity(new) == o.identity(new) == b"abcdef"
        assert g.is_running(new) and not g.is_running(7)
        fo, fg = o.fingerprints(), g.fingerprints()
        assert np.array_equal(fo, fg)
        assert g.peer_states(new) == o.peer_states(new)
        idents = np.zeros((cfg.capacity, 32), dtype=np.uint8)
        lens = np.zeros(cfg.capacity, dtype=np.uint8)
        for j in range(cfg.capacity):
            b = g.identity(j)
            idents[j, :len(b)] = np.frombuffer(b, dtype=np.uint8)
            lens[j] = len(b)
        for i in list(range(0, 500, 37)) + [new]:
            p = g.peers(i)
            want = f((C.c_uint32 * len(p))(*p), len(p), idents.ctypes.data, 32, lens.ctypes.data)
            assert want == fg[i], f"node {i}"
            ps = {e[0]: e[4] for e in g.peer_states(i)}
            assert ps.get(7, old7) == old7 and ps.get(new, b"abcdef") == b"abcdef"
        for _ in range(3):
            o.step(1)
            g.step(1)
            assert np.array_equal(o.fingerprints(), g.fingerprints())
            assert np.array_equal(o.row(new), g.row(new))


def test_wide_row_paths_are_hit(gpu):
    """The forced variants really run: every wide-row kernel path reports work (kb_sim_debug_paths)."""
    from kaboodle_amd._ffi import KB_DBG_ALL
    by = {n: (c, r) for n, c, r in parity.standard_cases()}
    mask = 0
    for name in ("config2_join_1k", "churn_loss_512", "hot_inbox"):
        case, rounds = by[name]
        with Sim(gpu, parity.with_cfg(case, debug_flags=KB_DBG_ALL)["cfg"]) as g:
            parity.setup(g, case)
            for r in range(rounds):
                parity.apply_events((g,), case, r)
                g.step(1)
            mask |= g.debug_paths()
    want = {"phaseB on HBM": 1, "responses from scratch, sampled": 2, "responses from scratch, complete": 4,
            "KnownPeers BIG on HBM": 8, "k_proc unsorted": 16, "Failed prep from HBM": 32}
    missing = [k for k, b in want.items() if not mask & b]
    assert not missing, f"paths not exercised: {missing} (mask {mask:#x})"
    # and without the flags the same cases take the LDS variants
    with Sim(gpu, by["config2_join_1k"][0]["cfg"]) as g:
        g.step(by["config2_join_1k"][1])
        assert g.debug_paths() & (128 | 64) and not g.debug_paths() & (1 | 8)


@pytest.mark.parametrize("name", ["config2_join_1k", "partition_heal"])
def test_parity_wide_row_paths_sharded(gpu, name):
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}[name]
    ok, msg, _ = parity.run_case(parity.with_cfg(case, debug_flags=KB_DBG_ALL, track_latency=1), rounds, shards=3,
                                 peer_states=True)
    assert ok, f"{name} x3 (debug_flags={KB_DBG_ALL}): {msg}"


def test_latency_ewma_measured(gpu):
    """PeerInfo.latency (src/kaboodle.rs:789-817) is really measured on the GPU: after a lossy run with
    churn, many entries carry a latency, of several values (direct Ack 2 ms, indirect 4 ms, EWMA mixes),
    and every node's peer_states equals the oracle's."""
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}["churn_loss_512"]
    cfg = parity.with_cfg(case, track_latency=1)["cfg"]
    with Sim(parity.oracle_lib(), cfg) as o, Sim(gpu, cfg) as g:
        o.step(rounds)
        g.step(rounds)
        vals = []
        for i in range(cfg.capacity):
            a = g.peer_states(i)
            assert a == o.peer_states(i), f"node {i}"
            vals += [e[3] for e in a if e[3] != 0xFFFFFFFF]
    assert len(vals) > cfg.capacity, len(vals)
    assert len(set(vals)) >= 3, sorted(set(vals))


def _shard_cases():
    """Every standard case as a sharded mesh (3 row shards, or as many as its capacity allows), plus
    the 1K join case at the full 8 shards of a node."""
    out = []
    for name, case, rounds in parity.standard_cases():
        C = case["cfg"].capacity
        k = 3 if C >= 9 else 2
        out.append((f"{name}-x{k}", case, rounds, k))
        if name == "config2_join_1k":
            out.append((f"{name}-x8", case, rounds, 8))
        if name == "churn_loss_512":
            out.append((f"{name}-x5", case, rounds, 5))
    return out


@pytest.mark.parametrize("name,case,rounds,shards", _shard_cases(), ids=[c[0] for c in _shard_cases()])
def test_sharded_parity_every_round(gpu, name, case, rounds, shards):
    """Row shards exchanging every wave (all-to-all-v of records, all-gather of broadcasts) reproduce
    the unsharded oracle bit for bit, every round."""
    ok, msg, _ = parity.run_case(case, rounds, shards=shards)
    assert ok, f"{name}: {msg}"


@pytest.mark.parametrize("name", ["churn_loss_512", "config2_join_1k", "partition_heal"])
def test_join_response_unions(gpu, name):
    """The Join-response union exchange: row shards whose wave-0 KnownPeers lists to the round's
    joiners cross as one bitmap per (source shard, joiner) equal the oracle every round (the lists' arms commute,
    src/kaboodle.rs:448-472), and so does the same mesh with the lists shipped whole (KB_DBG_NO_UNION); the unions
    cross fewer bytes whenever Join responses cross shards."""
    import ctypes as C
    from kaboodle_amd._ffi import KB_DBG_NO_UNION
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}[name]
    xb = {}
    for flags in (0, KB_DBG_NO_UNION):
        g = Sim(gpu, parity.with_cfg(case, debug_flags=flags)["cfg"], shards=4)
        ok, msg, st = parity.run_case(parity.with_cfg(case, debug_flags=flags), rounds, gpu=g)
        assert ok, f"{name} (debug_flags={flags}): {msg}"
        buf = (C.c_uint64 * 5)()
        assert gpu.lib.kb_sim_debug_counters(g.h, buf, 5) == 0
        xb[flags] = (buf[3], buf[4])
        g.close()
    assert xb[0][1] > 0 and xb[KB_DBG_NO_UNION][1] > 0, xb
    if st["join_responses"]:
        assert xb[0][0] < xb[KB_DBG_NO_UNION][0], xb


def test_host_waits_per_round(gpu):
    """Host waits on the device per round (kb_sim_host_syncs): unsharded at most two pinned hand-offs (the
    wave-0 outbox size when Join responses exist, the round's results); a row-sharded round one hand-off
    for the broadcast lists and every rank's error flag (one all-gather) plus one per delivery wave for
    the all-to-all-v counts; plus one stream synchronisation per kb_sim_step call."""
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}["churn_loss_512"]
    cfg = case["cfg"]
    with Sim(gpu, cfg) as g:
        g.step(1)
        n0 = g.host_syncs()
        g.step(rounds)
        assert g.host_syncs() - n0 <= 2 * rounds + 1
    with Sim(gpu, cfg, shards=3) as g:
        g.step(1)
        n0 = g.host_syncs()
        for _ in range(rounds):
            g.step(1)
        per_round = (g.host_syncs() - n0) / rounds
        assert per_round <= 1 + cfg.max_waves + 1 + 1, per_round


def test_rccl_rank_path_world1(gpu):
    """The RCCL transport itself (kb_sim_create_rank: ncclAllToAllv / AllGather / AllReduce on the
    simulator stream), as a 1-rank communicator on this GPU, against the oracle."""
    from kaboodle_amd._ffi import rccl_unique_id
    name, case, rounds = [c for c in parity.standard_cases() if c[0] == "churn_loss_512"][0]
    g = Sim(gpu, case["cfg"], rank=0, world=1, uid=rccl_unique_id(gpu))
    assert g.shard_info() == (0, 1, 0, case["cfg"].capacity)
    ok, msg, _ = parity.run_case(case, rounds, gpu=g)
    assert ok, f"{name} over RCCL: {msg}"


def test_sharded_full_size_64k(gpu):
    """BASELINE configs[2] at full size: 4 row shards against the unsharded GPU mesh, every counter,
    fingerprint and per-node scalar, and sampled whole rows."""
    cfg = SimConfig(capacity=65536 + 4096, initial_nodes=65536, init_mode=KB_INIT_CONVERGED, loss=0.01,
                    churn=0.001, seed=3)
    a = Sim(gpu, cfg)
    b = Sim(gpu, cfg, shards=4)
    assert b.shard_info()[1] == 4
    rng = np.random.default_rng(2)
    for r in range(4):
        a.step(1)
        b.step(1)
        assert a.stats() == b.stats(), f"round {r}"
        assert np.array_equal(a.fingerprints(), b.fingerprints()), f"round {r}"
        assert np.array_equal(a.scalars(), b.scalars()), f"round {r}"
        for i in rng.choice(cfg.capacity, 12, replace=False):
            assert np.array_equal(a.row(int(i)), b.row(int(i))), f"round {r} node {i}"
    a.close()
    b.close()


@pytest.mark.parametrize("name", [s["name"] for s in scenarios.SCENARIOS])
def test_gpu_matches_pyref_trace(gpu, name):
    traces = json.load(open(os.path.join(HERE, "golden", "traces.json")))
    sc = scenarios.BY_NAME[name]
    with Sim(gpu, sc["cfg"]) as g:
        scenarios.setup(g, sc)
        for r in range(sc["rounds"]):
            scenarios.apply_events(g, sc, r)
            g.step(1)
            assert scenarios.digest_sim(g) == traces[name]["rounds"][r], f"{name} round {r}"


def test_full_size_64k_against_oracle(gpu):
    """BASELINE configs[2] at full size (64K peers, 1% loss, 0.1% churn) for a few rounds: every
    fingerprint, scalar and counter, and a sample of complete stamp rows, against the OpenMP oracle."""
    cfg = SimConfig(capacity=65536 + 4096, initial_nodes=65536, init_mode=KB_INIT_CONVERGED, loss=0.01,
                    churn=0.001, seed=1)
    o = Sim(parity.oracle_lib(omp=True), cfg)
    g = Sim(gpu, cfg)
    rng = np.random.default_rng(0)
    for r in range(4):
        o.step(1)
        g.step(1)
        assert o.stats() == g.stats(), f"round {r}"
        assert np.array_equal(o.fingerprints(), g.fingerprints()), f"round {r}"
        assert np.array_equal(o.scalars(), g.scalars()), f"round {r}"
        for i in rng.choice(cfg.capacity, 24, replace=False):
            assert np.array_equal(o.row(int(i)), g.row(int(i))), f"round {r} node {i}"
            assert o.suspects(int(i)) == g.suspects(int(i))
    o.close()
    g.close()


def test_fingerprint_consistent_with_membership(gpu):
    """Size-independent property at bench scale: each node's incremental fingerprint equals the
    generate_fingerprint of the peer list the ABI reports for it (kb_fingerprint_of_set)."""
    import ctypes as C
    cfg = SimConfig(capacity=65536 + 4096, initial_nodes=65536, init_mode=KB_INIT_CONVERGED, loss=0.01,
                    churn=0.001, seed=2)
    lib = C.CDLL(parity.GPU_SO)
    f = lib.kb_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    with Sim(gpu, cfg) as g:
        g.step(12)
        fps = g.fingerprints()
        st = g.stats()
        assert st["alive"] == 65536 - st["churn_leaves"] + st["churn_joins"]
        assert st["next_free_id"] == 65536 + st["churn_joins"]
        for i in np.random.default_rng(1).choice(65536, 16, replace=False):
            if not g.is_running(int(i)):
                continue
            p = g.peers(int(i))
            assert f((C.c_uint32 * len(p))(*p), len(p), None, 0, None) == fps[i]


def test_deterministic_replay(gpu):
    cfg = SimConfig(capacity=5000, initial_nodes=4096, init_mode=KB_INIT_CONVERGED, loss=0.02, churn=0.002, seed=9)
    out = []
    for _ in range(2):
        with Sim(gpu, cfg) as g:
            g.step(20)
            out.append((g.stats(), g.fingerprints().copy(), g.rows()[::97].copy()))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


def test_kaboodle_view(gpu):
    import kaboodle_amd
    m = kaboodle_amd.Mesh(capacity=4, initial_nodes=0)
    for i, ident in enumerate(scenarios.CONFIG1_IDS):
        k = m.node(i)
        k.set_identity(ident)
        k.start()
    m.step(6)
    fps = {m.node(i).fingerprint() for i in range(4)}
    assert fps == {0x981285C8}
    assert m.node(0).self_addr() == "10.100.100.100:10000"
    assert sorted(m.node(2).peers()) == [f"10.100.100.100:1000{i}" for i in range(4)]


def test_profiling_levels(gpu):
    """Level 1 (the timed rounds' default) times the once-per-round counted kernels only, level 2 every
    launch, level 0 none; results do not depend on the level (kb_sim_set_profiling)."""
    cfg = SimConfig(capacity=5000, initial_nodes=4096, init_mode=KB_INIT_CONVERGED, loss=0.02, churn=0.002, seed=9)
    fps = []
    for level in (1, 2, 0):
        with Sim(gpu, cfg) as g:
            g.set_profiling(level)
            g.step(2)
            g.reset_kernel_time()
            g.step(3)
            names = set(g.kernel_breakdown())
            if level == 1:
                assert "k_rowpass" in names and "k_proc" not in names and "k_sortfast" not in names
            elif level == 2:
                assert {"k_rowpass", "k_proc", "k_sortfast", "k_route"} <= names
            else:
                assert not names
            fps.append((g.stats(), g.fingerprints().copy()))
    assert fps[0][0] == fps[1][0] == fps[2][0]
    assert np.array_equal(fps[0][1], fps[1][1]) and np.array_equal(fps[0][1], fps[2][1])
