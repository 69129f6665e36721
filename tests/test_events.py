"""Event streams — `handle_known_peers_events` (src/events.rs:18-125) behind Kaboodle::discover_peers /
discover_departures / discover_fingerprint_changes (src/lib.rs:186-263), as kb_sim_watch +
kb_sim_events (include/kaboodle_sim.h).

One drain is one batch: discovered / departed are the NET membership change of the watched node since
the previous drain (ascending ids), the fingerprint is reported when the map is non-empty and it
differs from the last one reported (events.rs:103-122).  The CPU tests pin the oracle's batches to
the diff of its own peer lists; the GPU tests require the HIP library's batches to equal the
oracle's, unsharded and as row shards."""
import ctypes as C

import pytest

import parity
from kaboodle_amd._ffi import KB_INIT_CONVERGED, KbError, Sim, SimConfig


def _cases():
    by = {name: (case, rounds) for name, case, rounds in parity.standard_cases()}
    return [
        ("config1_2x2", *by["config1_2x2"], [0, 1, 2, 3], 1),
        ("join_64", *by["join_64"], [0, 13, 63], 1),
        ("churn_loss_512", *by["churn_loss_512"], [0, 1, 200, 511, 600], 1),
        ("churn_loss_512_every3", *by["churn_loss_512"], [7, 300], 3),
        ("stop_start", *by["stop_start"], [5, 17, 120, 0], 1),
        ("partition_heal", *by["partition_heal"], [0, 128, 255], 2),
    ]


CASES = _cases()


@pytest.mark.parametrize("name,case,rounds,watched,every", CASES, ids=[c[0] for c in CASES])
def test_oracle_events_are_peer_list_diffs(name, case, rounds, watched, every):
    lib = parity.oracle_lib()
    ok, msg, n = parity.run_events_case(case, rounds, watched, every, libs=(lib, lib))
    assert ok, f"{name}: {msg}"
    assert n > 0


def test_oracle_first_drain_reports_everything():
    """Attached empty at creation (src/lib.rs:112): the first drain discovers every member, self
    included, and reports the fingerprint (initial previous fingerprint 0)."""
    with Sim(parity.oracle_lib(), SimConfig(capacity=64, initial_nodes=64, init_mode=KB_INIT_CONVERGED)) as s:
        s.watch(3)
        s.step(1)
        d, p, fp, ch = s.events(3)
        assert d == s.peers(3) and 3 in d and p == []
        assert ch and fp == s.fingerprint(3)
        # nothing changed since: empty batch, no fingerprint event
        d, p, fp2, ch = s.events(3)
        assert (d, p, ch) == ([], [], False) and fp2 == fp


def test_oracle_events_errors_and_size_query():
    lib = parity.oracle_lib()
    with Sim(lib, SimConfig(capacity=32, initial_nodes=32, init_mode=KB_INIT_CONVERGED)) as s:
        s.step(1)
        nd, npp, fp, ch = C.c_size_t(), C.c_size_t(), C.c_uint32(), C.c_int()
        with pytest.raises(KbError):                       # not watched
            lib.call("sim_events", s.h, 1, None, 0, C.byref(nd), None, 0, C.byref(npp), C.byref(fp), C.byref(ch))
        s.watch(1)
        s.watch(1)                                         # idempotent
        # size query drains nothing
        lib.call("sim_events", s.h, 1, None, 0, C.byref(nd), None, 0, C.byref(npp), C.byref(fp), C.byref(ch))
        assert nd.value == 32 and npp.value == 0 and ch.value == 1
        small = (C.c_uint32 * 4)()
        with pytest.raises(KbError):                       # too small: KB_CAPACITY, nothing drained
            lib.call("sim_events", s.h, 1, small, 4, C.byref(nd), None, 0, C.byref(npp), C.byref(fp), C.byref(ch))
        d, p, _, ch2 = s.events(1)
        assert d == list(range(32)) and p == [] and ch2


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [0, 3], ids=["unsharded", "x3"])
@pytest.mark.parametrize("name,case,rounds,watched,every", CASES, ids=[c[0] for c in CASES])
def test_gpu_events_match_oracle(name, case, rounds, watched, every, shards):
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    if shards and case["cfg"].capacity < 9:
        pytest.skip("too few ids for 3 shards")
    ok, msg, n = parity.run_events_case(case, rounds, watched, every, shards=shards)
    assert ok, f"{name}: {msg}"
    assert n > 0


@pytest.mark.gpu
def test_gpu_events_64k_drain():
    """Full workload width (capacity 71729, 2242 bitset words: three passes of the 1024-thread diff):
    the first drain of a converged row is the whole row; after churn rounds the batch equals the
    oracle-free peer-list diff of the HIP library itself."""
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    cfg = SimConfig(capacity=71729, initial_nodes=65536, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.001,
                    seed=1)
    with Sim(parity.gpu_lib(), cfg) as g:
        g.watch(12345)
        g.step(1)
        d, p, fp, ch = g.events(12345)
        before = g.peers(12345)
        assert d == before and p == [] and ch and fp == g.fingerprint(12345)
        g.step(3)
        d, p, fp2, ch = g.events(12345)
        after = g.peers(12345)
        assert d == sorted(set(after) - set(before)) and p == sorted(set(before) - set(after))
        assert ch == (fp2 != fp)


@pytest.mark.gpu
def test_gpu_discover_channels_2x2():
    """The Python mirror of discover_peers / discover_next_peer / discover_departures /
    discover_fingerprint_changes (src/lib.rs:186-263) on the config-1 2x2 mesh: every peer is
    discovered once, the last fingerprint reported is the golden 0x981285c8, and a stopped peer
    (silent stop, src/lib.rs:159-183) arrives on the departure channel once it is removed."""
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    with kaboodle_amd.Mesh(SimConfig(capacity=4, initial_nodes=0)) as m:
        names = [b"top-left", b"top-right", b"bottom-left", b"bottom-right"]
        k = [m.node(i) for i in range(4)]
        for i, n in enumerate(names):
            k[i].set_identity(n)
        peers, nxt = k[0].discover_peers(), k[0].discover_next_peer()
        deps, fps = k[0].discover_departures(), k[0].discover_fingerprint_changes()
        for x in k:
            x.start()
        m.step(6)
        got = peers.drain()                       # (addr, identity) per discovered peer (src/lib.rs:221-236)
        ids = {m.format_addr(i): i for i in range(4)}
        assert sorted(ids[a] for a, _ in got) == [0, 1, 2, 3]
        assert all(ident == names[ids[a]] for a, ident in got)
        assert len(nxt.drain()) == 1 and nxt.closed
        f = fps.drain()
        assert f and f[-1] == 0x981285C8 == k[0].fingerprint()
        k[3].stop()
        for _ in range(30):
            m.step(1)
            if 3 not in m.peers(0):
                break
        assert 3 not in m.peers(0)
        assert deps.drain() == [m.format_addr(3)]
        assert peers.drain() == []
        assert fps.drain()[-1] == k[0].fingerprint()


@pytest.mark.gpu
def test_gpu_events_rccl_rank_world1():
    """Event drains on the RCCL transport's handle (kb_sim_create_rank, 1-rank communicator)."""
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    from kaboodle_amd._ffi import rccl_unique_id
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}["churn_loss_512"]
    lib = parity.gpu_lib()
    g = Sim(lib, case["cfg"], rank=0, world=1, uid=rccl_unique_id(lib))
    ok, msg, n = parity.run_events_case(case, rounds, [0, 300, 600], gpu=g)
    assert ok, msg
    assert n > 0


def _handoff(impls):
    """Observers across a restart: node 5 is watched and restarts at a fresh address; an observer
    also attached to that new address before the round gives way to the instance's own (one batch stream, no
    duplicate).  Node 6 is not watched; an observer attached to its new address after start() returned starts
    from the inherited map, so its batches carry only later changes, not the whole map."""
    cfg = impls[0][1]
    sims = [Sim(lib, c) for lib, c in impls]
    for s in sims:
        s.watch(5)
    out = []
    for r in range(14):
        for s in sims:
            if r == 2:
                s.stop_node(5)
                s.stop_node(6)
            if r == 4:
                a, b = s.restart_node(5), s.restart_node(6)
                assert (a, b) == (cfg.initial_nodes, cfg.initial_nodes + 1)
                s.watch(a)
                s.watch(b)
            s.step(1)
        if r >= 4:
            ev = [(s.events(cfg.initial_nodes), s.events(cfg.initial_nodes + 1)) for s in sims]
            out.append(ev)
            if r == 4:                             # the new address's first batch: what changed since start()
                (_, (d6, p6, _, _)) = ev[0]
                assert len(d6) <= 2 and p6 == [], (d6, p6)
            assert all(e == ev[0] for e in ev), f"round {r}: {ev}"
    for s in sims:
        with pytest.raises(KbError):               # the old address has no observer left
            s.events(5)
        s.close()
    return out


def test_oracle_observer_handoff_on_restart():
    cfg = SimConfig(capacity=48, initial_nodes=40, init_mode=KB_INIT_CONVERGED, loss=0.02, seed=3)
    _handoff([(parity.oracle_lib(), cfg)])


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 4], ids=["dense", "sparse"])
def test_gpu_observer_handoff_on_restart(variant):
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    cfg = SimConfig(capacity=48, initial_nodes=40, init_mode=KB_INIT_CONVERGED, loss=0.02, seed=3, variant=variant)
    _handoff([(parity.oracle_lib(), cfg), (parity.gpu_lib(), cfg)])
