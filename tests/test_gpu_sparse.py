"""The configs[4] layout on the GPU (KB_VARIANT_SPARSE_ROWS): every view as a shared base set,
one sorted entry list per row (exceptions and explicit stamps), A3 from the base's rotated order, the indirect-
ping candidates by select over the base's prefix counts, KnownPeersRequest replies from the explicit stamps and
the fingerprint from base prefix folds corrected at the exceptions (src/structs.rs:12-41, src/kaboodle.rs:71-83,
:483-501, :558-703).  The HIP engine must reproduce the oracle's sparse rows (which reproduce the dense oracle,
tests/test_sparse.py) bit for bit: every state byte, every round."""
import numpy as np
import pytest

import parity
from kaboodle_amd._ffi import (KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_VARIANT_SPARSE_ROWS, KbError, Sim,
                               SimConfig)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    return parity.gpu_lib()


def sparse(case: dict, **kw) -> dict:
    return parity.with_cfg(case, variant=KB_VARIANT_SPARSE_ROWS, track_latency=0, **kw)


CASES = parity.standard_cases()


@pytest.mark.parametrize("name,case,rounds", CASES, ids=[c[0] for c in CASES])
def test_sparse_parity_every_round(gpu, name, case, rounds):
    """The standard matrix on the GPU's sparse rows against the oracle's: complete state every round and
    peer_states() of every node."""
    ok, msg, _ = parity.run_case(sparse(case), rounds, peer_states=True)
    assert ok, f"{name} (sparse rows): {msg}"


def test_sparse_small_row_cap(gpu):
    """A row cap far below the capacity: the standard converged cases keep their rows within it (views stay
    within a few entries of the base), and a row that outgrows it is KB_CAPACITY, never a truncation."""
    case = {"cfg": SimConfig(capacity=512, initial_nodes=512, init_mode=KB_INIT_CONVERGED, loss=0.05, seed=7,
                             failed_mode=KB_FAILED_SOCKET_FAITHFUL)}
    ok, msg, _ = parity.run_case(sparse(case, sparse_row_cap=160), 20)
    assert ok, msg
    g = Sim(gpu, SimConfig(capacity=256, initial_nodes=256, variant=KB_VARIANT_SPARSE_ROWS, sparse_row_cap=16))
    with pytest.raises(KbError):                     # join start: every member is an entry, 256 > 16
        g.step(4)
    g.close()


TRUNC_CASES = {
    # views of > 567 ids: every Join response is a sampled (truncated) one
    "trunc_1200": ({"cfg": SimConfig(capacity=1300, initial_nodes=1200, init_mode=KB_INIT_CONVERGED, churn=0.01, seed=23)}, 6),
    "trunc_loss_1800": ({"cfg": SimConfig(capacity=2000, initial_nodes=1800, init_mode=KB_INIT_CONVERGED, churn=0.005,
                                          loss=0.02, seed=5, id_len=3)}, 8),
}


@pytest.mark.parametrize("name", sorted(TRUNC_CASES))
def test_sparse_truncated_join_responses(gpu, name):
    """Join responses sampled by the keyed permutation over base Δ x, minus the joiners later entries inserted."""
    case, rounds = TRUNC_CASES[name]
    ok, msg, st = parity.run_case(sparse(case), rounds)
    assert ok and st["join_responses"] > 0, f"{name}: {msg}"


def partition_case(n: int, every: int, seed: int = 9, stat_flags: int = 0) -> dict:
    """configs[4]'s scenario at n peers: converged start, 5 % loss, two halves cut off
    for rounds 3-11, healed at round 12 by every `every`-th peer pinging the other half (ping_addrs), in the
    deployment-faithful reading of Failed."""
    cfg = SimConfig(capacity=n, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.05, partition_groups=2,
                    partition_start=3, partition_end=12, seed=seed, failed_mode=KB_FAILED_SOCKET_FAITHFUL,
                    variant=KB_VARIANT_SPARSE_ROWS, stat_flags=stat_flags)
    return {"cfg": cfg, "events": {12: [("ping", i, [(i + n // 2) % n]) for i in range(0, n, every)]}}


@pytest.mark.parametrize("n,rounds,every,flags", [(2048, 40, 64, 0), (2048, 40, 64, 1)],
                         ids=["2048", "2048-no-sf-failed-drops"])   # 131K: test_gpu_sparse_big.py
def test_sparse_partition_heal(gpu, n, rounds, every, flags):
    """The partition + heal scenario against the oracle's sparse rows: counters, every fingerprint and per-node
    scalar each round, sampled whole rows, suspect/curious tables and peer_states; and with
    KB_STAT_NO_SF_FAILED_DROPS (the Failed lists' drops not counted) on both."""
    case = partition_case(n, every, stat_flags=flags)
    o = Sim(parity.oracle_lib(omp=True), case["cfg"])
    g = Sim(gpu, case["cfg"])
    rng = np.random.default_rng(n)
    for r in range(rounds):
        parity.apply_events((o, g), case, r)
        o.step(1)
        g.step(1)
        diff = parity.compare_sampled(o, g, rng, nrows=16)
        assert not diff, f"n={n} round {r}: " + "; ".join(diff[:4])
    fo, fg = o.sparse_footprint(), g.sparse_footprint()
    assert (fo["rows_based"], fo["exceptions"], fo["stamps"]) == (fg["rows_based"], fg["exceptions"], fg["stamps"]), (fo, fg)
    o.close()
    g.close()


SHARD_CASES = [c for c in CASES if c[1]["cfg"].capacity > 4]   # config1_2x2's 4 ids cannot make 3 shards


@pytest.mark.parametrize("name,case,rounds", SHARD_CASES, ids=[c[0] for c in SHARD_CASES])
def test_sparse_sharded_parity_every_round(gpu, name, case, rounds):
    """The standard matrix on sparse rows split into 3 row shards inside one process (kb_sim_create_local): every
    wave's records routed on the sender's shard and all-to-all-v'd to the receiver's, the broadcast lists
    all-gathered, restarts moving the row (and its observer) between shards (src/kaboodle.rs:188-226, :394-548) —
    the complete state equals the oracle's every round."""
    ok, msg, _ = parity.run_case(sparse(case), rounds, shards=3)
    assert ok, f"{name} (sparse rows, 3 shards): {msg}"
