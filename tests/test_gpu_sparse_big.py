"""configs[4] at its full size on one MI355X: 4,194,304 peers on the GPU's sparse rows, 5 % loss,
a two-way partition (rounds 3-11) healed by ping_addrs across the halves (src/lib.rs:268-297), socket_faithful.

The oracle cannot follow a 4M-peer mesh (every round delivers ~0.1 N Failed broadcasts to N receivers: ~10^12
delivery draws), so parity is split:
  * against the oracle's sparse rows at 131,072 peers, the same scenario: every counter, fingerprint and per-node
    scalar each round, sampled whole rows, suspect/curious tables and peer_states;
  * at 4,194,304 peers, properties that do not depend on the size: every sampled row's fingerprint equals
    generate_fingerprint over its peers() list (src/kaboodle.rs:71-83, computed from scratch), the counters'
    invariants (alive = N every round, one Failed broadcast per A2 removal, no Failed honoured), the partition
    dropping deliveries exactly while it lasts, and the layout's footprint staying far below a dense row."""
import os
import sys

import numpy as np
import pytest

import parity
from kaboodle_amd._ffi import Sim

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import sparse_big  # noqa: E402


@pytest.fixture(scope="module")
def gpu():
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    return parity.gpu_lib()


@pytest.mark.timeout(900)
def test_sparse_oracle_parity_131k(gpu):
    """The oracle, the unsharded GPU mesh and the same mesh as 8 row shards, in lock step: GPU = oracle every round
    (compare_sampled), and the sharded mesh = the unsharded one every round (digest_diff)."""
    n, rounds = 131072, 15
    case = sparse_big.scenario(n, every=256)
    o = Sim(parity.oracle_lib(omp=True), case["cfg"])
    g = Sim(gpu, case["cfg"])
    x = Sim(gpu, case["cfg"], shards=8)
    rng = np.random.default_rng(3)
    for r in range(rounds):
        parity.apply_events((o, g, x), case, r)
        o.step(1)
        g.step(1)
        x.step(1)
        diff = parity.compare_sampled(o, g, rng, nrows=6)
        assert not diff, f"round {r}: " + "; ".join(diff[:4])
        diff = sparse_big.digest_diff(g, x, rng, nrows=3)
        assert not diff, f"round {r}, 8 shards: " + "; ".join(diff[:4])
    st = g.stats()
    assert st["bcast_failed"] > 0 and st["drop_partition"] > 0 and st["sent_kpr"] > 0
    fo, fg, fx = o.sparse_footprint(), g.sparse_footprint(), x.sparse_footprint()
    assert (fo["exceptions"], fo["stamps"]) == (fg["exceptions"], fg["stamps"]) == (fx["exceptions"], fx["stamps"])
    o.close()
    g.close()
    x.close()


def _deltas(tr, key):
    v = [t[key] for t in tr]
    return [b - a for a, b in zip([0] + v[:-1], v)]


@pytest.mark.timeout(900)
def test_sparse_1m_sharded(gpu):
    """configs[3]'s peer count through the row-shard exchange (src/kaboodle.rs:188-226): 1,048,576 peers, converged
    start, 1 % loss, socket_faithful, as 8 in-process row shards = the unsharded mesh every round (counters, every
    fingerprint and scalar, sampled rows, suspect/curious tables, peer_states), with the 4M test's size-independent
    checks: generate_fingerprint(peers()) on sampled rows and the counters' invariants."""
    from kaboodle_amd._ffi import KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, KB_VARIANT_SPARSE_ROWS, SimConfig
    n, rounds, ext = 1 << 20, 7, (1 << 20) + 1
    cfg = SimConfig(capacity=n + 64, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.01, seed=21,
                    failed_mode=KB_FAILED_SOCKET_FAITHFUL, variant=KB_VARIANT_SPARSE_ROWS, sparse_row_cap=2048)
    # an external instance (a real Kaboodle behind the bridge) broadcasts Join at round 3: ~1 % of the
    # 1M running peers answer with a KnownPeers of capj ids (src/kaboodle.rs:284-304, :356-392), ~6M ids exported in
    # one round — beyond the export buffers' initial 4M ids, which grow to the round's wave-0 totals
    res = sparse_big.run_twin({"cfg": cfg}, rounds, shards=8, externals=[ext], join_rounds=[3])
    assert not res["failures"], res["failures"][:4]
    st = res["final_stats"]
    assert st["alive"] == n and st["alive_rounds"] == n * rounds
    assert st["bcast_failed"] == st["removed_timeout"] > 0
    assert not (st["removed_failed"] or st["drop_dead"] or st["churn_joins"])
    assert st["sent_kpr"] > 0 and st["drop_loss"] > 0
    ex = res["exported"]
    assert ex["kp_to_ext"] > 5000 and ex["ids"] > (1 << 22), ex


@pytest.mark.timeout(900)
def test_sparse_4m_partition_heal(gpu):
    """configs[4] at 4,194,304 peers, unsharded and as 8 row shards in lock step for its 16 rounds (digest_diff every
    round), with the size-independent checks on the sharded mesh."""
    n, rounds = 4 * 1024 * 1024, 16
    from kaboodle_amd._ffi import KB_STAT_NO_SF_FAILED_DROPS
    # the Failed lists' lost deliveries are not counted at 4M (KB_STAT_NO_SF_FAILED_DROPS: in socket_faithful mode
    # they change no state); the counting path is checked against the oracle at 131K and 2K
    case = sparse_big.scenario(n, every=256, row_cap=2048, stat_flags=KB_STAT_NO_SF_FAILED_DROPS)
    res = sparse_big.run_twin(case, rounds, shards=8, nrows=2)
    assert not res["failures"], res["failures"][:4]
    tr = res["trajectory"]
    part = _deltas(tr, "drop_partition")
    assert all(p == 0 for p in part[:3]) and all(p > 0 for p in part[3:12]) and all(p == 0 for p in part[12:]), part
    fb = _deltas(tr, "bcast_failed")
    assert all(f > 0 for f in fb[5:]), fb
    assert not sparse_big.check_invariants(res["final_stats"], n, rounds)
    fp = res["footprint"]
    assert fp["bytes"] / n < 4096 and fp["max_row_entries"] <= 2048, fp    # dense row: 4 MiB
