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
    n, rounds = 131072, 15
    case = sparse_big.scenario(n, every=256)
    o = Sim(parity.oracle_lib(omp=True), case["cfg"])
    g = Sim(gpu, case["cfg"])
    rng = np.random.default_rng(3)
    for r in range(rounds):
        parity.apply_events((o, g), case, r)
        o.step(1)
        g.step(1)
        diff = parity.compare_sampled(o, g, rng, nrows=6)
        assert not diff, f"round {r}: " + "; ".join(diff[:4])
    st = g.stats()
    assert st["bcast_failed"] > 0 and st["drop_partition"] > 0 and st["sent_kpr"] > 0
    fo, fg = o.sparse_footprint(), g.sparse_footprint()
    assert (fo["exceptions"], fo["stamps"]) == (fg["exceptions"], fg["stamps"])
    o.close()
    g.close()


@pytest.mark.timeout(900)
def test_sparse_4m_partition_heal(gpu):
    n, rounds = 4 * 1024 * 1024, 16
    res = sparse_big.run(n, rounds, every=256, row_cap=2048, check_rows=3, verbose=False)
    assert not res["failures"], res["failures"][:4]
    tr = res["trajectory"]
    part = [t["drop_partition"] for t in tr]
    assert all(p == 0 for p in part[:3]) and all(p > 0 for p in part[3:12]) and all(p == 0 for p in part[12:]), part
    assert all(t["failed_bcasts"] > 0 for t in tr[5:]), [t["failed_bcasts"] for t in tr]
    last = [t for t in tr if "bytes_per_row" in t][-1]
    assert last["bytes_per_row"] < 4096 and last["max_row_entries"] <= 2048, last    # dense row: 4 MiB
