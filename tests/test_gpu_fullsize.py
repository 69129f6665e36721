"""Full-size parity on an MI355X: the HIP library against the OpenMP oracle at the sizes the bench and the
wide-row configs run, through the C ABI.

- configs[2] exactly as the driver's `bench.py --steps 20 --warmup 5` runs it (65,536 peers, capacity
  73,728, 1 % loss, 0.1 %/round churn, faults until round 25, the latency EWMA on, A3 in exact-instant order;
  tests/test_bench.py checks this config against bench.rank_config) over the whole benched horizon (the 25
  rounds of warmup + timed steps), every round: counters, every fingerprint and per-node scalar, and sampled whole
  rows, suspect and curious tables and peer_states with latency (src/kaboodle.rs:746-779, :789-817).
- a 140K-id mesh: rows wider than RESP_LDS_W = 131,072 ids, so Join responses take the HBM-scratch
  path a >= 1M-id mesh takes (kb_sim.hip, the W > RESP_LDS_W branch), unsharded and as 8 row shards.
- configs[4] scaled to one GPU: 32,768 peers (dense rows; the sparse rows run it at 131K and 4M in
  test_gpu_sparse_big.py), 5 % loss, a two-way partition, then the heal by injected
  ping_addrs across the halves.

Each scenario is split into chunks of rounds (one test each, sharing the handles) so no single test
runs for minutes without output."""
import numpy as np
import pytest

import parity
from kaboodle_amd._ffi import KB_INIT_CONVERGED, KB_VARIANT_EXACT_LRU, Sim, SimConfig

pytestmark = pytest.mark.gpu

BENCH_CFG = SimConfig(capacity=65536 + 8192, initial_nodes=65536, init_mode=KB_INIT_CONVERGED, loss=0.01,
                      churn=0.001, fault_end_round=25, seed=1, track_latency=1,
                      variant=KB_VARIANT_EXACT_LRU)   # bench.rank_config, --steps 20 --warmup 5 (A3 in exact-instant order)


class Pair:
    """An oracle handle and a GPU handle advanced in lock step."""

    def __init__(self, cfg, shards=0, events=None, omp=True):
        import kaboodle_amd
        kaboodle_amd.require_gpu()
        self.o = Sim(parity.oracle_lib(omp=omp), cfg)
        self.g = Sim(parity.gpu_lib(), cfg, shards=shards)
        self.events = events or {}
        self.round = 0
        self.rng = np.random.default_rng(cfg.seed)

    def advance(self, upto, nrows=24):
        while self.round < upto:
            parity.apply_events((self.o, self.g), {"events": self.events}, self.round)
            self.o.step(1)
            self.g.step(1)
            d = parity.compare_sampled(self.o, self.g, self.rng, nrows)
            assert not d, f"round {self.round}: " + "; ".join(d[:4])
            self.round += 1

    def close(self):
        self.o.close()
        self.g.close()


@pytest.fixture(scope="module")
def horizon():
    p = Pair(BENCH_CFG)
    yield p
    p.close()


@pytest.mark.parametrize("upto", [7, 14, 21, 25])
def test_bench_horizon_64k(horizon, upto):
    """The bench's workload over exactly the rounds the driver's command runs (5 warmup + 20 timed = rounds 0-24,
    the faulty ones), in chunks."""
    horizon.advance(upto)
    if upto == 25:
        st = horizon.g.stats()
        assert st["churn_joins"] > 0 and st["removed_failed"] > 0 and st["join_responses"] > 0


@pytest.fixture(scope="module")
def wide():
    cfg = SimConfig(capacity=140000, initial_nodes=136000, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.001,
                    seed=5)
    p = Pair(cfg)
    yield p
    p.close()


@pytest.mark.parametrize("upto", [2, 4])
def test_wide_rows_140k(wide, upto):
    """W = 147,456: Join responses by wave, the rows read in place (k_resp_wave<true>)."""
    wide.advance(upto, nrows=12)
    if upto == 4:
        assert wide.g.stats()["join_responses"] > 0


def test_wide_rows_140k_sharded(wide):
    """The same mesh as 8 row shards (kb_sim_create_local, all-to-all-v of every wave) equals the
    unsharded GPU mesh after 4 rounds."""
    cfg = wide.g.cfg
    with Sim(parity.gpu_lib(), cfg, shards=8) as s:
        s.step(wide.round)
        a, b = wide.g, s
        assert a.stats() == b.stats()
        assert np.array_equal(a.fingerprints(), b.fingerprints())
        assert np.array_equal(a.scalars(), b.scalars())
        for i in np.random.default_rng(3).choice(cfg.capacity, 16, replace=False):
            assert np.array_equal(a.row(int(i)), b.row(int(i))), f"node {i}"
    assert wide.g.debug_paths() & (2 | 4 | 256), "no Join response took a wide-row path"


@pytest.fixture(scope="module")
def split():
    n = 32768
    cfg = SimConfig(capacity=n, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.05, partition_groups=2,
                    partition_start=3, partition_end=12, seed=9)
    # heal: every 256th peer of each half is told an address in the other half (Kaboodle::ping_addrs)
    heal = {12: [("ping", i, [(i + n // 2) % n]) for i in range(0, n, 256)]}
    p = Pair(cfg, events=heal)
    yield p
    p.close()


@pytest.mark.parametrize("upto", [6, 12, 18, 24])
def test_partition_heal_32k(split, upto):
    """configs[4] on one GPU: 5 % loss, the halves cut off for rounds 3-11, healed at round 12."""
    split.advance(upto, nrows=16)
    if upto == 24:
        st = split.g.stats()
        assert st["drop_partition"] > 0


# ---- a long quiet tail: stamps age through many window rebases (k_rebase's saturation edge, the A3
# ---- rotation base sweeping the ancient peers, timeouts of dead peers) -----------------------------
LONG_N = 8192


def _long_cfg(mode):
    from kaboodle_amd._ffi import KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL
    return SimConfig(capacity=LONG_N + 512, initial_nodes=LONG_N, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.001,
                     fault_end_round=25, seed=1,
                     failed_mode=KB_FAILED_SOCKET_FAITHFUL if mode == "sock" else KB_FAILED_SIM_SENDER)


@pytest.fixture(scope="module", params=["sock", "sim"])
def long_tail(request):
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    cfg = _long_cfg(request.param)
    o, g = Sim(parity.oracle_lib(omp=True), cfg), Sim(parity.gpu_lib(), cfg)
    yield {"o": o, "g": g, "round": 0}
    o.close()
    g.close()


@pytest.mark.parametrize("upto", [300, 600, 900, 1200])
def test_long_tail_8k(long_tail, upto):
    """configs[2]'s shape at 8K peers, both failed modes, 1200 rounds (18 window rebases): every stamp row,
    fingerprint, scalar and counter equal the oracle's every 100 rounds."""
    o, g = long_tail["o"], long_tail["g"]
    while long_tail["round"] < upto:
        o.step(100)
        g.step(100)
        long_tail["round"] += 100
        r = long_tail["round"]
        assert o.stats() == g.stats(), f"round {r}: counters"
        assert np.array_equal(o.fingerprints(), g.fingerprints()), f"round {r}: fingerprints"
        assert np.array_equal(o.scalars(), g.scalars()), f"round {r}: scalars"
        ro, rg = o.rows(), g.rows()
        if not np.array_equal(ro, rg):
            bad = np.argwhere(ro != rg)
            i, j = bad[0]
            pytest.fail(f"round {r}: {len(bad)} stamp bytes differ, first node {i} peer {j}: {ro[i, j]} != {rg[i, j]}")
