"""The configs[4] representation: the oracle's KB_VARIANT_SPARSE_ROWS keeps every view as
a shared base set (the initial members), per-row exceptions and an explicit list of the non-ancient stamps,
and runs A3 from the base's rotated order, KnownPeersRequest replies from the explicit list and the
fingerprint from base prefix folds corrected at the exceptions (src/structs.rs:12-41, src/kaboodle.rs:71-83,
:483-501, :662-675).  It must reproduce the dense oracle bit for bit: every state byte, every round, on the
standard matrix and on the partition + heal scenario of configs[4] (5 % loss, socket_faithful: Failed never
honoured, the deployment reading of Q1), at sizes the CPU suite finishes in seconds."""
import ctypes as C
from dataclasses import replace

import numpy as np
import pytest

import parity
from kaboodle_amd._ffi import KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, Sim, SimConfig

SPARSE = 4   # KB_VARIANT_SPARSE_ROWS


def _pair(case):
    cfg = replace(case["cfg"], track_latency=0)
    return Sim(parity.oracle_lib(), cfg), Sim(parity.oracle_lib(), replace(cfg, variant=SPARSE))


def footprint(sim) -> dict:
    """kbo_sparse_footprint: exceptions, explicit stamps and the largest row, in entries and bytes"""
    f = sim.lib.lib.kbo_sparse_footprint
    f.restype = C.c_int
    out = (C.c_uint64 * 6)()
    assert f(sim.h, out, 6) == 0
    keys = ("rows_based", "exceptions", "stamps", "max_row_entries", "bytes", "rows")
    return dict(zip(keys, (int(v) for v in out)))


CASES = [c for c in parity.standard_cases()]


@pytest.mark.parametrize("name,case,rounds", CASES, ids=[c[0] for c in CASES])
def test_sparse_equals_dense(name, case, rounds):
    d, s = _pair(case)
    rng = np.random.default_rng(2)
    parity.setup(d, case)
    parity.setup(s, case)
    for r in range(rounds):
        parity.apply_events((d, s), case, r)
        d.step(1)
        s.step(1)
        diff = parity.diff_states(parity.state_of(d), parity.state_of(s))
        if not diff:
            diff = parity.diff_peer_states(d, s, rng.choice(case["cfg"].capacity, min(16, case["cfg"].capacity), replace=False))
        assert not diff, f"{name} round {r}: " + "; ".join(diff[:4])
    d.close()
    s.close()


def test_partition_heal_sparse_socket_faithful():
    """configs[4]'s scenario scaled down: converged start, 5 % loss, two halves cut off for rounds 3-11,
    healed at round 12 by injected ping_addrs across the halves, socket_faithful.
    Bit-exact with the dense oracle every round; the views stay within a few exceptions of the base and
    the explicit stamps stay a small fraction of a dense row."""
    n = 2048
    cfg = SimConfig(capacity=n, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.05, partition_groups=2,
                    partition_start=3, partition_end=12, seed=9, failed_mode=KB_FAILED_SOCKET_FAITHFUL)
    case = {"cfg": cfg, "events": {12: [("ping", i, [(i + n // 2) % n]) for i in range(0, n, 64)]}}
    d, s = _pair(case)
    rng = np.random.default_rng(4)
    for r in range(40):
        parity.apply_events((d, s), case, r)
        d.step(1)
        s.step(1)
        diff = parity.compare_sampled(d, s, rng, nrows=32)
        assert not diff, f"round {r}: " + "; ".join(diff[:4])
    fp = footprint(s)
    assert fp["rows"] == n and fp["rows_based"] == n
    assert fp["exceptions"] / n < 8 and fp["max_row_entries"] < n / 8, fp
    d.close()
    s.close()


def test_sparse_refuses_latency():
    with pytest.raises(Exception):
        Sim(parity.oracle_lib(), SimConfig(capacity=16, initial_nodes=16, variant=SPARSE, track_latency=1))


def test_no_sf_failed_drops_changes_only_the_count():
    """KB_STAT_NO_SF_FAILED_DROPS (kb_config.stat_flags): socket_faithful Failed broadcasts change no state, so
    skipping the count of their lost deliveries leaves every state byte, fingerprint and counter but drop_bcast
    as it was; drop_bcast keeps the Join / Probe losses only."""
    from dataclasses import replace
    from kaboodle_amd._ffi import KB_STAT_NO_SF_FAILED_DROPS, KB_VARIANT_SPARSE_ROWS
    base = SimConfig(capacity=600, initial_nodes=512, init_mode=KB_INIT_CONVERGED, loss=0.05, churn=0.002,
                     partition_groups=2, partition_start=3, partition_end=12, seed=4, failed_mode=KB_FAILED_SOCKET_FAITHFUL)
    for variant in (0, KB_VARIANT_SPARSE_ROWS):
        a = Sim(parity.oracle_lib(), replace(base, variant=variant))
        b = Sim(parity.oracle_lib(), replace(base, variant=variant, stat_flags=KB_STAT_NO_SF_FAILED_DROPS))
        fewer = 0
        for r in range(30):
            a.step(1)
            b.step(1)
            sa, sb = parity.state_of(a), parity.state_of(b)
            da, db = sa["stats"].pop("drop_bcast"), sb["stats"].pop("drop_bcast")
            assert not parity.diff_states(sa, sb), f"variant {variant} round {r}"
            assert db <= da
            fewer += db < da
        assert fewer > 0 and b.stats()["bcast_failed"] > 0
        a.close()
        b.close()
