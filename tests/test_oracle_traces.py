"""The C oracle against the committed round traces of tests/pyref.py (tests/golden/traces.json), and a
live pin of the oracle against pyref on the full state (not only digests) for a few scenarios.

pyref is an independent dict-based restatement written in the reference's own shape
(known_peers map per peer, literal zlib fingerprint); agreement of the two on every round of every
scenario is what pins the oracle.  Parity with the Rust reference itself is unpinned by any reference
test (it has none, and it is entropy-seeded: SURVEY.md §8c)."""
import json
import os

import numpy as np
import pytest
from dataclasses import replace

import pyref
import scenarios
from kaboodle_amd._ffi import Sim
from parity import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
TRACES = json.load(open(os.path.join(HERE, "golden", "traces.json")))


@pytest.mark.parametrize("name", [s["name"] for s in scenarios.SCENARIOS])
def test_oracle_matches_trace(name):
    sc = scenarios.BY_NAME[name]
    want = TRACES[name]["rounds"]
    assert len(want) == sc["rounds"]
    with Sim(oracle_lib(), sc["cfg"]) as o:
        scenarios.setup(o, sc)
        for r in range(sc["rounds"]):
            scenarios.apply_events(o, sc, r)
            o.step(1)
            got = scenarios.digest_sim(o)
            assert got == want[r], f"{name} round {r}: {got} != {want[r]}"
        assert o.stats()["first_converged_round"] == TRACES[name]["first_converged"]


@pytest.mark.parametrize("name", ["config1", "churn40", "partition", "stop_start", "rebase", "identity_change"])
def test_oracle_live_pin(name):
    """Full-state comparison with pyref, every round: rows, suspects, curious, peer_states (across the
    64-round stamp-window rebases in "rebase"), fingerprints, counters."""
    sc = scenarios.BY_NAME[name]
    pm = scenarios.pymesh_of(sc)
    measured = 0
    with Sim(oracle_lib(), replace(sc["cfg"], track_latency=1)) as o:
        scenarios.setup(o, sc)
        scenarios.setup(pm, sc)
        for r in range(sc["rounds"]):
            scenarios.apply_events(o, sc, r)
            scenarios.apply_events(pm, sc, r)
            o.step(1)
            pm.step()
            for i in range(sc["cfg"].capacity):
                assert np.array_equal(o.row(i), np.array(pm.row(i), np.uint8)), f"round {r} node {i} row"
                assert o.suspects(i) == pm.suspects(i), f"round {r} node {i} suspects"
                assert o.curious(i) == pm.curious_view(i), f"round {r} node {i} curious"
                ps = o.peer_states(i)
                assert ps == pm.peer_states(i), f"round {r} node {i} peer_states"
                measured += sum(1 for e in ps if e[3] != 0xFFFFFFFF)
                want = pyref.view_fingerprint(pm.peers[i].known) if pm.peers[i].running else 0
                assert o.fingerprint(i) == want if pm.peers[i].running else True
            st = o.stats()
            assert {k: st[k] for k in scenarios.STAT_KEYS} == {k: pm.stats[k] for k in scenarios.STAT_KEYS}
            assert st["agree"] == pm.agree
    assert measured > 0, "no latency was ever measured: the EWMA is untested"


@pytest.mark.parametrize("name", ["churn40", "stop_start"])
def test_alive_rounds_counts_every_round(name):
    """kb_stats.alive_rounds (what bench.py's `value` divides by wall time) is the running-peer count of
    every simulated round, summed: the peers running after a round are those its tick counted."""
    sc = scenarios.BY_NAME[name]
    with Sim(oracle_lib(), sc["cfg"]) as o:
        scenarios.setup(o, sc)
        total = o.stats()["alive_rounds"]
        assert total == 0
        for r in range(sc["rounds"]):
            scenarios.apply_events(o, sc, r)
            o.step(1)
            total += o.stats()["alive"]
            assert o.stats()["alive_rounds"] == total, f"{name} round {r}"
