"""External peers: real Kaboodle instances attached to a simulated mesh through a bridge.  An
address marked external never runs in the mesh; records simulated peers address to it are exported instead of
delivered (the real network carries them, src/kaboodle.rs:197-226), and what the bridge decodes from a real socket
is injected as that peer's wave-0 records of the next round (:394-403).  The CPU tests pin the oracle's rules; the
GPU tests (test_gpu_external in tests/test_gpu_parity.py) require the HIP engines to export and absorb identically."""
import pytest

import parity
from kaboodle_amd._ffi import KB_INIT_CONVERGED, KbError, Sim, SimConfig
from parity import K_ACK, K_JOIN, K_KP, K_KPR, K_PING

CFG = SimConfig(capacity=48, initial_nodes=40, init_mode=KB_INIT_CONVERGED, seed=5)


def test_ping_from_external_is_acked_and_exported():
    with Sim(parity.oracle_lib(), CFG) as s:
        s.set_external(44)
        s.step(1)
        s.inject(44, 3, K_PING)
        s.step(1)
        ex = s.exported()
        acks = [e for e in ex if e[3] == 44 and e[5] == K_ACK]
        assert len(acks) == 1
        rnd, wave, sender, dest, seq, kind, a, fp, n, ids = acks[0]
        assert (rnd, wave, sender, a) == (1, 1, 3, 3) and fp == s.fingerprint(3) and n == 41   # 40 + the external peer
        assert 44 in s.peers(3)                       # the prologue inserted the external sender (:406-415)
        assert not s.is_running(44) and s.stats()["exported"] == len(ex)
        assert 44 not in s.peers(5)                   # only the peer it talked to knows it


def test_known_peers_request_and_list_from_external():
    with Sim(parity.oracle_lib(), CFG) as s:
        s.set_external(45)
        s.inject(45, 7, K_KP, ids=[41, 42])           # a KnownPeers list from outside: unknown ids inserted (:448-472)
        s.inject(45, 7, K_KPR, fp=1, n=1)             # then a KnownPeersRequest: a KnownPeers reply of fresh entries
        s.step(1)
        ex = s.exported()
        kp = [e for e in ex if e[5] == K_KP]
        assert kp and kp[0][2] == 7 and kp[0][3] == 45 and not {7, 45} & set(kp[0][9])
        assert not {41, 42} & set(kp[0][9])           # KnownPeers inserts are Known(r - 10): too old to share (:483-501)
        assert {41, 42, 45} <= set(s.peers(7))


def test_join_broadcast_from_external():
    """An external peer's Join (maybe_broadcast_join, src/kaboodle.rs:228-251) reaches every running simulated peer in
    the next round's broadcast phase: each inserts it, and those should_respond_to_broadcast picks answer with
    KnownPeers (:284-304), exported to it.  It does not appear in the mesh's own broadcast lists."""
    with Sim(parity.oracle_lib(), CFG) as s:
        s.set_external(46)
        s.step(1)
        s.inject(46, 0, K_JOIN)
        with pytest.raises(KbError):
            s.inject(46, 0, K_JOIN)                   # one Join per external peer per round
        s.step(1)
        assert all(46 in s.peers(i) for i in range(40))
        kp = [e for e in s.exported() if e[5] == K_KP]
        assert kp and all(e[3] == 46 and e[0] == 1 and e[1] == 0 for e in kp)
        assert len(kp) == s.stats()["join_responses"] and 0 < len(kp) <= 40
        assert all(b[1] != 46 for b in s.broadcasts())


def test_external_is_not_fresh_and_needs_unbound_address():
    with Sim(parity.oracle_lib(), SimConfig(capacity=48, initial_nodes=40, init_mode=KB_INIT_CONVERGED, seed=5,
                                            churn=0.2, fault_end_round=3)) as s:
        with pytest.raises(KbError):
            s.set_external(3)                         # a running instance's address
        s.set_external(40)
        s.step(3)                                     # churn joins take fresh ids: 40 is skipped
        assert not s.is_running(40) and s.stats()["churn_joins"] > 0
        with pytest.raises(KbError):
            s.inject(41, 3, K_PING)                   # not an external peer
        for _ in range(33):
            s.inject(40, 3, K_PING)
        with pytest.raises(KbError):
            s.inject(40, 3, K_PING)                   # 33 records per external peer per round


def test_oracle_external_case_runs():
    case, rounds = {n: (c, r) for n, c, r in parity.standard_cases()}["converged_loss_256"]
    lib = parity.oracle_lib()
    cfg = SimConfig(capacity=260, initial_nodes=256, init_mode=KB_INIT_CONVERGED, loss=0.05, seed=7)
    ok, msg, nx = parity.run_external_case({"cfg": cfg}, 20, [257, 259], [lib, lib])
    assert ok and nx > 20, msg
