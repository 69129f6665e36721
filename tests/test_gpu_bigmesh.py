"""configs[3]'s per-GPU footprint on one MI355X (BASELINE.json configs[3]: 1M peers on
8 GPUs = 131,072 rows of 1M-id rows per rank, ≈ 139 GB of stamps + 17 GB of member bits).

A single-GPU mesh of 372,736 peers (capacity 380,928: rows of W = 385,024 ids) holds the same stamp bytes per
GPU as one configs[3] rank (372,736 x 385,024 ≈ 143.5 GB vs 131,072 x 1,056,768 ≈ 138.5 GB), with the
latency table off as bench.py turns it off at that size.  Its rows take the wide-row kernel variants
naturally where a 1M-id row would (Join responses from HBM scratch above 131,072 ids).
The workload is configs[2]'s shape (converged start, 1 % loss, 0.01 %/round churn, sim_sender), 6 rounds (the first Failed broadcasts are honoured in round 5):
  - every round's digest (all fingerprints, per-node scalars, counters) of the unsharded mesh equals that of
    the same mesh as 8 in-process row shards exchanging every wave (LocalXfer) and of the unsharded mesh
    with every wide-row variant forced (KB_DBG_ALL);
  - sampled rows: generate_fingerprint of peers() (kb_fingerprint_of_set) equals the row's fingerprint
    (src/kaboodle.rs:71-83), and the rows are byte-identical across the three runs;
  - the counters' invariants (alive = initial - leaves + joins, next_free = initial + joins).
The runs cannot be resident together (≈ 160 GB each): each records its digests and is destroyed first.
Oracle parity at scale: 131,072 peers (the dense CPU oracle needs 19 GB of host RAM and ≈ 10 s per round on
the box's 16 cores there; the 372K oracle would need 145 GB and minutes per round), every fingerprint and
sampled rows, 6 rounds: the first honoured Failed list (round 5) on rows wider than the LDS paths is checked
against the oracle, not only GPU against GPU; the same at 131,072 peers in the exact A3 order checks the
exact kernel of 128K-512K-id rows (`k_a3_exact<8>`) against the oracle."""
import ctypes as C
import hashlib
import json

import numpy as np
import pytest

import parity
from kaboodle_amd._ffi import KB_DBG_ALL, KB_INIT_CONVERGED, Sim, SimConfig

pytestmark = pytest.mark.gpu

BIG = 372736
BIG_CFG = SimConfig(capacity=BIG + 8192, initial_nodes=BIG, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.0001, seed=3)
ROUNDS = 6
SAMPLE = sorted(int(x) for x in np.random.default_rng(11).choice(BIG, 6, replace=False))


def _digest(m) -> str:
    h = hashlib.sha256()
    h.update(m.fingerprints().tobytes())
    h.update(m.scalars().tobytes())
    h.update(json.dumps(m.stats(), sort_keys=True).encode())
    return h.hexdigest()


def _fp_of_set():
    f = C.CDLL(parity.GPU_SO).kb_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
    return f


def _run(shards=0, dbg=0):
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    from dataclasses import replace
    with Sim(parity.gpu_lib(), replace(BIG_CFG, debug_flags=dbg), shards=shards) as m:
        digests = []
        for _ in range(ROUNDS):
            m.step(1)
            digests.append(_digest(m))
        rows = {i: hashlib.sha256(m.row(i).tobytes()).hexdigest() for i in SAMPLE}
        fps = m.fingerprints()
        f = _fp_of_set()
        for i in SAMPLE:
            if m.is_running(i):
                p = np.ascontiguousarray(np.asarray(m.peers(i), dtype=np.uint32))
                assert f(p.ctypes.data_as(C.POINTER(C.c_uint32)), len(p), None, 0, None) == fps[i], f"node {i}"
        st = m.stats()
        paths = m.debug_paths()
    return digests, rows, st, paths


@pytest.fixture(scope="module")
def unsharded():
    return _run()


def test_big_mesh_unsharded(unsharded):
    digests, rows, st, paths = unsharded
    assert st["alive"] == BIG - st["churn_leaves"] + st["churn_joins"]
    assert st["next_free_id"] == BIG + st["churn_joins"]
    assert st["join_responses"] > 0 and st["removed_failed"] > 0 and st["churn_joins"] > 0
    assert paths & (2 | 4), "rows of 380K ids take the HBM-scratch Join responses"


def test_big_mesh_8_shards_equal(unsharded):
    """The same mesh as 8 row shards (kb_sim_create_local: every wave an all-to-all-v between shards, the
    broadcast lists all-gathered): identical digests every round and identical sampled rows."""
    digests, rows, st, _ = _run(shards=8)
    assert digests == unsharded[0]
    assert rows == unsharded[1] and st == unsharded[2]


def test_big_mesh_forced_variants_equal(unsharded):
    """Every wide-row variant forced (KB_DBG_ALL: broadcast phase and KnownPeers groups on the HBM bitset,
    Join responses by workgroup from HBM scratch, BIG KnownPeers groups, k_proc's unsorted path)."""
    digests, rows, st, paths = _run(dbg=KB_DBG_ALL)
    assert digests == unsharded[0]
    assert rows == unsharded[1] and st == unsharded[2]
    assert paths & 1 and paths & 8


def test_oracle_parity_131k():
    """The HIP mesh against the dense CPU oracle at 131,072 peers: counters, every fingerprint and per-node
    scalar, and sampled whole rows, suspect and curious tables, every round for 6 rounds (round 5 honours the
    first Failed broadcasts)."""
    import kaboodle_amd
    kaboodle_amd.require_gpu()
    n = 131072
    cfg = SimConfig(capacity=n + 8192, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.0001, seed=3)
    o = Sim(parity.oracle_lib(omp=True), cfg)
    g = Sim(parity.gpu_lib(), cfg)
    rng = np.random.default_rng(7)
    try:
        for r in range(6):
            o.step(1)
            g.step(1)
            d = parity.compare_sampled(o, g, rng, nrows=6)
            assert not d, f"round {r}: " + "; ".join(d[:4])
        st = g.stats()
        assert st["join_responses"] > 0 and st["removed_failed"] > 0
    finally:
        g.close()
        o.close()


def test_oracle_parity_131k_exact_order():
    """The exact A3 order (KB_VARIANT_EXACT_LRU, the bench's default) on rows of 139,264 ids: 136 blocks of 1024
    ids, so `k_a3_exact<8>` (the width between 128K and 512K ids) against the dense CPU oracle, which then holds
    the C x C instants too (≈ 78 GB of host RAM beside the 19 GB of stamps).  Counters, every fingerprint and
    per-node scalar, sampled rows, every round for 6 rounds."""
    import kaboodle_amd
    from kaboodle_amd._ffi import KB_VARIANT_EXACT_LRU
    kaboodle_amd.require_gpu()
    n = 131072
    cfg = SimConfig(capacity=n + 8192, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.0001, seed=5,
                    variant=KB_VARIANT_EXACT_LRU)
    o = Sim(parity.oracle_lib(omp=True), cfg)
    g = Sim(parity.gpu_lib(), cfg)
    rng = np.random.default_rng(11)
    try:
        for r in range(6):
            o.step(1)
            g.step(1)
            d = parity.compare_sampled(o, g, rng, nrows=6)
            assert not d, f"round {r}: " + "; ".join(d[:4])
        st = g.stats()
        assert st["join_responses"] > 0 and st["removed_failed"] > 0
    finally:
        g.close()
        o.close()
