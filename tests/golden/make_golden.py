"""Generates the committed golden fixtures (run from the repo root: python tests/golden/make_golden.py).

vectors.json — known-answer vectors that do not depend on any code in this repository:
  * CRC-32/ISO-HDLC check value (crc32fast 1.3.2 == zlib.crc32, Cargo.lock:111-112);
  * Philox4x32-10 known-answer vectors as published with Random123 (kat_vectors: zero, all-ones, pi);
  * fingerprints of canonical peer sets, computed literally as generate_fingerprint does
    (src/kaboodle.rs:71-83: CRC-32 over ascending SocketAddr order of addr.to_string() ‖ identity) with
    zlib, for the canonical address mapping of SURVEY.md §8a;
  * canonical address strings.
traces.json — per-round digests (stamp rows, fingerprints, suspect/curious tables, counters) of the
small scenarios in tests/scenarios.py, produced by tests/pyref.py: the independent dict-based Python
restatement of round semantics v1.  The C oracle and the HIP library are both checked against these.
"""
from __future__ import annotations

import json
import os
import random
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import pyref  # noqa: E402
import scenarios  # noqa: E402

# Random123 kat_vectors, philox4x32 10 rounds: (ctr[4], key[2]) -> out[4]
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def literal_fp(ids, idents):
    h = 0
    for p in sorted(ids):
        h = zlib.crc32(pyref.addr(p).encode(), h)
        h = zlib.crc32(idents.get(p, b""), h)
    return h


def vectors() -> dict:
    rng = random.Random(20261015)
    fps = []

    def add(name, ids, idents=None):
        idents = idents or {}
        fps.append({"name": name, "ids": sorted(ids), "identities": {str(k): v.hex() for k, v in idents.items()},
                    "fp": literal_fp(ids, idents)})

    add("empty", [])
    add("one_0", [0])
    add("four_0_3", [0, 1, 2, 3])
    add("range_1024", list(range(1024)))
    add("config1_2x2", [0, 1, 2, 3], {i: n for i, n in enumerate(scenarios.CONFIG1_IDS)})
    add("sparse_64k", rng.sample(range(65536), 300))
    add("crosses_50000", [49998, 49999, 50000, 50001, 99999, 100000])
    ids = rng.sample(range(5000), 200)
    add("ids_len5", ids, {i: pyref.default_identity(i, 5) for i in ids})
    ids = rng.sample(range(2000), 120)
    add("ids_ragged", ids, {i: bytes(rng.randrange(256) for _ in range(rng.randrange(0, 33))) for i in ids})
    return {
        "crc32_check": {"input": b"123456789".hex(), "crc": zlib.crc32(b"123456789")},
        "philox4x32_10": [{"ctr": c, "key": k, "out": o} for c, k, o in PHILOX_KAT],
        "fingerprints": fps,
        "addrs": {str(i): pyref.addr(i) for i in (0, 1, 49999, 50000, 65535, 1048575, 4194303)},
    }


def traces() -> dict:
    out = {}
    for sc in scenarios.SCENARIOS:
        pm = scenarios.pymesh_of(sc)
        scenarios.setup(pm, sc)
        rounds = []
        for r in range(sc["rounds"]):
            scenarios.apply_events(pm, sc, r)
            pm.step()
            rounds.append(scenarios.digest_pymesh(pm))
        out[sc["name"]] = {"first_converged": pm.first_converged, "rounds": rounds}
        print(f"{sc['name']}: {sc['rounds']} rounds, agree {pm.agree}", flush=True)
    return out


def main() -> None:
    assert all(list(pyref.philox(*c, *k)) == o for c, k, o in PHILOX_KAT), "pyref philox fails the Random123 KAT"
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(vectors(), f, indent=1)
    with open(os.path.join(HERE, "traces.json"), "w") as f:
        json.dump(traces(), f, separators=(",", ":"))


if __name__ == "__main__":
    main()
