"""AddressSanitizer + UndefinedBehaviorSanitizer on the host code (CPU only; SURVEY.md §5's planned sanitizer
build).  oracle/Makefile's `sanitize` target builds tests/cpp/sanitize_harness.cpp against the C oracle and
the HIP library's wire decoder (kaboodle_amd/csrc/kb_wire.h, host code fed by bridge.py from real sockets),
both with -fsanitize=address,undefined and no recovery: any heap overflow, use after free, leak, signed
overflow or null memcpy aborts the run.

- the oracle through the whole kbo_ ABI on eleven small scenarios (joins, loss, churn, partition and heal,
  stop / restart / set_identity, probes, event drains, latency, both failed modes, every variant: same-window
  broadcasts, exact LRU, sparse rows);
- kb_wire_decode on 200,000 random and mutated datagrams (seeded), valid encodings round-tripping;
- kb_wire_decode on datagrams hypothesis generates (structured: valid headers with random tails, and raw
  bytes), each decoded from an exactly sized heap buffer on every channel."""
import os
import shutil
import struct
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_build", "sanitize_harness")
ENV = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with the sanitizer runtimes")


@pytest.fixture(scope="module")
def harness():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    return HARNESS


def _run(harness, *args, stdin=None):
    p = subprocess.run([harness, *args], input=stdin, capture_output=True, env=ENV, timeout=300)
    assert p.returncode == 0, (p.stdout.decode(errors="replace") + p.stderr.decode(errors="replace"))[-4000:]
    assert b"runtime error" not in p.stderr and b"ERROR: AddressSanitizer" not in p.stderr
    return p.stdout.decode()


def test_oracle_scenarios_sanitized(harness):
    assert "11 run, 0 failures" in _run(harness, "scenarios")


def test_wire_decode_fuzz_sanitized(harness):
    assert "200000 datagrams, 0 failures" in _run(harness, "fuzz", "200000")


def _u32(v):
    return struct.pack("<I", v)


def _u64(v):
    return struct.pack("<Q", v)


_addr = st.builds(lambda t, ip, port: _u32(t) + bytes(ip) + struct.pack("<H", port),
                  st.sampled_from([0, 0, 1, 7]), st.lists(st.integers(0, 255), min_size=4, max_size=4),
                  st.integers(0, 65535))
_blob = st.builds(lambda n, b: _u64(n) + b, st.one_of(st.integers(0, 40), st.integers(0, 2**64 - 1)),
                  st.binary(max_size=40))
_entries = st.lists(st.tuples(_addr, _blob), max_size=6).map(lambda es: b"".join(a + b for a, b in es))
_unicast = st.builds(lambda idb, tag, body: idb + _u32(tag) + body, _blob, st.integers(0, 6),
                     st.one_of(_addr, st.binary(max_size=24),
                               st.builds(lambda n, e: _u64(n) + e, st.integers(0, 2**64 - 1), _entries)))
_bcast = st.builds(lambda tag, a, b: _u32(tag) + a + b, st.integers(0, 4), _addr, st.one_of(st.just(b""), _blob))
_datagram = st.one_of(_unicast, _bcast, _blob, st.binary(max_size=128))


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.lists(st.tuples(_datagram, st.integers(0, 8)), min_size=1, max_size=40))
def test_wire_decode_hypothesis_sanitized(harness, batch):
    """Structured datagrams (valid headers, wrong tags, huge lengths, truncations) through kb_wire_decode."""
    data = b""
    for dg, cut in batch:
        dg = dg[: max(0, len(dg) - cut)] if cut < 8 else dg
        data += _u32(len(dg)) + dg
    out = _run(harness, "decode", stdin=data)
    assert f"decode: {len(batch)} datagrams, 0 failures" in out
