"""Known-answer vectors (tests/golden/vectors.json) against the C oracle, the Python restatement and the
host helpers of the HIP library.  Pins: CRC-32 (crc32fast == zlib), Philox4x32-10 (Random123 KAT),
generate_fingerprint (src/kaboodle.rs:71-83) on canonical sets, the canonical address mapping."""
import ctypes as C
import json
import os

import pytest

import pyref
from parity import GPU_SO, oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
VEC = json.load(open(os.path.join(HERE, "golden", "vectors.json")))


def _set_args(fp):
    """ids plus identity tables indexed by id (identities[id*stride ..], lens[id]), as the ABI takes them"""
    ids = fp["ids"]
    n = len(ids)
    idents = {int(k): bytes.fromhex(v) for k, v in fp["identities"].items()}
    stride = max([len(v) for v in idents.values()] + [1])
    top = max(ids) + 1 if ids else 1
    buf = (C.c_uint8 * (stride * top))()
    lens = (C.c_uint8 * top)()
    for i, b in idents.items():
        for q, x in enumerate(b):
            buf[i * stride + q] = x
        lens[i] = len(b)
    return (C.c_uint32 * max(n, 1))(*ids), n, buf, stride, lens


def test_crc32_check_value():
    lib = oracle_lib().lib
    lib.kbo_crc32.restype = C.c_uint32
    data = bytes.fromhex(VEC["crc32_check"]["input"])
    assert lib.kbo_crc32(data, len(data)) == VEC["crc32_check"]["crc"] == 0xCBF43926


@pytest.mark.parametrize("kat", VEC["philox4x32_10"])
def test_philox_kat(kat):
    lib = oracle_lib().lib
    out = (C.c_uint32 * 4)()
    lib.kbo_philox(*[C.c_uint32(x) for x in kat["ctr"] + kat["key"]], out)
    assert list(out) == kat["out"]
    assert list(pyref.philox(*kat["ctr"], *kat["key"])) == kat["out"]


@pytest.mark.parametrize("fp", VEC["fingerprints"], ids=lambda f: f["name"])
def test_fingerprint_oracle(fp):
    lib = oracle_lib().lib
    f = lib.kbo_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_uint8)]
    assert f(*_set_args(fp)) == fp["fp"]


@pytest.mark.parametrize("fp", VEC["fingerprints"], ids=lambda f: f["name"])
def test_fingerprint_pyref(fp):
    idents = {int(k): bytes.fromhex(v) for k, v in fp["identities"].items()}
    full = {i: idents.get(i, b"") for i in fp["ids"]}
    assert pyref.fingerprint(fp["ids"], full) == fp["fp"]


def test_fixed_goldens():
    """The values SURVEY.md §8a quotes, hard-coded here so a regenerated fixture cannot drift."""
    by = {f["name"]: f["fp"] for f in VEC["fingerprints"]}
    assert by["four_0_3"] == 0x42561112
    assert by["one_0"] == 0xD392E310
    assert by["range_1024"] == 0x4B0568B0
    assert by["config1_2x2"] == 0x981285C8
    assert by["empty"] == 0


@pytest.mark.skipif(not os.path.exists(GPU_SO), reason="HIP library not built")
@pytest.mark.parametrize("fp", VEC["fingerprints"], ids=lambda f: f["name"])
def test_fingerprint_hip_host_helper(fp):
    lib = C.CDLL(GPU_SO)
    f = lib.kb_fingerprint_of_set
    f.restype = C.c_uint32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_uint8)]
    assert f(*_set_args(fp)) == fp["fp"]


@pytest.mark.parametrize("i,s", sorted(VEC["addrs"].items()))
def test_addrs(i, s):
    buf = C.create_string_buffer(32)
    assert oracle_lib().lib.kbo_format_addr(int(i), buf, 32) == 0
    assert buf.value.decode() == s == pyref.addr(int(i))
    if os.path.exists(GPU_SO):
        assert C.CDLL(GPU_SO).kb_format_addr(int(i), buf, 32) == 0
        assert buf.value.decode() == s
