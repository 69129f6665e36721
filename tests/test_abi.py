"""The C-ABI boundary (include/kaboodle_sim.h): both implementations export every declared symbol, the
HIP library loads without a GPU and fails loudly (KB_NO_DEVICE) instead of computing on the CPU, and the
host-side mirror (kaboodle_amd) refuses to run without the HIP path."""
import ctypes as C
import os
import re

import pytest

import kaboodle_amd
from kaboodle_amd._ffi import KB_ABI_VERSION, KB_NO_DEVICE, KbConfig, KbStats, SimConfig
from parity import GPU_SO, ORACLE_SO

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kaboodle_sim.h")


def declared():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(kb_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_surface():
    names = declared()
    for must in ("kb_sim_create", "kb_sim_destroy", "kb_sim_step", "kb_sim_fingerprint", "kb_sim_peers",
                 "kb_sim_peer_states", "kb_sim_start_node", "kb_sim_stop_node", "kb_sim_ping_addrs",
                 "kb_sim_set_identity", "kb_sim_stats", "kb_sim_is_running", "kb_format_addr"):
        assert must in names
    m = re.search(r"#define\s+KB_ABI_VERSION\s+(\d+)", open(HEADER).read())
    assert int(m.group(1)) == KB_ABI_VERSION


@pytest.mark.skipif(not os.path.exists(GPU_SO), reason="HIP library not built (run __graft_entry__.build())")
def test_hip_library_exports_every_symbol():
    lib = C.CDLL(GPU_SO)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing


def test_oracle_exports_every_symbol():
    lib = C.CDLL(ORACLE_SO)
    skip = {"kb_sim_kernel_time", "kb_sim_reset_kernel_time", "kb_sim_kernel_bytes",   # GPU timing surface
            "kb_sim_set_profiling", "kb_sim_kernel_breakdown", "kb_sim_host_syncs",
            "kb_sim_debug_paths", "kb_sim_debug_counters",                             # GPU kernel variants
            "kb_rccl_unique_id", "kb_ipc_unique_id", "kb_sim_create_rank", "kb_sim_create_local", "kb_sim_shard_info",  # sharding
            "kb_wire_encode", "kb_wire_decode", "kb_wire_addr_of_id", "kb_wire_id_of_addr"}     # wire codec (host)
    missing = [n for n in declared() if n not in skip and not hasattr(lib, "kbo_" + n[3:])]
    assert not missing


def test_struct_layouts_match_header():
    # kb_config: 18 scalar fields (seed is u64) + reserved[3]; kb_stats: 6 x 4-byte + 20 x u64 + reserved[7]
    assert C.sizeof(KbConfig) == 4 * 4 + 8 + 4 * 12 + 4 * 4
    assert C.sizeof(KbStats) == 6 * 4 + 20 * 8 + 7 * 8
    from kaboodle_amd._ffi import KbKernelTime
    assert C.sizeof(KbKernelTime) == 24 + 8 + 8 + 8 + 4 + 4 + 9 * 8


def test_config_default_matches_mirror():
    for path, fn in ((GPU_SO, "kb_config_default"), (ORACLE_SO, "kbo_config_default")):
        if not os.path.exists(path):
            continue
        c = KbConfig()
        getattr(C.CDLL(path), fn)(C.byref(c))
        d = SimConfig().to_c()
        for f, _ in KbConfig._fields_:
            if f not in ("reserved",):
                assert getattr(c, f) == getattr(d, f), f


@pytest.mark.skipif(not os.path.exists(GPU_SO), reason="HIP library not built")
def test_no_gpu_means_no_device_error():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    lib = C.CDLL(GPU_SO)
    lib.kb_last_error.restype = C.c_char_p
    c = SimConfig(capacity=8, initial_nodes=8).to_c()
    h = C.c_void_p()
    assert lib.kb_sim_create(C.byref(c), C.byref(h)) == KB_NO_DEVICE
    assert b"device" in lib.kb_last_error()
    with pytest.raises(Exception):
        kaboodle_amd.require_gpu()
    with pytest.raises(kaboodle_amd.KbError):
        kaboodle_amd.Mesh(capacity=8, initial_nodes=8)


def test_thresholds():
    c = SimConfig(loss=0.01, churn=0.001).to_c()
    assert c.loss_threshold == round(0.01 * 2**32) and c.churn_threshold == round(0.001 * 2**32)
    assert SimConfig(loss=1.0).to_c().loss_threshold == 2**32 - 1
