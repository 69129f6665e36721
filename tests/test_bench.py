"""CPU checks of bench.py's workload set-up (no GPU): the configuration the driver's command builds is the
one the full-size GPU parity test runs, and capacity does not depend on the step count."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _cfg(argv):
    return bench.rank_config(bench.parse(argv), 0, 1, 0)


def test_driver_config_is_the_parity_config():
    from test_gpu_fullsize import BENCH_CFG
    cfg = _cfg(["--gpus", "1", "--steps", "20", "--warmup", "5"])
    for f in ("capacity", "initial_nodes", "init_mode", "loss", "churn", "fault_end_round", "seed", "failed_mode",
              "track_latency", "max_waves", "id_len", "variant"):
        assert getattr(cfg, f) == getattr(BENCH_CFG, f), f


def test_capacity_independent_of_steps():
    caps = {_cfg(["--steps", str(k), "--warmup", "5"]).capacity for k in (5, 20, 50)}
    assert caps == {65536 + bench.CHURN_RESERVE}


def test_records_match_by_binary_or_sources(tmp_path, monkeypatch):
    """bench.py attaches a PMC or convergence record made with this library: the same binary, or (hipcc's output
    is not byte-reproducible) the same build inputs; a change to any input changes the source identity."""
    import pytest
    import kaboodle_amd
    from kaboodle_amd import build as kb_build
    if not os.path.exists(kaboodle_amd.LIB_PATH):
        pytest.skip("library not built")
    src = kb_build.src_sha16()
    assert src == kb_build.src_sha16() and len(src) == 16
    assert bench.same_build({"lib_sha16": bench.lib_sha16()})
    assert bench.same_build({"lib_sha16": "0" * 16, "lib_src_sha16": src})
    assert not bench.same_build({"lib_sha16": "0" * 16, "lib_src_sha16": "0" * 16})
    assert not bench.same_build({"lib_sha16": "0" * 16})
    dep = tmp_path / "kb_extra.h"
    dep.write_text("// a build input\n")
    monkeypatch.setattr(kb_build, "deps", lambda: [kb_build.SRC, str(dep)])
    a = kb_build.src_sha16()
    dep.write_text("// a build input, changed\n")
    assert kb_build.src_sha16() != a
