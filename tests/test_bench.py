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
