"""include/kaboodle_sim.hpp (the thin C++ Kaboodle-like wrapper) compiles against the C ABI and links
to the HIP library; without a GPU, mesh creation fails loudly with KB_NO_DEVICE."""
import os
import shutil
import subprocess

import pytest

from parity import GPU_SO

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    if not os.path.exists(GPU_SO):
        pytest.skip("HIP library not built")
    exe = str(tmp_path / "wrapper_demo")
    lib = os.path.dirname(GPU_SO)
    subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "wrapper_demo.cpp"), "-L", lib, "-lkaboodle_sim",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    return exe


def test_wrapper_host_side(tmp_path):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible (covered by the gpu test)")
    except ImportError:
        pass
    out = subprocess.run([build(tmp_path)], capture_output=True, text=True, check=True).stdout
    assert "addr 10.100.100.101:10001" in out
    assert "fp 42561112" in out
    assert "error 3" in out


@pytest.mark.gpu
def test_wrapper_on_gpu(tmp_path):
    out = subprocess.run([build(tmp_path), "--gpu"], capture_output=True, text=True, check=True).stdout
    assert out.count("fp 981285c8") == 5 and "mesh ok" in out
    assert "events 0: disc 4 dep 0 changed 1 fp 981285c8" in out
    assert "external acks 1" in out                # kb_sim_set_external / kb_sim_inject / kb_sim_exported
