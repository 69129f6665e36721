set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06g
bash tools/ab_run.sh r06g/ab base a3v2 lean4 lean3 > gpurun_out/r06g/ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "every_round or exact_lru or wide_row or horizon or wave_graph or external" > gpurun_out/r06g/pytest.log 2>&1
