set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06k
bash tools/ab_run.sh r06k/ab base a3kpl both > gpurun_out/r06k/ab.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "every_round or exact or horizon or wide_row or sharded" > gpurun_out/r06k/pytest.log 2>&1
