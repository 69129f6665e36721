set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06l
bash tools/ab_run.sh r06l/ab base a3k32 > gpurun_out/r06l/ab.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "exact or horizon" > gpurun_out/r06l/pytest.log 2>&1
