set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06h
bash tools/sparse_ab.sh r06h/ab sp_kp sp_shift sp_shift4 > gpurun_out/r06h/ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_big.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h/pytest.log 2>&1
