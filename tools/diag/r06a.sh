set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=0 > gpurun_out/r06a/pytest_gpu.log 2>&1
