set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06e
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=0 > gpurun_out/r06e/pytest_gpu.log 2>&1
