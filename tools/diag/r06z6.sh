set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06z6
timeout -k 10 400 python -u -m pytest tests/test_gpu_bigmesh.py -m gpu -x -v --timeout 300 --timeout-method thread -k "131k" --durations=5 > gpurun_out/r06z6/pytest.log 2>&1; rc=$?; tail -12 gpurun_out/r06z6/pytest.log; exit $rc
