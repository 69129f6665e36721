set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06z7
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z7/smoke.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=30 > gpurun_out/r06z7/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r06z7/pytest_gpu.log; exit $rc
