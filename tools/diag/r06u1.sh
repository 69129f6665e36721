set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06u
bash tools/gpu_measure.sh r06u pmc > gpurun_out/r06u/measure.log 2>&1 &&
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06u/smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=30 > gpurun_out/r06u/pytest_gpu.log 2>&1
