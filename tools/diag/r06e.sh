set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06e
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --seeds "" > gpurun_out/r06e/bench.json 2> gpurun_out/r06e/bench.err &&
timeout -k 10 930 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=0 > gpurun_out/r06e/pytest_gpu.log 2>&1
