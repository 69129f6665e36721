#!/bin/bash
# usage: tools/gpu_round.sh <tag>   — gpu tests, default bench, kernel-trace profile and PMC passes of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run --output-format csv -- python3 bench.py --no-cpu --no-conv --steps 20 > gpurun_out/$TAG/prof_bench.json 2> gpurun_out/$TAG/prof_bench.err || exit $?
python3 tools/prof_summary.py stats gpurun_out/$TAG/prof 20 > gpurun_out/$TAG/kernel_stats.txt; head -30 gpurun_out/$TAG/kernel_stats.txt; tail -1 gpurun_out/$TAG/kernel_stats.txt
bash tools/gpu_pmc.sh $TAG/pmc --steps 10 --warmup 3
