#!/bin/bash
# usage: tools/gpu_dev.sh <tag>  — gpu tests, sweep ablations, kernel trace of a short bench (dev loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-dev}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -15 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for ab in 0 1 2 3; do
  KB_ABLATE=$ab timeout -k 10 200 python tools/quick_perf.py 65536 10 > gpurun_out/$TAG/perf_ab$ab.log 2>&1 || exit 1
  echo "ablate=$ab: $(grep N= gpurun_out/$TAG/perf_ab$ab.log)"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/age" -o run --output-format csv -- python3 tools/age_perf.py 65536 300 50 > gpurun_out/$TAG/age.log 2>&1 || exit 1
cat gpurun_out/$TAG/age.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run --output-format csv -- python3 bench.py --no-cpu --no-conv --steps 20 > gpurun_out/$TAG/prof_bench.json 2> gpurun_out/$TAG/prof_bench.err || exit $?
cat gpurun_out/$TAG/prof_bench.json
python3 tools/prof_summary.py stats gpurun_out/$TAG/prof > gpurun_out/$TAG/stats.txt; head -24 gpurun_out/$TAG/stats.txt
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/sq" -o run --output-format csv -- python3 bench.py --no-cpu --no-conv --steps 5 --warmup 2 > gpurun_out/$TAG/sq.log 2>&1 || exit $?
python3 tools/prof_summary.py sq gpurun_out/$TAG/sq > gpurun_out/$TAG/sq.txt; cat gpurun_out/$TAG/sq.txt
