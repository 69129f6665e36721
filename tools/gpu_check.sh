#!/bin/bash
# usage: tools/gpu_check.sh <tag> — GPU parity tests, the default bench line, and a rocprofv3
# kernel-trace summary of a short bench run, all under gpurun_out/<tag>/.  Every GPU step has its
# own time limit and the steps are chained: the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -30 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu --no-conv > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $OUT/prof_bench.err; exit $rc; }
python3 tools/prof_summary.py stats $OUT/prof | tee $OUT/kernel_stats.txt | head -40
