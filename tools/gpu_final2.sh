#!/bin/bash
# usage: tools/gpu_final2.sh <tag>: GPU parity file, the default bench line, and the rocprofv3 kernel
# statistics of the bench command (PMC summaries reused from the last tools/gpu_final.sh run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-conv --no-modes > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 1; }
python3 tools/prof_summary.py stats $OUT/prof 50 > $OUT/kernel_stats.txt
head -8 $OUT/kernel_stats.txt; tail -2 $OUT/kernel_stats.txt
