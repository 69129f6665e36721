#!/bin/bash
# usage: tools/gpu_quick.sh <tag> "<pytest -k expr>" [quick_perf args...]: a parity subset, then quick_perf
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; K="$2"; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 280 --timeout-method thread -k "$K" \
    > $OUT/pytest.log 2>&1
  rc=$?
  tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 120 python3 tools/quick_perf.py "$@" > $OUT/quick.log 2>&1 || { tail -20 $OUT/quick.log; exit 1; }
cat $OUT/quick.log
