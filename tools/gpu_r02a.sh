#!/bin/bash
# usage: tools/gpu_r02a.sh <tag> [pytest targets...] — the GPU suite (with durations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02a}; shift
mkdir -p $OUT
export TMPDIR=/tmp
T=${@:-tests}
timeout -k 10 1100 python -u -m pytest $T -m gpu -x -v --timeout 280 --timeout-method thread --durations=40 \
  > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/pytest.log | tail -70
tail -3 $OUT/pytest.log
exit $rc
