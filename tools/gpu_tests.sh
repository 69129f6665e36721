#!/bin/bash
# usage: tools/gpu_tests.sh <tag> [pytest args...]   GPU tests (default: the whole -m gpu suite) -> gpurun_out/<tag>/pytest.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
[ $# -eq 0 ] && set -- tests
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "$@" > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/pytest.log | tail -5; tail -3 $OUT/pytest.log
exit $rc
