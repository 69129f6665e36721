#!/bin/bash
# round-2 check: the whole GPU suite (with durations), then per-wave kernel traces of the 64K workload in
# both failed modes (sim_sender = honoured Failed, sock = socket_faithful)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread --durations=40 \
  > $OUT/pytest.log 2>&1
rc=$?
tail -60 $OUT/pytest.log
exit $rc
