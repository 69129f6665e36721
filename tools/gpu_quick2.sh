#!/bin/bash
# usage: tools/gpu_quick2.sh <tag> [pytest -k expr] — 30-round timing of the 64K workload in both modes + a parity subset
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
for m in sim sock; do
  timeout -k 10 200 python3 tools/quick_perf.py 65536 30 $m lat > $OUT/q_$m.log 2>&1 || { tail $OUT/q_$m.log; exit 1; }
  echo "$m: $(grep N= $OUT/q_$m.log)"
done
K=${2:-parity_every_round and not sharded}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "$K" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
