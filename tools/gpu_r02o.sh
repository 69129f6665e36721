#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02o}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread --durations=10 > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/pytest.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sim lat > $OUT/quick_sim.log 2>&1 || { tail -20 $OUT/quick_sim.log; exit 1; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sock lat > $OUT/quick_sock.log 2>&1 || { tail -20 $OUT/quick_sock.log; exit 1; }
grep N= $OUT/quick_*.log
