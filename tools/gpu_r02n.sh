#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02n}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread --durations=10 > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/pytest.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u tools/find_divergence.py 8192 sock 1200 100 rows 2>&1 | tee $OUT/div8k_sock.log
timeout -k 10 300 python3 -u tools/find_divergence.py 8192 sim 700 100 rows 2>&1 | tee $OUT/div8k_sim.log
