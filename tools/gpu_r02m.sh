#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02m}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 280 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/pytest.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sim lat > $OUT/quick_sim.log 2>&1 || { tail -20 $OUT/quick_sim.log; exit 1; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sock lat > $OUT/quick_sock.log 2>&1 || { tail -20 $OUT/quick_sock.log; exit 1; }
grep N= $OUT/quick_*.log
KB_DEV=64 KB_DEBUG_WAVES=1 timeout -k 10 120 python3 tools/quick_perf.py 65536 12 sim lat > $OUT/dbgwaves_sim.log 2>&1 || { tail -20 $OUT/dbgwaves_sim.log; exit 1; }
grep "round 12 wave [0-2]" $OUT/dbgwaves_sim.log
timeout -k 10 400 python3 -u tools/tail_probe.py 65536 sock 45000 5000 gpu 2>&1 | tee $OUT/tail_sock.log
