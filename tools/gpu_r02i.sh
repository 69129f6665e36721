#!/bin/bash
# parity after the KPR probe, then quick perf (sim, sock) and a KB_DEBUG_WAVES breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 280 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sim lat > $OUT/quick_sim.log 2>&1 || { tail -20 $OUT/quick_sim.log; exit 1; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sock lat > $OUT/quick_sock.log 2>&1 || { tail -20 $OUT/quick_sock.log; exit 1; }
grep N= $OUT/quick_*.log
KB_DEBUG_WAVES=1 timeout -k 10 120 python3 tools/quick_perf.py 65536 12 sim lat > $OUT/dbgwaves_sim.log 2>&1 || { tail -20 $OUT/dbgwaves_sim.log; exit 1; }
grep "round 12 " $OUT/dbgwaves_sim.log
