#!/bin/bash
# parity (wave kernels changed), quick perf, then the convergence tail run longer (both modes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02p}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 280 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/pytest.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sim lat > $OUT/quick_sim.log 2>&1 || { tail -20 $OUT/quick_sim.log; exit 1; }
timeout -k 10 120 python3 tools/quick_perf.py 65536 20 sock lat > $OUT/quick_sock.log 2>&1 || { tail -20 $OUT/quick_sock.log; exit 1; }
grep N= $OUT/quick_*.log
timeout -k 10 420 python3 -u tools/converge.py --mode sock --cap-factor 3 --every 4096 --budget-s 380 --out $OUT/converge_sock.json 2>&1 | tee $OUT/converge_sock.log | tail -12
timeout -k 10 500 python3 -u tools/converge.py --mode sim --cap-factor 4 --every 4096 --budget-s 460 --out $OUT/converge_sim.json 2>&1 | tee $OUT/converge_sim.log | tail -12
