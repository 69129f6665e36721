#!/bin/bash
# GPU parity (incl. latency EWMA), then quick perf in both failed modes (+ latency on) with per-wave traces
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02f}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${@:-tests/test_gpu_parity.py} -m gpu -x -v --timeout 280 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc



for mode in sim sock; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$mode" -o run --output-format csv -- \
    python3 tools/quick_perf.py 65536 20 $mode lat > $OUT/quick_$mode.log 2>&1 || { tail -20 $OUT/quick_$mode.log; exit 1; }
  f=$(find $OUT/prof_$mode -name "*kernel_trace.csv" | head -1)
  python3 tools/wave_prof.py "$f" > $OUT/waves_$mode.txt
  python3 tools/prof_summary.py stats $OUT/prof_$mode > $OUT/stats_$mode.txt
  grep N= $OUT/quick_$mode.log; head -22 $OUT/stats_$mode.txt; tail -12 $OUT/waves_$mode.txt
done
