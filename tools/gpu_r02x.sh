#!/bin/bash
# usage: tools/gpu_r02x.sh <tag> — per-wave kernel trace of the benched 64K workload (latency on), both failed modes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-waves}
mkdir -p $OUT
export TMPDIR=/tmp
for mode in sim sock; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/prof_$mode" -o run --output-format csv -- \
    python3 tools/quick_perf.py 65536 12 $mode lat > $OUT/quick_$mode.log 2>&1 || { tail -20 $OUT/quick_$mode.log; exit 1; }
  f=$(find $OUT/prof_$mode -name "*kernel_trace.csv" | head -1)
  python3 tools/wave_prof.py "$f" > $OUT/waves_$mode.txt; tail -24 $OUT/waves_$mode.txt
  cat $OUT/quick_$mode.log
done
KB_DEBUG_WAVES=1 timeout -k 10 200 python3 tools/quick_perf.py 65536 6 sim lat > $OUT/debug_waves.log 2>&1 || exit 1
grep "round 7" $OUT/debug_waves.log | head -30
