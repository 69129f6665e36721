#!/bin/bash
# per-wave kernel traces of the aged 64K workload in both failed modes + SQ counters of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02b}
mkdir -p $OUT
export TMPDIR=/tmp
for mode in sim sock; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$mode" -o run --output-format csv -- \
    python3 tools/quick_perf.py 65536 20 $mode > $OUT/quick_$mode.log 2>&1 || { tail -20 $OUT/quick_$mode.log; exit 1; }
  f=$(find $OUT/prof_$mode -name "*kernel_trace.csv" | head -1)
  python3 tools/wave_prof.py "$f" > $OUT/waves_$mode.txt
  python3 tools/prof_summary.py stats $OUT/prof_$mode > $OUT/stats_$mode.txt
  grep N= $OUT/quick_$mode.log; head -25 $OUT/stats_$mode.txt; tail -14 $OUT/waves_$mode.txt
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/sq" -o run --output-format csv -- python3 tools/quick_perf.py 65536 6 sim > $OUT/sq.log 2>&1 || exit 1
python3 tools/prof_summary.py sq $OUT/sq > $OUT/sq.txt; head -30 $OUT/sq.txt
