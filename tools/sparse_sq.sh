#!/bin/bash
# SQ counters of the sparse engine over configs[4]'s scenario at 1M peers with the Failed-list drops counted
# (k_sp_bfail_sf's VALU statement and k_sp_handle's instruction mix), plus the kernel times of the
# same command.  tools/sparse_sq.sh <tag> -> gpurun_out/<tag>/{sq.txt,stats.txt,run.json}
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-spsq}; mkdir -p $OUT
export TMPDIR=/tmp
CMD="tools/sparse_big.py --nodes 1048576 --rounds 8 --count-sf-failed-drops --check-rows 0"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_WAIT_ANY SQ_INSTS_VMEM_RD --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/sq" -o run --output-format csv -- \
  python3 $CMD --out $OUT/run_pmc.json > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
python3 tools/prof_summary.py sq $OUT/sq > $OUT/sq.txt
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/st" -o run --output-format csv -- \
  python3 $CMD --out $OUT/run.json > $OUT/st.log 2>&1 || { tail -5 $OUT/st.log; exit 1; }
python3 tools/prof_summary.py stats $OUT/st > $OUT/stats.txt
head -12 $OUT/sq.txt; head -12 $OUT/stats.txt
