#!/bin/bash
# usage: tools/gpu_sq.sh <tag> [mode] — SQ counter pass (8 counters) over a short 64K run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sq}; MODE=${2:-sim}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/sq" -o run --output-format csv -- python3 tools/quick_perf.py 65536 6 $MODE > $OUT/sq.log 2>&1 || exit 1
python3 tools/prof_summary.py sq $OUT/sq > $OUT/sq.txt; head -16 $OUT/sq.txt
