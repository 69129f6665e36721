#!/bin/bash
# usage: tools/gpu_sq.sh <tag> [mode]  — two SQ counter passes (8 SQ counters each, separate runs) over a
# short 64K run of the benched workload: instruction mix / wave cycles, then LDS bank conflicts and waits.
# -> gpurun_out/<tag>/sq{1,2}.txt (per-kernel averages per dispatch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sq}; MODE=${2:-sim}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES"
k=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/sq$k" -o run --output-format csv -- \
    python3 tools/quick_perf.py 65536 6 $MODE > $OUT/sq$k.log 2>&1 || { tail -5 $OUT/sq$k.log; exit 1; }
  python3 tools/prof_summary.py sq $OUT/sq$k > $OUT/sq$k.txt; head -14 $OUT/sq$k.txt
  k=$((k+1))
done
